# w64 interior epilogue: split + ws suites, headline bench x2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_split_gemm_gpu.py tests/test_ws_gpu.py tests/test_solver_gpu.py > gpurun_out/r4e2_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4e2_pytest.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/r4e2_headline_$k.json > /dev/null 2> gpurun_out/r4e2_headline_$k.err || exit 1
  python3 -c "
import json
d=json.loads(open('gpurun_out/r4e2_headline_$k.json').read())
print('headline', d['value'], 'gram', d['gram_gemm_s'], 'loop', d['smo_loop_s_min'], 'rounds', d['rounds'], 'b', d['b'], 'ref', d['reference_check']['abs_b_diff'])
"
done
timeout -k 10 200 python3 -u bench/gram_ab.py --only split --reps 5 2>&1 | grep '^split'
