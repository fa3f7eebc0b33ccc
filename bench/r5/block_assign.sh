# merge block assignment: shifts for power-of-two P, rows per block from the layout (no LDS atomics)
# ws tests, bench, stamps
set -o pipefail
mkdir -p gpurun_out/r5ba
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ws_kernels_gpu.py tests/test_ws_gpu.py \
  > gpurun_out/r5ba/pytest.log 2>&1 || { tail -40 gpurun_out/r5ba/pytest.log; exit 1; }
tail -1 gpurun_out/r5ba/pytest.log
for rep in 1 2 3; do
  timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 3 --secondary off > gpurun_out/r5ba/b_$rep.json 2> gpurun_out/r5ba/b_$rep.err || { tail -5 gpurun_out/r5ba/b_$rep.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r5ba/b_$rep.json').read().strip().splitlines()[-1]); rc=d['reference_check']; print('bench', d['value'], 'rounds', d['rounds'], 'it', d['iterations'], 'gram', d['gram_gemm_s'], 'b', d['b'], 'conv', d['converged'], rc['decision_sign_agreement'])"
done
timeout -k 10 300 python3 -u bench/ws_stamps.py --out gpurun_out/r5ba/stamps.json > gpurun_out/r5ba/stamps.txt 2>&1 || { tail -5 gpurun_out/r5ba/stamps.txt; exit 1; }
tail -1 gpurun_out/r5ba/stamps.txt
