# wide-wave Gram as the default: ws / split suites, headline bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_split_gemm_gpu.py tests/test_ws_gpu.py tests/test_kernels_gpu.py > gpurun_out/r4x_pytest.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/r4x_headline.json > /dev/null 2> gpurun_out/r4x_headline.err
rc=$?
tail -3 gpurun_out/r4x_pytest.log
python3 -c "
import json
d=json.loads(open('gpurun_out/r4x_headline.json').read())
print('headline', d['value'], 'gram', d['gram_gemm_s'], 'loop', d['smo_loop_s_min'], d['smo_loop_s_max'], 'rounds', d['rounds'], 'b', d['b'], 'ref', d['reference_check']['abs_b_diff'], d['reference_check']['decision_sign_agreement'])
"
exit $rc
timeout -k 10 200 python3 -u bench/ws_stamps.py --data covtype --samples 7500 --features 54 --C 2048 --gamma 0.03125 --clip box --ws-blocks 1 --out gpurun_out/r4x_stamps_cov7500.json > /dev/null 2> gpurun_out/r4x_stamps_cov7500.err
cat gpurun_out/r4x_stamps_cov7500.json
