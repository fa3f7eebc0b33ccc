# branch-free pair step (box clipping, WSS2 choice): ws tests, per-step cost
# on a small coupled problem, covtype box (shrink auto) end to end
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ws_gpu.py tests/test_ws_kernels_gpu.py > gpurun_out/r4s_pytest.log 2>&1 &&
timeout -k 10 200 python3 -u bench/ws_stamps.py --data covtype --samples 7500 --features 54 --C 2048 --gamma 0.03125 --clip box --ws-blocks 1 --out gpurun_out/r4s_stamps_cov7500.json > /dev/null 2> gpurun_out/r4s_stamps_cov7500.err &&
timeout -k 10 300 python3 -u bench.py --no-accuracy --reference-check off --steps 1 --warmup 0 --config covtype --clip box --max-iter 60000000 --log-every 5000000 --json-out gpurun_out/r4s_covbox.json > /dev/null 2> gpurun_out/r4s_covbox.err
rc=$?
tail -2 gpurun_out/r4s_pytest.log
python3 -c "
import json
d=json.loads(open('gpurun_out/r4s_stamps_cov7500.json').read()); print('cov7500', d['rounds'], d['pair_steps'], d['fit_time_s'], d['b'], 'solve_us', d['solve_us'], 'per_step', d['solve_per_step_us'], 'period', d['round_period_us'])
d=json.loads(open('gpurun_out/r4s_covbox.json').read()); print('covbox', d['value'], d['rounds'], d['b'], d['converged'], d['shrink']['phase_log'])
"
exit $rc
