# dense gathers at world 1 load the upper triangle of the sub-Gram and mirror it (half the random-line loads):
# ws + solver tests, mnist-parity (32 x 96 gather) and the headline, covtype box (one-block gathers)
set -o pipefail
mkdir -p gpurun_out/r5gs
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_ws_kernels_gpu.py tests/test_ws_gpu.py tests/test_solver_gpu.py \
  > gpurun_out/r5gs/pytest.log 2>&1 || { tail -40 gpurun_out/r5gs/pytest.log; exit 1; }
tail -1 gpurun_out/r5gs/pytest.log
for rep in 1 2; do
  timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 3 > gpurun_out/r5gs/b_$rep.json 2> gpurun_out/r5gs/b_$rep.err || { tail -5 gpurun_out/r5gs/b_$rep.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r5gs/b_$rep.json').read().strip().splitlines()[-1]); rc=d['reference_check']; s=d.get('secondary') or {}; print('headline', d['value'], 'rounds', d['rounds'], 'gram', d['gram_gemm_s'], 'b', d['b'], rc['decision_sign_agreement'], '| parity', s.get('value'), s.get('rounds'), s.get('b'))"
done
C="python3 -u bench.py --no-accuracy --reference-check off --steps 1 --warmup 0 --config covtype --clip box --max-iter 60000000 --log-every 5000000"
timeout -k 10 300 $C --json-out gpurun_out/r5gs/covbox.json > gpurun_out/r5gs/covbox.log 2>&1 || { tail -5 gpurun_out/r5gs/covbox.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r5gs/covbox.json')); print('covbox', d['value'], d['rounds'], d['iterations'], d['b'], d['converged'], d['n_sv'], d['shrink']['phase_log'])"
