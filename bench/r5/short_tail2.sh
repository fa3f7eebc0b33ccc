# short tail with hysteresis: headline / makefile benches, covtype box (long one-block phases: the single-round
# launches must not linger), solver + ws tests
set -o pipefail
mkdir -p gpurun_out/r5st3
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_ws_gpu.py tests/test_solver_gpu.py \
  > gpurun_out/r5st3/pytest.log 2>&1 || { tail -40 gpurun_out/r5st3/pytest.log; exit 1; }
tail -1 gpurun_out/r5st3/pytest.log
for rep in 1 2; do
  timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 3 > gpurun_out/r5st3/b_$rep.json 2> gpurun_out/r5st3/b_$rep.err || { tail -5 gpurun_out/r5st3/b_$rep.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r5st3/b_$rep.json').read().strip().splitlines()[-1]); rc=d['reference_check']; s=d.get('secondary') or {}; print('headline', d['value'], 'rounds', d['rounds'], 'it', d['iterations'], 'gram', d['gram_gemm_s'], 'b', d['b'], rc['decision_sign_agreement'], 'parity', s.get('value'), s.get('rounds'))"
done
timeout -k 10 240 python3 -u bench.py --config mnist-makefile --steps 5 --warmup 2 > gpurun_out/r5st3/m.json 2> gpurun_out/r5st3/m.err || { tail -5 gpurun_out/r5st3/m.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r5st3/m.json').read().strip().splitlines()[-1]); print('makefile', d['value'], 'rounds', d['rounds'], 'b', d['b'])"
C="python3 -u bench.py --no-accuracy --reference-check off --steps 1 --warmup 0 --config covtype --clip box --max-iter 60000000 --log-every 5000000"
timeout -k 10 300 $C --json-out gpurun_out/r5st3/covbox.json > gpurun_out/r5st3/covbox.log 2>&1 || { tail -5 gpurun_out/r5st3/covbox.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r5st3/covbox.json')); print('covbox', d['value'], d['rounds'], d['iterations'], d['b'], d['converged'], d['n_sv'], d['shrink']['phase_log'])"
