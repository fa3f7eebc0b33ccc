# late-round validation: full GPU suite, headline bench (with the mnist-parity secondary), mnist-makefile preset,
# covtype box end to end
set -o pipefail
mkdir -p gpurun_out/r5vl
timeout -k 10 1000 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r5vl/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r5vl/pytest.log; grep -E "FAILED|ERROR" gpurun_out/r5vl/pytest.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --json-out gpurun_out/r5vl/bench.json > gpurun_out/r5vl/bench.log 2>&1 || { tail -20 gpurun_out/r5vl/bench.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5vl/bench.json')); s=d.get('secondary') or {}; print('headline', d['value'], d['gram_gemm_s'], d['rounds'], d['converged'], d['reference_check']['decision_sign_agreement'], 'secondary', {k: s.get(k) for k in ('value','rounds','converged','n_sv')})"
timeout -k 10 300 python3 -u bench.py --config mnist-makefile --steps 5 --warmup 2 --json-out gpurun_out/r5vl/makefile.json > gpurun_out/r5vl/makefile.log 2>&1 || { tail -20 gpurun_out/r5vl/makefile.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5vl/makefile.json')); print('makefile', d['value'], d['rounds'], d['converged'], d['ws_blocks'], (d.get('reference_check') or {}).get('decision_sign_agreement'))"
C="python3 -u bench.py --no-accuracy --reference-check off --steps 1 --warmup 0 --config covtype --clip box --max-iter 60000000 --log-every 5000000"
timeout -k 10 300 $C --json-out gpurun_out/r5vl/covbox.json > gpurun_out/r5vl/covbox.log 2>&1 || { tail -5 gpurun_out/r5vl/covbox.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r5vl/covbox.json')); print('covbox', d['value'], d['rounds'], d['iterations'], d['b'], d['converged'], d['n_sv'], d['shrink']['phase_log'])"
