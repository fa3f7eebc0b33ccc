# covtype box end to end (shrinking phases; phase 0 on ws-cache), recompute rounds vs the row cache
set -o pipefail
mkdir -p gpurun_out
C="python3 -u bench.py --no-accuracy --reference-check off --steps 1 --warmup 0 --config covtype --clip box --max-iter 60000000 --log-every 5000000"
timeout -k 10 300 $C --json-out gpurun_out/r5r_covbox_recompute.json > gpurun_out/r5r_covbox_recompute.log 2>&1 || { tail -5 gpurun_out/r5r_covbox_recompute.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r5r_covbox_recompute.json')); print('recompute', d['value'], d['rounds'], d['iterations'], d['b'], d['converged'], d['shrink']['phase_log'])"
DPSVM_WS_RECOMPUTE=2 timeout -k 10 300 $C --json-out gpurun_out/r5r_covbox_cache.json > gpurun_out/r5r_covbox_cache.log 2>&1 || { tail -5 gpurun_out/r5r_covbox_cache.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r5r_covbox_cache.json')); print('cache', d['value'], d['rounds'], d['iterations'], d['b'], d['converged'], d['shrink']['phase_log'])"
