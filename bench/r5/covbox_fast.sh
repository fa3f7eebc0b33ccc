# (historical: the A/B switch / code this script exercised was removed after its measurement; see profiles/)
# covtype box end to end with the hardware exp in the recompute rounds
set -o pipefail
mkdir -p gpurun_out
C="python3 -u bench.py --no-accuracy --reference-check off --steps 1 --warmup 0 --config covtype --clip box --max-iter 60000000 --log-every 5000000"
DPSVM_RECOMPUTE_EXP=fast timeout -k 10 300 $C --json-out gpurun_out/r5e_covbox_fast.json > gpurun_out/r5e_covbox_fast.log 2>&1 || { tail -5 gpurun_out/r5e_covbox_fast.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r5e_covbox_fast.json')); print('fast', d['value'], d['rounds'], d['iterations'], d['b'], d['converged'], d['n_sv'], d['shrink']['phase_log'])"
