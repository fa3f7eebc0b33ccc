# covtype box (shrink auto): rows replaced per one-block round below the 3/4 default
set -o pipefail
mkdir -p gpurun_out
C="python3 -u bench.py --no-accuracy --reference-check off --steps 1 --warmup 0 --config covtype --clip box --max-iter 60000000 --log-every 5000000"
for w in 96 120; do
  timeout -k 10 300 $C --ws-new $w --json-out gpurun_out/r4c_cov_new$w.json > /dev/null 2> gpurun_out/r4c_cov_new$w.err || exit $?
done
for w in 96 120; do python3 -c "
import json
d=json.loads(open('gpurun_out/r4c_cov_new$w.json').read())
print('new$w', d['value'], 'rounds', d['rounds'], 'conv', d['converged'], 'b', d['b'], d['shrink']['phase_log'])
"; done
