# defaults check after the round-4 shrink / ROWS work: headline, mnist-parity,
# covtype-ref (Makefile:77, 500k rows, 3M cap) with shrink auto vs off
set -o pipefail
mkdir -p gpurun_out
B="python3 -u bench.py"
timeout -k 10 300 $B --steps 5 --warmup 1 --json-out gpurun_out/r4k_headline.json > /dev/null 2> gpurun_out/r4k_headline.err &&
timeout -k 10 300 $B --config mnist-parity --steps 3 --warmup 1 --json-out gpurun_out/r4k_parity.json > /dev/null 2> gpurun_out/r4k_parity.err &&
timeout -k 10 200 $B --config covtype-ref --steps 1 --warmup 0 --no-accuracy --reference-check off --json-out gpurun_out/r4k_covref_auto.json > /dev/null 2> gpurun_out/r4k_covref_auto.err &&
timeout -k 10 200 $B --config covtype-ref --shrink off --steps 1 --warmup 0 --no-accuracy --reference-check off --json-out gpurun_out/r4k_covref_off.json > /dev/null 2> gpurun_out/r4k_covref_off.err
rc=$?
for f in headline parity covref_auto covref_off; do python3 -c "
import json
d=json.loads(open('gpurun_out/r4k_$f.json').read())
print('$f', d['value'], 'rounds', d['rounds'], 'iters', d['iterations'], 'conv', d['converged'], 'b', d['b'], 'acc', d['train_accuracy'], 'ref', d.get('reference_check'), d['shrink'])
" 2>/dev/null; done
exit $rc
