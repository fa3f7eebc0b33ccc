# working-set parameters of the one-block rounds on the big configs (defaults:
# ws_size 192, ws_new 3/4 of it): covtype box (shrink auto) by size,
# synthetic-2m by rows replaced per round (its B panel streams once per round
# whatever the miss count, so progress per round is what counts)
set -o pipefail
mkdir -p gpurun_out
C="python3 -u bench.py --no-accuracy --reference-check off --steps 1 --warmup 0 --config covtype --clip box --max-iter 60000000"
S="python3 -u bench.py --no-accuracy --reference-check off --steps 1 --warmup 0 --config synthetic-2m"
for q in 96 128; do
  timeout -k 10 300 $C --ws-size $q --log-every 5000000 --json-out gpurun_out/r4q_cov_q$q.json > /dev/null 2> gpurun_out/r4q_cov_q$q.err || exit $?
done
for w in 192 96; do
  timeout -k 10 400 $S --ws-new $w --log-every 1000000 --json-out gpurun_out/r4q_syn_new$w.json > /dev/null 2> gpurun_out/r4q_syn_new$w.err || exit $?
done
for f in cov_q96 cov_q128 syn_new192 syn_new96; do python3 -c "
import json
d=json.loads(open('gpurun_out/r4q_$f.json').read())
print('$f', d['value'], 'rounds', d['rounds'], 'conv', d['converged'], 'b', d['b'], d['shrink']['phase_log'])
"; done
