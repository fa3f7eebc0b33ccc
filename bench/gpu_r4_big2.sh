# refresh of the 8-GPU plan inputs with the round-4 ROWS kernels: synthetic-2m
# kernel profile (capped) and the full synthetic-2m / covtype box solves under
# the defaults (shrink=auto), 1 MI355X
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 -u $R/bench.py --no-accuracy --reference-check off --steps 1 --warmup 0"
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4c_prof_syn -o syn --output-format csv -- python3 -u $R/bench.py --no-accuracy --reference-check off --shrink off --steps 1 --warmup 0 --config synthetic-2m --max-iter 120000 --json-out $R/gpurun_out/r4c_syn_prof.json > $R/gpurun_out/r4c_prof_syn.log 2>&1) &&
timeout -k 10 300 $B --shrink off --config synthetic-2m --max-iter 120000 --json-out $R/gpurun_out/r4c_syn_local.json > /dev/null 2> $R/gpurun_out/r4c_syn_local.err &&
timeout -k 10 400 $B --config synthetic-2m --log-every 1000000 --verbose --json-out $R/gpurun_out/r4c_syn_auto.json > /dev/null 2> $R/gpurun_out/r4c_syn_auto.err &&
timeout -k 10 400 $B --config synthetic-2m --shrink off --log-every 1000000 --json-out $R/gpurun_out/r4c_syn_off.json > /dev/null 2> $R/gpurun_out/r4c_syn_off.err &&
timeout -k 10 300 $B --config covtype --clip box --max-iter 60000000 --shrink off --log-every 5000000 --json-out $R/gpurun_out/r4c_covbox_off.json > /dev/null 2> $R/gpurun_out/r4c_covbox_off.err
rc=$?
for f in syn_local syn_auto syn_off covbox_off; do python3 -c "
import json
d=json.loads(open('gpurun_out/r4c_$f.json').read())
print('$f', d['value'], 'rounds', d['rounds'], 'conv', d['converged'], 'b', d['b'], d['shrink'])
" 2>/dev/null; done
exit $rc
