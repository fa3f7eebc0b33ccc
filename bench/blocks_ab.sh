#!/bin/bash
# A/B of ws_blocks on the headline: bench/blocks_ab.sh "1 4 8" [bench.py args]
# -> gpurun_out/blk$P.log per value, one summary line each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PS=$1; shift
for P in $PS; do
  timeout -k 10 200 python -u bench.py --ws-blocks "$P" "$@" > "gpurun_out/blk$P.log" 2>&1 || { rc=$?; echo "P=$P failed rc=$rc"; tail -20 "gpurun_out/blk$P.log"; exit $rc; }
  grep '^{' "gpurun_out/blk$P.log" | tail -1 | python3 -c "import json,sys
d=json.loads(sys.stdin.read()); r=d.get('reference_check') or {}
print('P=$P', d['value'], 'steps', d['iterations'], 'rounds', d['rounds'], 'conv', d['converged'], 'b', round(d['b'], 6), 'gap', d['final_gap'], 'nsv', d['n_sv'], 'acc', d['train_accuracy'], 'ref |db|', r.get('abs_b_diff'), 'agree', r.get('decision_sign_agreement'), d['engine_note'])"
done
