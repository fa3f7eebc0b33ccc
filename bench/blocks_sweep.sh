#!/bin/bash
# ws_blocks x ws_rel x ws_new sweep on the headline (one bench process per point):
#   bench/blocks_sweep.sh "8" "0.2 0.3 0.5" "120 144 168"  -> gpurun_out/sweep.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/sweep.txt
for P in $1; do for R in $2; do for NW in $3; do
  timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --reference-check off --no-accuracy \
      --ws-blocks "$P" --ws-rel "$R" --ws-new "$NW" > gpurun_out/sweep_pt.log 2>&1 || { echo "P=$P rel=$R new=$NW failed"; tail -5 gpurun_out/sweep_pt.log; exit 1; }
  grep '^{' gpurun_out/sweep_pt.log | tail -1 | python3 -c "import json,sys
d=json.loads(sys.stdin.read())
print('P=$P rel=$R new=$NW', d['value'], 'steps', d['iterations'], 'rounds', d['rounds'], 'conv', d['converged'])" | tee -a gpurun_out/sweep.txt
done; done; done
