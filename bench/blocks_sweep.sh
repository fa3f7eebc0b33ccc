#!/bin/bash
# Headline parameter sweep, one bench process per point; each argument is one
# point's extra bench.py flags:
#   bench/blocks_sweep.sh "--ws-blocks 8 --ws-rel 0.15" "--ws-size 160" "--ws-inner 96"
# -> gpurun_out/sweep.txt (value, pair steps, rounds, converged per point)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/sweep.txt
for PT in "$@"; do
  # shellcheck disable=SC2086
  timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --reference-check off --no-accuracy $PT \
      > gpurun_out/sweep_pt.log 2>&1 || { echo "[$PT] failed"; tail -5 gpurun_out/sweep_pt.log; exit 1; }
  grep '^{' gpurun_out/sweep_pt.log | tail -1 | python3 -c "import json,sys
d=json.loads(sys.stdin.read())
print('[$PT]', d['value'], 'steps', d['iterations'], 'rounds', d['rounds'], 'conv', d['converged'])" | tee -a gpurun_out/sweep.txt
done
