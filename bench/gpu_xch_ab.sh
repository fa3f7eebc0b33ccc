#!/bin/bash
# Exchange poll A/B on the headline problem: entry stride (u64 slots per
# publisher entry), poll batch (entries per lane per round; 0 = from the entry
# count, larger values add loads of entry 0) and s_sleep(1) count per round.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARIANTS:-4,0,1 4,4,1 4,0,1 4,4,1}; do
  IFS=, read -r st kb sl <<< "$v"
  DPSVM_XCH_STRIDE=$st DPSVM_XCH_KB=$kb DPSVM_XCH_SLEEP=$sl timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-accuracy > gpurun_out/xab.log 2>&1 || exit $?
  echo -n "stride=$st kb=$kb sleep=$sl "; grep '^{' gpurun_out/xab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['iterations'], d['b'])"
done
