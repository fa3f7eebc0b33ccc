#!/bin/bash
# A/B of the dense engines on the headline problem (no diagnostics)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for p in on off on; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-accuracy --persist $p > gpurun_out/ab_$p.log 2>&1 || exit $?
  echo -n "persist=$p "; grep '^{' gpurun_out/ab_$p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['smo_loop_s_max'], d['iteration'])"
done
