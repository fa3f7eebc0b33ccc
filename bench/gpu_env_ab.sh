#!/bin/bash
# Generic env A/B on the headline bench: each argument is one variant, a
# space-separated list of VAR=value assignments ("-" = no override).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i + 1))
  [ "$v" = "-" ] && v=""
  env $v timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-accuracy ${BENCH_ARGS:-} > gpurun_out/envab_$i.log 2>&1 || { tail -5 gpurun_out/envab_$i.log; exit 1; }
  echo -n "[$v] "; grep '^{' gpurun_out/envab_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['iterations'], d['b'], d.get('gram_gemm_s'))"
done
