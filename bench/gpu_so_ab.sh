#!/bin/bash
# A/B of in-tree builds on one command: each argument is a DPSVM_NATIVE_SO path
# ("-" = the default module); runs CMD (default: the covtype cache stats).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CMD=${CMD:-"python bench/cache_stats.py --config covtype --max-iter 200000 --spec 8"}
for so in "$@"; do
  if [ "$so" = "-" ]; then unset DPSVM_NATIVE_SO; else export DPSVM_NATIVE_SO=$so; fi
  echo -n "[$so] "
  timeout -k 10 300 $CMD > gpurun_out/soab.log 2>&1 || { tail -3 gpurun_out/soab.log; exit 1; }
  grep '^{' gpurun_out/soab.log | tail -1
done
