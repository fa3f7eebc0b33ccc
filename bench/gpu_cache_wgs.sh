#!/bin/bash
# Cache-mode grid size A/B on a bench preset (capped iterations): workgroups
# targeted by the fused cache kernel's geometry (DPSVM_CACHE_WGS).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in ${WGS:-256 512 1024}; do
  echo -n "wgs=$w "
  DPSVM_CACHE_WGS=$w timeout -k 10 300 python bench/cache_stats.py --config ${CFG:-covtype} \
    --max-iter ${ITERS:-200000} --spec ${SPEC:-8} > gpurun_out/wgs_$w.log 2>&1 || { tail -3 gpurun_out/wgs_$w.log; exit 1; }
  grep '^{' gpurun_out/wgs_$w.log | tail -1
done
