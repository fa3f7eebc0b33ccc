#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in 14 0; do
  DPSVM_STAMPS=/tmp/lst$spec timeout -k 10 300 python bench/lru_profile_run.py $spec 30000 > gpurun_out/lru_stamps_$spec.log 2>&1 || exit $?
  python bench/stamps_report.py /tmp/lst$spec.rank0 --lru > gpurun_out/lru_stamps_$spec.json 2>&1
  echo "spec=$spec"; cat gpurun_out/lru_stamps_$spec.json
done
