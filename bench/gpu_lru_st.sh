#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
DPSVM_STAMPS=/tmp/lst14 timeout -k 10 300 python bench/lru_profile_run.py 14 30000 > gpurun_out/lru_stamps_14.log 2>&1 || exit $?
python bench/stamps_report.py /tmp/lst14.rank0 --lru > gpurun_out/lru_stamps_14.json 2>&1; cat gpurun_out/lru_stamps_14.json
