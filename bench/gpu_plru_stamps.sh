#!/bin/bash
# Persistent cache engine phases on the covtype-shape preset (spec 8, capped).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
DPSVM_STAMPS=/tmp/pls timeout -k 10 300 python bench/lru_profile_run.py ${SPEC:-8} ${ITERS:-200000} covtype 581012 0 > gpurun_out/plru_stamps.log 2>&1 || exit $?
tail -2 gpurun_out/plru_stamps.log
python bench/stamps_report.py /tmp/pls.rank0 --plru | tee gpurun_out/plru_stamps.json
