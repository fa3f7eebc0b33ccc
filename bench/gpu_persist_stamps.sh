#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
DPSVM_STAMPS=/tmp/pst timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-accuracy > gpurun_out/pstamps_bench.log 2>&1 || exit $?
python bench/stamps_report.py /tmp/pst.rank0 --persist > gpurun_out/persist_stamps.json 2>&1; cat gpurun_out/persist_stamps.json
