#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lruprof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lruprof/s14 -o run --output-format csv -- python3 bench/lru_profile_run.py 14 30000 > gpurun_out/lruprof/s14.log 2>&1
rc=$?; echo "s14 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python bench/lru_trace_report.py gpurun_out/lruprof/s14/run_kernel_trace.csv
