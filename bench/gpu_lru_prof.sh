#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lruprof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lruprof/s14 -o run --output-format csv -- python3 bench/lru_profile_run.py 14 20000 > gpurun_out/lruprof/s14.log 2>&1
rc=$?; echo "s14 rc=$rc"; tail -3 gpurun_out/lruprof/s14.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lruprof/s0 -o run --output-format csv -- python3 bench/lru_profile_run.py 0 20000 > gpurun_out/lruprof/s0.log 2>&1
rc=$?; echo "s0 rc=$rc"; tail -3 gpurun_out/lruprof/s0.log
find gpurun_out/lruprof -name "*.csv" | xargs ls -la
exit $rc
