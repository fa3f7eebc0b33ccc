#!/bin/bash
# Full GPU check: test suite, headline bench (N=1), kernel stats profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/bench1.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/bench1.log | tail -1
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o bench --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-accuracy > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; find gpurun_out/prof_bench -name "*kernel_stats.csv" | head -1 | xargs head -6
exit $rc
