#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp DPSVM_XCH_TIMEOUT_S=20
timeout -k 10 300 python -m pytest tests/test_solver_gpu.py -q -x -k "persistent or peer_exchange" > gpurun_out/pytest_persist.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_persist.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench/iter_latency.py --out gpurun_out/iter_latency.jsonl > gpurun_out/iter_latency.log 2>&1
rc=$?; echo "iter_latency rc=$rc"; grep smo_loop gpurun_out/iter_latency.log
exit $rc
