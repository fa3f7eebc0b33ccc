#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp DPSVM_XCH_TIMEOUT_S=20
for poll in 0 1; do
  DPSVM_XCH_POLL=$poll timeout -k 10 300 python -m pytest tests/test_solver_gpu.py -q -x -k "two_processes and persistent" > gpurun_out/xdbg_$poll.log 2>&1
  echo "poll=$poll rc=$?"; grep -E "assert [0-9]+ ==|passed|failed" gpurun_out/xdbg_$poll.log | head -3
done
exit 0
