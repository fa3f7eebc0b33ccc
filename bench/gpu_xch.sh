#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_solver_gpu.py -q -x -k "peer_exchange or simulated_ranks or rccl" > gpurun_out/pytest_xch.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_xch.log
[ $rc -eq 0 ] || exit $rc
bash bench/gpu_multiproc.sh
