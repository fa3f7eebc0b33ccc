#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_solver_gpu.py -q -x -k "fused_cache or cache_policies or matches_cpu or verify" > gpurun_out/pytest_lru.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_lru.log
[ $rc -eq 0 ] || exit $rc
bash bench/gpu_cov_stamps.sh
timeout -k 10 600 python bench/lru_sweep.py --spec 14 --variants fused,chain > gpurun_out/lru_sweep.log 2>&1
rc=$?; echo "lru_sweep rc=$rc"; grep '^{' gpurun_out/lru_sweep.log
exit $rc
