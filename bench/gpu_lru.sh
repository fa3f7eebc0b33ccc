#!/bin/bash
# fused cache-mode iteration: GPU tests of the solver + per-iteration latency A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_solver_gpu.py -q -x -k "fused_cache or cache_policies or matches_cpu or rccl" > gpurun_out/pytest_lru.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_lru.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench/lru_sweep.py --out gpurun_out/lru_sweep.jsonl > gpurun_out/lru_sweep.log 2>&1
rc=$?; echo "lru_sweep rc=$rc"; tail -20 gpurun_out/lru_sweep.log
exit $rc
