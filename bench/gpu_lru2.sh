#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_solver_gpu.py -q -x -k "fused_cache or cache_policies or matches_cpu or rccl" > gpurun_out/pytest_lru.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_lru.log
[ $rc -eq 0 ] || exit $rc
DPSVM_STAMPS=/tmp/lst14 timeout -k 10 300 python bench/lru_profile_run.py 14 30000 > gpurun_out/lru_stamps_14.log 2>&1 || exit $?
python bench/stamps_report.py /tmp/lst14.rank0 --lru > gpurun_out/lru_stamps_14.json 2>&1; cat gpurun_out/lru_stamps_14.json
timeout -k 10 600 python bench/lru_sweep.py --spec 4,8,14 --variants fused --out gpurun_out/lru_sweep.jsonl > gpurun_out/lru_sweep.log 2>&1
rc=$?; echo "lru_sweep rc=$rc"; tail -4 gpurun_out/lru_sweep.log
exit $rc
