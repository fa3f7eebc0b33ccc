#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp DPSVM_XCH_TIMEOUT_S=20
timeout -k 10 600 python -m pytest tests/test_solver_gpu.py -q -x -k "persistent or peer_exchange or simulated or checkpoint or fault or box" > gpurun_out/xdbg.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "assert [0-9]+ ==|passed|failed" gpurun_out/xdbg.log | head -5
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python -m pytest tests/test_solver_gpu.py -q -x -k "two_processes" > gpurun_out/xdbg_mp$i.log 2>&1
  echo "mp run $i rc=$?"; grep -E "passed|failed" gpurun_out/xdbg_mp$i.log | tail -1
done
DPSVM_STAMPS=/tmp/pst timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-accuracy > gpurun_out/pstamps_bench.log 2>&1 || exit $?
python bench/stamps_report.py /tmp/pst.rank0 --persist > gpurun_out/persist_stamps.json 2>&1; cat gpurun_out/persist_stamps.json
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/bench1.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/bench1.log | tail -1
exit $rc
