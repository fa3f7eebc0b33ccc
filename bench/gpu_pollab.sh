#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_solver_gpu.py -q -x -k "persistent or two_processes" > gpurun_out/pab.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pab.log | tail -1
[ $rc -eq 0 ] || exit $rc
for poll in 0; do
  DPSVM_XCH_POLL=$poll DPSVM_STAMPS=/tmp/pst$poll timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-accuracy > gpurun_out/pab_bench$poll.log 2>&1 || exit $?
  echo "poll=$poll"; grep '^{' gpurun_out/pab_bench$poll.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['smo_loop_s_max'])"
  python bench/stamps_report.py /tmp/pst$poll.rank0 --persist | tr -d '\n '; echo
done
