#!/bin/bash
# Persistent engine: rows per workgroup (grid size) sweep on the headline problem,
# plus phase stamps for each geometry.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in ${ROWS:-256 512 768 1024}; do
  DPSVM_FUSED_ROWS=$r timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-accuracy > gpurun_out/geom_$r.log 2>&1 || exit $?
  echo -n "rows=$r "; grep '^{' gpurun_out/geom_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['smo_loop_s_max'], d['iterations'], d['iteration'])"
  DPSVM_FUSED_ROWS=$r DPSVM_STAMPS=/tmp/pst$r timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-accuracy > gpurun_out/geom_st_$r.log 2>&1 || exit $?
  python bench/stamps_report.py /tmp/pst$r.rank0 --persist > gpurun_out/geom_stamps_$r.json 2>&1; cat gpurun_out/geom_stamps_$r.json
done
