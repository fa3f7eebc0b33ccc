#!/bin/bash
# Eight ranks as eight processes sharing the one GPU: the headline problem over
# the in-kernel peer exchange at world 8 (rehearsal of the 8-GPU run; every
# rank's persistent grid must be co-resident, ~15 workgroups each).
# DPSVM_VERIFY=1 checks the cross-rank alpha digest after the run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp DPSVM_FORCE_DEVICE=0 DPSVM_XCH_TIMEOUT_S=30 DPSVM_VERIFY=1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29681 bench.py --gpus 8 --steps 2 --warmup 1 \
  --comm gloo ${EXTRA:-} > gpurun_out/mp8.log 2>&1 || { tail -20 gpurun_out/mp8.log; exit 1; }
grep '^{' gpurun_out/mp8.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['iterations'], d['n_sv'], d['b'], d['exchange'], d['exchange_mem'], d['iteration'], round(1e6*d['smo_loop_s_max']/d['iterations'],2), 'us/iter')"
grep -i "verify\|mismatch" gpurun_out/mp8.log | head -5
exit 0
