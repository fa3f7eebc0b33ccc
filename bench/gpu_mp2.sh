#!/bin/bash
# Two ranks as two processes sharing the one GPU (rehearsal of the multi-GPU
# path): bench.py over the in-kernel peer exchange, receive buffers in uncached
# vs coarse-grained memory.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp DPSVM_FORCE_DEVICE=0 DPSVM_XCH_TIMEOUT_S=30
for mem in ${MEMS:-uncached coarse}; do
  DPSVM_XCH_MEM=$mem timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29650 bench.py --gpus 2 --samples ${N:-20000} --steps 3 --warmup 1 \
    --comm gloo ${EXTRA:-} > gpurun_out/mp2_$mem.log 2>&1 || { tail -5 gpurun_out/mp2_$mem.log; exit 1; }
  echo -n "$mem: "; grep '^{' gpurun_out/mp2_$mem.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['iterations'], d['exchange'], d['exchange_mem'], d['iteration'], round(1e6*d['smo_loop_s_max']/d['iterations'],2), 'us/iter')"
done
