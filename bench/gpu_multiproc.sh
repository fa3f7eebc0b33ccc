#!/bin/bash
# Rehearse N > 1 on a one-GPU box: 2 processes share device 0 (gloo bootstrap;
# RCCL refuses two ranks on one GPU).  Runs the communicator all-reduce path
# and the in-kernel peer exchange (IPC-mapped receive buffers).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp DPSVM_FORCE_DEVICE=0 DPSVM_VERIFY=1 DPSVM_XCH_TIMEOUT_S=30
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --samples 20000 --steps 1 --warmup 0 --comm gloo --exchange allreduce > gpurun_out/mp_gloo.log 2>&1
rc=$?; echo "gloo allreduce rc=$rc"; grep '^{' gpurun_out/mp_gloo.log | tail -1
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 \
  bench.py --gpus 2 --samples 20000 --steps 2 --warmup 1 --comm gloo --exchange peer > gpurun_out/mp_peer.log 2>&1
rc=$?; echo "gloo peer rc=$rc"; grep '^{' gpurun_out/mp_peer.log | tail -1; grep -i "error\|fail" gpurun_out/mp_peer.log | head -5
exit $rc
