#!/bin/bash
# Rehearse N > 1 on a one-GPU box: 2 processes share device 0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp DPSVM_FORCE_DEVICE=0 DPSVM_VERIFY=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --samples 20000 --steps 1 --warmup 0 --comm gloo > gpurun_out/mp_gloo.log 2>&1
echo "gloo rc=$?"; grep '^{' gpurun_out/mp_gloo.log | tail -1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 \
  bench.py --gpus 2 --samples 20000 --steps 1 --warmup 0 --comm rccl > gpurun_out/mp_rccl.log 2>&1
echo "rccl rc=$?"; grep '^{' gpurun_out/mp_rccl.log | tail -1; grep -i "error\|duplicate" gpurun_out/mp_rccl.log | head -5
exit 0
