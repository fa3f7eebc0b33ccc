#!/bin/bash
# PMC counters for the hot kernels on the headline config (run on the GPU box).
# Counters need their own run (no --sys-trace / runtime tracing with --pmc).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc}
mkdir -p "$OUT"
# dense headline: fused SMO kernel + Gram GEMM
timeout -k 10 900 rocprofv3 --kernel-trace --stats --pmc FETCH_SIZE SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_F32 \
  -d "$OUT/dense" -o pmc --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-accuracy || exit $?
# LRU mode: row kernel (X pass, MFMA 16x16x4) + finalize
timeout -k 10 900 rocprofv3 --kernel-trace --stats --pmc FETCH_SIZE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_F32 \
  -d "$OUT/lru" -o pmc --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-accuracy \
  --cache-lines 20000 || exit $?
