#!/bin/bash
# PMC counters for the hot kernels (run on the GPU box).  Counters need their
# own run (no --sys-trace / runtime tracing together with --pmc).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc}
mkdir -p "$OUT"
timeout -k 10 120 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || true
# headline (ws-dense): split Gram GEMM (f16 MFMA) + the working-set round kernels
timeout -k 10 600 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d "$OUT/dense_mfma" -o pmc --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-accuracy || exit $?
python3 bench/pmc_summary.py "$OUT" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
