#!/bin/bash
# PMC passes over one GEMM, one counter group per run (rocprofv3 does not split
# counters over passes):
#   bench/pmc_gemm.sh TAG gram   the headline split Gram GEMM (bench/gram_ab.py; DPSVM_SPLIT_GEMM picks the variant)
#   bench/pmc_gemm.sh TAG rows   the ws-cache miss-row GEMM at the synthetic-2m shape (bench/rows_probe.py)
# then: python3 bench/pmc_summary.py gpurun_out/pmc_TAG_*
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-gemm}
WHAT=${2:-gram}
if [ "$WHAT" = rows ]; then CMD="python3 bench/rows_probe.py --reps 1"; else CMD="python3 bench/gram_ab.py --only split --reps 1"; fi
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "gpurun_out/pmc_${TAG}_$name" -o run -- \
    $CMD > "gpurun_out/pmc_${TAG}_$name.log" 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  return $rc
}
pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT &&
pass sq2 SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_WAVES &&
pass tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT
