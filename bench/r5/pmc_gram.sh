# PMC re-take of the headline split Gram (w64 kernel, compact tiles, un-spilled epilogue): one counter group
# per run (rocprofv3 does not split counters over passes), each under its own kill timeout; stop at the first failure
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r5pmc
export TMPDIR=/tmp
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 60 rocprofv3 --pmc "$@" --output-format csv -d "gpurun_out/r5pmc/$name" -o run -- \
    python3 bench/gram_ab.py --only split --reps 1 > "gpurun_out/r5pmc/$name.log" 2>&1
}
pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT || { echo "pass sq failed"; exit 1; }
pass sq2 SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_F16 || { echo "pass sq2 failed"; exit 1; }
pass tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT || { echo "pass tcc failed"; exit 1; }
python3 bench/pmc_summary.py gpurun_out/r5pmc | grep -E "==|w64" | cut -c1-600
