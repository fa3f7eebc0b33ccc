#!/bin/bash
# Split-GEMM diagnostics on the headline Gram (bench/gram_ab.py): k blocks per
# stage (DPSVM_SPLIT_KB), store ablations (DPSVM_SPLIT_ABLATE), PMC passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # label env...
  local label=$1; shift
  env "$@" timeout -k 10 200 python -u bench/gram_ab.py --only split --reps 3 > gpurun_out/gram_$label.log 2>&1 || exit 1
  echo "$label $(tail -1 gpurun_out/gram_$label.log)"
}
run kb2 DPSVM_SPLIT_KB=2
run kb1 DPSVM_SPLIT_KB=1
run kb2_nostore DPSVM_SPLIT_KB=2 DPSVM_SPLIT_ABLATE=1
run kb2_nomirror DPSVM_SPLIT_KB=2 DPSVM_SPLIT_ABLATE=2
timeout -k 10 200 python -u bench/gram_ab.py --only f32 --reps 3 > gpurun_out/gram_f32.log 2>&1 || exit 1
echo "f32 $(tail -1 gpurun_out/gram_f32.log)"
DPSVM_SPLIT_KB=${PMC_KB:-2} timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmc_split1 -o run -- python3 bench/gram_ab.py --only split --reps 1 > gpurun_out/pmc_split1.log 2>&1
echo "pmc1 rc=$?"
DPSVM_SPLIT_KB=${PMC_KB:-2} timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/pmc_split2 -o run -- python3 bench/gram_ab.py --only split --reps 1 > gpurun_out/pmc_split2.log 2>&1
echo "pmc2 rc=$?"
