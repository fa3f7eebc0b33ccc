#!/bin/bash
# PMC counters of the persistent dense engine on the headline problem (SQ block:
# instruction mix and wait cycles; TCC: L2 traffic).  Run through the SVC API
# (bench/pmc_diag.py), two single-block passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp DPSVM_XCH_TIMEOUT_S=10
OUT=${OUT:-gpurun_out/pmc_persist}
mkdir -p "$OUT"
# two counters per pass: with more SQ counters in one pass the in-kernel
# exchange self test fails under the profiler (ping=0) and the persistent engine
# is refused (profiles/r1_pmc_tlb.txt)
i=0
for pair in "SQ_WAVES SQ_BUSY_CYCLES" "SQ_WAIT_INST_ANY SQ_WAIT_ANY" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD" "SQ_INSTS_SALU SQ_INSTS_LDS" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $pair -d "$OUT/p$i" -o pmc --output-format csv -- \
    python3 bench/pmc_diag.py mnist > "$OUT/p$i.log" 2>&1 || exit $?
  echo -n "$pair: "; grep -E "^OK|^ERR" "$OUT/p$i.log"
done
python3 bench/pmc_summary.py "$OUT" > "$OUT/summary.txt"
grep -E "^==|persist_kernel<false, 2, 4>|rbf_gemm" "$OUT/summary.txt" | grep -v "0.00[0-9] ms"
find "$OUT" -name "*.csv" -delete
