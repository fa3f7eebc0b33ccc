#!/bin/bash
# UTCL1 (per-CU address translation) counters of the persistent engines:
# dense headline vs cache mode (covtype-shape, capped): TLB-reach check.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_tlb}
mkdir -p "$OUT"
CNT="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_TCC_READ_REQ_sum"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CNT -d "$OUT/dense" -o pmc --output-format csv -- \
  python3 bench.py --steps 1 --warmup 0 --no-accuracy > "$OUT/dense.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CNT -d "$OUT/cache" -o pmc --output-format csv -- \
  python3 bench/lru_profile_run.py 8 100000 covtype 581012 0 > "$OUT/cache.log" 2>&1 || exit $?
python3 bench/pmc_summary.py "$OUT" > "$OUT/summary.txt"
grep -E "^==|persist|fused|gemm" "$OUT/summary.txt" | grep -v "REQUEST_sum=0,"
grep -h '^{' "$OUT/dense.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('dense engine:', d['iteration'], d['exchange'])"
grep -h "iteration" "$OUT/cache.log" | head -2
find "$OUT" -name "*.csv" -delete
