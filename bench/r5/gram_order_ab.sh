# symmetric split Gram: tile-table group height (DPSVM_GRAM_GM, tile rows of 256) and chunk (DPSVM_GRAM_CH, tiles an
# XCD takes in a row) — L2 reuse of the operand panels; bench/gram_ab.py --only split, 5 reps each
set -o pipefail
mkdir -p gpurun_out/r5go
for cfg in ${CFGS:-"8 64" "4 64" "16 64" "8 32" "8 128" "4 32" "16 128" "8 64"}; do
  set -- $cfg
  DPSVM_GRAM_GM=$1 DPSVM_GRAM_CH=$2 timeout -k 10 200 python3 -u bench/gram_ab.py --only split --reps 5 > gpurun_out/r5go/gm$1_ch$2.txt 2>&1 || { tail -5 gpurun_out/r5go/gm$1_ch$2.txt; exit 1; }
  echo "GM $1 CH $2: $(grep -o '"ms": [0-9.]*' gpurun_out/r5go/gm$1_ch$2.txt | head -1)"
done
