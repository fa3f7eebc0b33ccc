# symmetric split Gram tile order, finer sweep around GM 4 / CH 32 (bench/gram_ab.py --only split, 5 reps each)
set -o pipefail
mkdir -p gpurun_out/r5go
for c in "4 32" "2 32" "4 16" "2 16" "4 8" "8 16" "2 64" "4 32" "8 64"; do
  set -- $c
  DPSVM_GRAM_GM=$1 DPSVM_GRAM_CH=$2 timeout -k 10 200 python3 -u bench/gram_ab.py --only split --reps 5 > gpurun_out/r5go/b_gm$1_ch$2.txt 2>&1 || { tail -5 gpurun_out/r5go/b_gm$1_ch$2.txt; exit 1; }
  echo "GM $1 CH $2: $(grep -o '"ms": [0-9.]*' gpurun_out/r5go/b_gm$1_ch$2.txt | head -1)"
done
