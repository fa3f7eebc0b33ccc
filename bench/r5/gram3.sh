# Gram: merged P+Q accumulator diagnostic (NT=3) vs the default (NT=0)
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/r5g3_ab.txt
for k in 1 2 3; do
  for T in 0 3; do
    DPSVM_GRAM_NT=$T timeout -k 10 200 python3 -u bench/gram_ab.py --only split --reps 5 2>&1 | grep '^split' | sed "s/^/nt=$T /" >> gpurun_out/r5g3_ab.txt || exit 1
  done
done
cat gpurun_out/r5g3_ab.txt | cut -c1-80
