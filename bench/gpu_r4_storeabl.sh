set -o pipefail
mkdir -p gpurun_out
for nt in 0 2 0 2; do
  echo "== DPSVM_GRAM_NT=$nt" >> gpurun_out/r4s_abl.txt
  DPSVM_GRAM_NT=$nt timeout -k 10 200 python3 -u bench/gram_ab.py --only split --reps 5 >> gpurun_out/r4s_abl.txt 2>&1 || exit 1
done
cat gpurun_out/r4s_abl.txt
