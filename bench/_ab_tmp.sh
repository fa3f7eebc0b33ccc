export TMPDIR=/tmp
for st in 0 4 8 12 0; do
  DPSVM_H1_STAGGER_US=$st timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_st_$st -o run --output-format csv -- python3 bench/gram_adapt_probe.py --reps 3 --cases sym --adaptive-only > gpurun_out/st_$st.log 2>&1 || exit 1
  echo "st $st done"
done
