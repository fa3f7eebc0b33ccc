export TMPDIR=/tmp
for gc in 4:32 2:32 8:32 4:16 4:64 8:64 2:16 16:64; do
  gm=${gc%%:*}; ch=${gc##*:}
  DPSVM_GRAM_GM=$gm DPSVM_GRAM_CH=$ch timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gc_${gm}_${ch} -o run --output-format csv -- python3 bench/gram_adapt_probe.py --reps 3 --cases sym --adaptive-only > gpurun_out/gc_${gm}_${ch}.log 2>&1 || exit 1
  echo "gc $gm $ch done"
done
