# per-kernel time of a headline solve at 6,144- vs 3,072-row unions (rocprofv3 kernel trace)
set -o pipefail
export TMPDIR=/tmp
for u in 6144 3072; do
  mkdir -p gpurun_out/r5ut$u
  DPSVM_WS_UNION=$u timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5ut$u -o run -- python3 -u bench.py --steps 2 --warmup 1 --reference-check off --secondary off --no-accuracy > gpurun_out/r5ut$u/out.txt 2> gpurun_out/r5ut$u/err.txt || { tail -5 gpurun_out/r5ut$u/err.txt; exit 1; }
  echo "== union $u"; python3 bench/timeline_gaps.py gpurun_out/r5ut$u | tail -12
done
