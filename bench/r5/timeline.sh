# headline solve timeline: kernel busy time vs wall span per solve, largest inter-kernel gaps
set -o pipefail
mkdir -p gpurun_out/r5tl
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5tl -o run -- python3 -u bench.py --steps 3 --warmup 1 --reference-check off --secondary off --no-accuracy > gpurun_out/r5tl/out.txt 2> gpurun_out/r5tl/err.txt || { tail -5 gpurun_out/r5tl/err.txt; exit 1; }
python3 bench/timeline_gaps.py gpurun_out/r5tl
