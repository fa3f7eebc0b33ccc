# kernel-time profile of the recompute rounds (covtype phase-0 shape, 300k pair steps)
set -o pipefail
mkdir -p gpurun_out/r5rp
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5rp -o run -- python3 -u bench/ws_stamps.py --data covtype --samples 581012 --features 54 --C 2048 --gamma 0.03125 --clip box --ws-blocks 1 --max-iter 300000 > gpurun_out/r5rp/out.txt 2> gpurun_out/r5rp/err.txt || { tail -5 gpurun_out/r5rp/err.txt; exit 1; }
f=$(find gpurun_out/r5rp -name "*kernel_stats.csv" | head -1); head -12 "$f"
