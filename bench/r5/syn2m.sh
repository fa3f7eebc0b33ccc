# synthetic-2m shape (2M x 1024, ws-cache): round anatomy over 100k pair steps (stamps) + kernel times
set -o pipefail
mkdir -p gpurun_out/r5s2m
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r5s2m -o run --output-format csv -- python3 -u bench/ws_stamps.py --data uniform --samples 2000000 --features 1024 --C 1 --gamma 0.0009765625 --clip independent --max-iter 100000 --out gpurun_out/r5s2m/stamps.json > gpurun_out/r5s2m/out.txt 2> gpurun_out/r5s2m/err.txt || { tail -5 gpurun_out/r5s2m/err.txt; exit 1; }
cat gpurun_out/r5s2m/stamps.json
f=$(find gpurun_out/r5s2m -name "*kernel_stats.csv" | head -1); head -14 "$f" | cut -d, -f1-5
