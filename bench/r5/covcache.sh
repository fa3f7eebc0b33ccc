# covtype box phase-0 shape (581k rows, ws-cache) round anatomy: 1M pair steps with stamps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u bench/ws_stamps.py --data covtype --samples 581012 --features 54 --C 2048 --gamma 0.03125 --clip box --ws-blocks 1 --max-iter 1000000 --out gpurun_out/r5c_stamps_cov581k_cache.json > /dev/null 2> gpurun_out/r5c_stamps.err || { tail -5 gpurun_out/r5c_stamps.err; exit 1; }
cat gpurun_out/r5c_stamps_cov581k_cache.json
