# one-block round anatomy of a small coupled problem (covtype-shape 7.5k rows,
# C=2048, box: the size of covtype's shrunk phase), and the headline's rounds
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 -u bench/ws_stamps.py --data covtype --samples 7500 --features 54 --C 2048 --gamma 0.03125 --clip box --ws-blocks 1 --out gpurun_out/r4z_stamps_cov7500.json > /dev/null 2> gpurun_out/r4z_stamps_cov7500.err &&
timeout -k 10 200 python3 -u bench/ws_stamps.py --out gpurun_out/r4z_stamps_headline.json > /dev/null 2> gpurun_out/r4z_stamps_headline.err
rc=$?
cat gpurun_out/r4z_stamps_cov7500.json gpurun_out/r4z_stamps_headline.json
exit $rc
