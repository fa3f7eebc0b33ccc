set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 bench/ws_stamps.py --out gpurun_out/r4s_stamps_local.json > /dev/null 2>gpurun_out/r4s_local.err &&
timeout -k 10 200 python3 bench/ws_stamps.py --exchange peer --out gpurun_out/r4s_stamps_peer.json > /dev/null 2>gpurun_out/r4s_peer.err
rc=$?; cat gpurun_out/r4s_stamps_local.json gpurun_out/r4s_stamps_peer.json; exit $rc
