set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_ws_gpu.py -k "peer" > gpurun_out/r4_pytest_ws_peer.log 2>&1
rc=$?; tail -15 gpurun_out/r4_pytest_ws_peer.log; exit $rc
