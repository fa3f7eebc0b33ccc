set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_ws_recompute_gpu.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/r5r_pytest3.log 2>&1
rc=$?; grep -E "passed|failed|FAIL|Error|rounds .* vs|blocks" gpurun_out/r5r_pytest3.log | tail -10; [ $rc -eq 0 ] || exit $rc
bash bench/r5/covbox.sh
