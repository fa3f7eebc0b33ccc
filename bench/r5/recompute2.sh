set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_ws_recompute_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r5r_pytest2.log 2>&1
rc=$?; grep -E "passed|failed|FAIL|Error|rounds .* vs" gpurun_out/r5r_pytest2.log | tail -8; [ $rc -eq 0 ] || exit $rc
DPSVM_WS_RECOMPUTE=1 timeout -k 10 400 python3 -u bench/ws_stamps.py --data covtype --samples 581012 --features 54 --C 2048 --gamma 0.03125 --clip box --ws-blocks 1 --max-iter 1000000 --out gpurun_out/r5r_stamps_cov581k_1b.json > /dev/null 2> gpurun_out/r5r_stamps_1b.err || { tail -5 gpurun_out/r5r_stamps_1b.err; exit 1; }
cat gpurun_out/r5r_stamps_cov581k_1b.json
