# persistent small-problem rounds: bit-identity tests, then the covtype-shape
# 7.5k-row sub-problem's round anatomy persistent vs graph
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_ws_persist_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r5p_pytest.log 2>&1
rc=$?; grep -E "passed|failed|PASS|FAIL|Error|persistent .* s graph" gpurun_out/r5p_pytest.log | tail -15; [ $rc -eq 0 ] || exit $rc
for m in on off; do
timeout -k 10 300 python3 -u bench/ws_stamps.py --data covtype --samples 7500 --features 54 --C 2048 --gamma 0.03125 --clip box --ws-blocks 1 --ws-persist $m --out gpurun_out/r5p_stamps_cov7500_$m.json > /dev/null 2> gpurun_out/r5p_stamps_$m.err || { tail -5 gpurun_out/r5p_stamps_$m.err; exit 1; }
cat gpurun_out/r5p_stamps_cov7500_$m.json
done
