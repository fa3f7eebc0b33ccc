# full GPU suite + headline bench (the driver's round-end check)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r5s_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r5s_pytest.log; grep -E "FAILED|ERROR" gpurun_out/r5s_pytest.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --json-out gpurun_out/r5s_bench.json > gpurun_out/r5s_bench.log 2>&1 || { tail -20 gpurun_out/r5s_bench.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5s_bench.json')); print(d['value'], d['gram_gemm_s'], d['rounds'], d['converged'], d['reference_check']['decision_sign_agreement'])"
