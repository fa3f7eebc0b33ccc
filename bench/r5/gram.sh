# Gram w64 kernel with one epilogue path (no scratch): bit identity, Gram time, headline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_split_gemm_gpu.py > gpurun_out/r5g_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r5g_pytest.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2 3; do
  timeout -k 10 200 python3 -u bench/gram_ab.py --only split --reps 5 2>&1 | grep '^split' >> gpurun_out/r5g_ab.txt || exit 1
done
cat gpurun_out/r5g_ab.txt
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 > gpurun_out/r5g_bench.log 2>&1 || exit 1
grep '^{' gpurun_out/r5g_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['gram_gemm_s'], d['rounds'], d['converged'])"
