# w64 interior-tile epilogue: bit identity, then headline Gram time (before: 10.33-10.37 ms)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_split_gemm_gpu.py > gpurun_out/r4e_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4e_pytest.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2 3; do
  timeout -k 10 200 python3 -u bench/gram_ab.py --only split --reps 5 2>&1 | grep '^split' >> gpurun_out/r4e_ab.txt || exit 1
done
cat gpurun_out/r4e_ab.txt
