# symmetric Gram: compact tile table (only the upper tiles launched) vs the full grid
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_split_gemm_gpu.py > gpurun_out/r5g2_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r5g2_pytest.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2 3; do
  for C in 0 1; do
    DPSVM_GRAM_COMPACT=$C timeout -k 10 200 python3 -u bench/gram_ab.py --only split --reps 5 2>&1 | grep '^split' | sed "s/^/compact=$C /" >> gpurun_out/r5g2_ab.txt || exit 1
  done
done
cat gpurun_out/r5g2_ab.txt | cut -c1-60
