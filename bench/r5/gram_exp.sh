# (historical: the A/B switch / code this script exercised was removed after its measurement; see profiles/)
# split Gram epilogue: hardware exp (default) vs libm expf (DPSVM_GRAM_NT=4), then the headline
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/r5x_ab.txt
for k in 1 2 3; do
  for T in 0 4; do
    DPSVM_GRAM_NT=$T timeout -k 10 200 python3 -u bench/gram_ab.py --only split --reps 5 2>&1 | grep '^split' | sed "s/^/nt=$T /" >> gpurun_out/r5x_ab.txt || exit 1
  done
done
cut -c1-70 gpurun_out/r5x_ab.txt
timeout -k 10 300 python3 -u -m pytest tests/test_split_gemm_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5x_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r5x_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --json-out gpurun_out/r5x_b.json > gpurun_out/r5x_b.log 2>&1 || { tail -5 gpurun_out/r5x_b.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r5x_b.json')); rc=d['reference_check']; print(d['value'], d['gram_gemm_s'], d['rounds'], d['converged'], rc['decision_sign_agreement'], rc['abs_b_diff'], d['secondary']['value'])"
