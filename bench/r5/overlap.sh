# (historical: the A/B switch / code this script exercised was removed after its measurement; see profiles/)
# progressive Gram: equivalence test, then headline / mnist-parity A/B (DPSVM_GRAM_OVERLAP=0: Gram first)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gram_progressive_gpu.py -x -v -s --timeout 500 --timeout-method thread > gpurun_out/r5o_pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAIL|Error|gram-first" gpurun_out/r5o_pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/r5o_ab.txt
for k in 1 2; do
  for ov in 0 1; do
    for cfg in mnist mnist-parity; do
      DPSVM_GRAM_OVERLAP=$ov timeout -k 10 300 python3 -u bench.py --config $cfg --steps 5 --warmup 2 --json-out gpurun_out/r5o_b.json > gpurun_out/r5o_b.log 2>&1 || { tail -5 gpurun_out/r5o_b.log; exit 1; }
      python3 -c "
import json; d=json.load(open('gpurun_out/r5o_b.json')); rc=d.get('reference_check') or {}
print('overlap=$ov', '$cfg', d['value'], 'gram', d['gram_gemm_s'], 'rounds', d['rounds'], 'conv', d['converged'], 'agree', rc.get('decision_sign_agreement'), 'db', rc.get('abs_b_diff'))" >> gpurun_out/r5o_ab.txt
    done
  done
done
cat gpurun_out/r5o_ab.txt
