# A/B: plain vs non-temporal Gram stores in the wide-wave split GEMM (headline)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_split_gemm_gpu.py > gpurun_out/r4nt_pytest.log 2>&1 || exit 1
for nt in 0 1 0 1; do
  DPSVM_GRAM_NT=$nt timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/r4nt_$nt.json > /dev/null 2> gpurun_out/r4nt_$nt.err || exit 1
  python3 -c "
import json
d=json.loads(open('gpurun_out/r4nt_$nt.json').read())
print('nt=$nt', d['value'], 'gram', d['gram_gemm_s'], 'loop', d['smo_loop_s_min'], 'rounds', d['rounds'], 'b', d['b'])
" | tee -a gpurun_out/r4nt_summary.txt
done
tail -1 gpurun_out/r4nt_pytest.log
