# synthetic-2m miss-row GEMM (LDS-DMA ROWS kernel): B streamed nt vs default, capped runs
set -o pipefail
mkdir -p gpurun_out
B="python3 -u bench.py --no-accuracy --reference-check off --shrink off --steps 1 --warmup 0 --config synthetic-2m --max-iter 120000"
timeout -k 10 300 $B --json-out gpurun_out/r4y_syn_nt.json > /dev/null 2> gpurun_out/r4y_syn_nt.err &&
DPSVM_ROWS_BNT=0 timeout -k 10 300 $B --json-out gpurun_out/r4y_syn_def.json > /dev/null 2> gpurun_out/r4y_syn_def.err
rc=$?
for f in syn_nt syn_def; do python3 -c "
import json
d=json.loads(open('gpurun_out/r4y_$f.json').read())
print('$f', d['value'], 'rounds', d['rounds'], 'b', d['b'], 'us/round', round(1e6*d['value']/max(1,d['rounds']),1))
" 2>/dev/null; done
exit $rc
