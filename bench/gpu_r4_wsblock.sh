# rounds per hipGraph block (ws_block): the rounds after convergence run as early-exit kernels until the
# host sees the status one block behind; headline bench at 32 (default) / 16 / 8 / 4, alternating
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for wb in 32 16 8 4; do
  timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --ws-block $wb --json-out gpurun_out/r4wb_$wb.json > /dev/null 2> gpurun_out/r4wb_$wb.err || exit 1
  python3 -c "
import json
d=json.loads(open('gpurun_out/r4wb_$wb.json').read())
print('ws_block=$wb', d['value'], 'gram', d['gram_gemm_s'], 'loop', d['smo_loop_s_min'], d['smo_loop_s_max'], 'rounds', d['rounds'], 'b', d['b'])
" | tee -a gpurun_out/r4wb_summary.txt
done
done
