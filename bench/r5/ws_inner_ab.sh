# per-block pair-step cap of the multi-block rounds (ws_inner; default 4 q = 192 for 48-row blocks): the round's
# solve waits for its slowest block
set -o pipefail
mkdir -p gpurun_out/r5wi
for rep in 1 2; do
  for wi in 0 64 48 36; do
    timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 3 --secondary off --reference-check off --ws-inner $wi > gpurun_out/r5wi/b${wi}_$rep.json 2> gpurun_out/r5wi/b${wi}_$rep.err || { tail -5 gpurun_out/r5wi/b${wi}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r5wi/b${wi}_$rep.json').read().strip().splitlines()[-1]); print('ws_inner $wi', d['value'], 'rounds', d['rounds'], 'it', d['iterations'], 'gram', d['gram_gemm_s'], 'b', d['b'], 'conv', d['converged'])"
  done
done
