# rounds per hipGraph block (ws_block) with 6,144-row unions: the host polls one block behind, so up to two
# blocks of no-op rounds follow convergence
set -o pipefail
mkdir -p gpurun_out/r5wb
for rep in 1 2; do
  for wb in 2 4 8; do
    timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 3 --secondary off --reference-check off --ws-block $wb \
      > gpurun_out/r5wb/b${wb}_$rep.json 2> gpurun_out/r5wb/b${wb}_$rep.err || { tail -5 gpurun_out/r5wb/b${wb}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r5wb/b${wb}_$rep.json').read().strip().splitlines()[-1]); print('ws_block $wb', d['value'], 'rounds', d.get('rounds'), 'gram', d.get('gram_gemm_s'), 'loop', d.get('smo_loop_s_min'), d.get('smo_loop_s_max'))"
  done
done
