# headline rounds vs the round's union size (blocks x 48 rows): does the round count scale as 1 / union?
set -o pipefail
mkdir -p gpurun_out/r5u
for b in 64 32 16; do
  timeout -k 10 240 python3 -u bench.py --steps 3 --warmup 1 --reference-check off --secondary off --ws-blocks $b --ws-size 48 \
    > gpurun_out/r5u/b$b.json 2> gpurun_out/r5u/b$b.err || { tail -5 gpurun_out/r5u/b$b.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r5u/b$b.json').read().strip().splitlines()[-1]); print('blocks $b', d['value'], d.get('ws_rounds'), d.get('iterations'), d.get('gram_gemm_s'))"
done
