# direct sub-Gram loads for 96-row blocks too (DPSVM_WS_DIRECT_SUB=2) on the coupled mnist-parity preset
# (32 x 96 blocks), vs the gather kernel; then headline stamps with the default (<= 64-row blocks direct)
set -o pipefail
mkdir -p gpurun_out/r5d96
for rep in 1 2; do
  for d in 2 1; do
    DPSVM_WS_DIRECT_SUB=$d timeout -k 10 240 python3 -u bench.py --config mnist-parity --steps 10 --warmup 3 --reference-check off > gpurun_out/r5d96/p${d}_$rep.json 2> gpurun_out/r5d96/p${d}_$rep.err || { tail -5 gpurun_out/r5d96/p${d}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r5d96/p${d}_$rep.json').read().strip().splitlines()[-1]); print('parity direct_env $d', d['value'], 'rounds', d['rounds'], 'it', d['iterations'], 'b', d['b'], 'conv', d['converged'])"
  done
done
timeout -k 10 300 python3 -u bench/ws_stamps.py --out gpurun_out/r5d96/stamps.json > gpurun_out/r5d96/stamps.txt 2>&1 || { tail -5 gpurun_out/r5d96/stamps.txt; exit 1; }
tail -1 gpurun_out/r5d96/stamps.txt
