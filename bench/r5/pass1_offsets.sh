# pass 1: apply-segment offsets by one wave scan + binary search; merge hash tables in 4-slot buckets; pass 2 at
# world > 1: the non-owned rows' alphas over flat slots.  ws tests (+ the multi-process exchange tests), bench,
# stamps, then the sharded headline rehearsed with 2 ranks on one GPU
set -o pipefail
mkdir -p gpurun_out/r5po
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_ws_kernels_gpu.py tests/test_ws_gpu.py \
  > gpurun_out/r5po/pytest.log 2>&1 || { tail -40 gpurun_out/r5po/pytest.log; exit 1; }
tail -1 gpurun_out/r5po/pytest.log
for rep in 1 2 3; do
  timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 3 --secondary off > gpurun_out/r5po/b_$rep.json 2> gpurun_out/r5po/b_$rep.err || { tail -5 gpurun_out/r5po/b_$rep.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r5po/b_$rep.json').read().strip().splitlines()[-1]); rc=d['reference_check']; print('bench', d['value'], 'rounds', d['rounds'], 'it', d['iterations'], 'gram', d['gram_gemm_s'], 'b', d['b'], 'conv', d['converged'], rc['decision_sign_agreement'])"
done
timeout -k 10 300 python3 -u bench/ws_stamps.py --out gpurun_out/r5po/stamps.json > gpurun_out/r5po/stamps.txt 2>&1 || { tail -5 gpurun_out/r5po/stamps.txt; exit 1; }
tail -1 gpurun_out/r5po/stamps.txt
DPSVM_FORCE_DEVICE=0 timeout -k 10 400 python3 -u bench.py --gpus 2 --dp shard --steps 3 --warmup 1 \
    --json-out gpurun_out/r5po/g2.json > gpurun_out/r5po/g2.log 2>&1 || { tail -8 gpurun_out/r5po/g2.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r5po/g2.json')); print('P=2', d['value'], d['config']['parallelism'], d['ws_exchange'], d['ws_blocks'], d['converged'], d['rounds'], d['b'], d['engine_note'])"
