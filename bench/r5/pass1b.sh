# wide pass 1 as the default: kernel numerics, pass-1 probe at the shard shapes, headline, 4/8-rank rehearsals
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ws_kernels_gpu.py tests/test_ws_gpu.py -k "select or multi_block or peer_exchange" > gpurun_out/r5w_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r5w_pytest.log; [ $rc -eq 0 ] || { grep -E "^E " gpurun_out/r5w_pytest.log | head; exit $rc; }
timeout -k 10 300 python3 -u bench/pass1_probe.py --cols 7500,15000,30000,60000 --ks 1,2,4,8 --out gpurun_out/r5w_probe_v1.jsonl > /dev/null 2>&1 || exit 1
timeout -k 10 300 python3 -u bench/pass1_probe.py --cols 7500,15000,30000,60000 --ks 4,8,17,32 --wide --out gpurun_out/r5w_probe_wide.jsonl > /dev/null 2>&1 || exit 1
python3 -c "
import json
for f in ('v1','wide'):
    for l in open(f'gpurun_out/r5w_probe_{f}.jsonl'):
        d=json.loads(l); print(f, d['cols'], d['p1G'], d['ks'], d['workgroups'], d['pass1_us_median'], d['GBps'])"
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --json-out gpurun_out/r5w_bench.json > gpurun_out/r5w_bench.log 2>&1 || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r5w_bench.json')); print('headline', d['value'], d['gram_gemm_s'], d['rounds'], d['converged'], d['b'], d['reference_check']['decision_sign_agreement'])"
for N in 4 8; do
  DPSVM_FORCE_DEVICE=0 timeout -k 10 400 python3 -u bench.py --gpus $N --dp shard --steps 3 --warmup 1 --no-accuracy --reference-check off --json-out gpurun_out/r5w_mp$N.json > gpurun_out/r5w_mp$N.log 2>&1 || { tail -20 gpurun_out/r5w_mp$N.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5w_mp$N.json')); print('shard $N ranks (one GPU)', d['value'], d['ws_exchange'], d['rounds'], d['converged'], d['b'])"
done
# blocks per round: 32 x 96 (default) vs 64 x 48 (one slot per lane in the solve)
for B in 32 64 32 64; do
  DPSVM_WS_AUTO_BLOCKS=$B timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --reference-check off --no-accuracy --json-out gpurun_out/r5b_$B.json > gpurun_out/r5b_$B.log 2>&1 || { tail -20 gpurun_out/r5b_$B.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5b_$B.json')); print('blocks $B', d['value'], d['rounds'], d['iterations'], d['ws_blocks'], d['converged'], d['b'])" | tee -a gpurun_out/r5b_summary.txt
done
for cfg in mnist-parity mnist-makefile; do
  for B in 32 64; do
    DPSVM_WS_AUTO_BLOCKS=$B timeout -k 10 300 python3 -u bench.py --config $cfg --steps 5 --warmup 1 --reference-check off --no-accuracy --json-out gpurun_out/r5b_${cfg}_$B.json > gpurun_out/r5b_${cfg}_$B.log 2>&1 || { tail -20 gpurun_out/r5b_${cfg}_$B.log; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r5b_${cfg}_$B.json')); print('$cfg blocks $B', d['value'], d['rounds'], d['iterations'], d['ws_blocks'], d['converged'], d['b'])" | tee -a gpurun_out/r5b_summary.txt
  done
done
DPSVM_WS_AUTO_BLOCKS=64 timeout -k 10 300 python3 -u bench/ws_stamps.py --out gpurun_out/r5b_stamps_64.json > /dev/null 2> gpurun_out/r5b_stamps_64.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r5b_stamps_64.json')); print(d)" | tee -a gpurun_out/r5b_summary.txt
