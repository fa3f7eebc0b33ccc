# LDS-DMA ROWS GEMM (ws-cache miss rows): bit-identity tests, then capped
# synthetic-2m / covtype runs, new kernel vs the register-staged one (A/B)
set -o pipefail
mkdir -p gpurun_out
B="python3 -u bench.py --no-accuracy --reference-check off --shrink off --steps 1 --warmup 0"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_split_gemm_gpu.py tests/test_ws_gpu.py -k "cache or rows or split" > gpurun_out/r4r_pytest.log 2>&1 &&
timeout -k 10 300 $B --config synthetic-2m --max-iter 120000 --json-out gpurun_out/r4r_syn_new.json > /dev/null 2> gpurun_out/r4r_syn_new.err &&
DPSVM_ROWS_KERNEL=reg timeout -k 10 300 $B --config synthetic-2m --max-iter 120000 --json-out gpurun_out/r4r_syn_reg.json > /dev/null 2> gpurun_out/r4r_syn_reg.err &&
timeout -k 10 200 $B --config covtype --clip box --max-iter 2000000 --json-out gpurun_out/r4r_cov_new.json > /dev/null 2> gpurun_out/r4r_cov_new.err &&
DPSVM_ROWS_KERNEL=reg timeout -k 10 200 $B --config covtype --clip box --max-iter 2000000 --json-out gpurun_out/r4r_cov_reg.json > /dev/null 2> gpurun_out/r4r_cov_reg.err &&
DPSVM_ROWS_KERNEL=glds timeout -k 10 200 $B --config covtype --clip box --max-iter 2000000 --json-out gpurun_out/r4r_cov_glds.json > /dev/null 2> gpurun_out/r4r_cov_glds.err &&
HSA_ENABLE_IPC_MODE_LEGACY=0 DPSVM_FORCE_DEVICE=0 timeout -k 10 400 python3 -u bench.py --gpus 2 --comm gloo --config covtype --samples 120000 --clip box --shrink on --max-iter 60000000 --steps 1 --warmup 0 --no-accuracy --json-out gpurun_out/r4r_shrink2p.json > /dev/null 2> gpurun_out/r4r_shrink2p.err
rc=$?
tail -4 gpurun_out/r4r_pytest.log
for f in syn_new syn_reg cov_new cov_reg cov_glds shrink2p; do python3 -c "
import json
d=json.loads(open('gpurun_out/r4r_$f.json').read())
print('$f', d['value'], 'rounds', d['rounds'], 'steps', d['iterations'], 'b', d['b'], 'gap', d['final_gap'], 'us/round', round(1e6*d['value']/max(1,d['rounds']),1))
" 2>/dev/null; done
exit $rc
