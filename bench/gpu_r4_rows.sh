# LDS-DMA ROWS GEMM (ws-cache miss rows): bit-identity tests, then capped
# synthetic-2m / covtype runs, new kernel vs the register-staged one (A/B)
set -o pipefail
mkdir -p gpurun_out
B="python3 -u bench.py --no-accuracy --reference-check off --shrink off --steps 1 --warmup 0"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_split_gemm_gpu.py tests/test_ws_gpu.py -k "cache or rows or split" > gpurun_out/r4r_pytest.log 2>&1 &&
timeout -k 10 200 $B --config covtype --clip box --max-iter 2000000 --json-out gpurun_out/r4r_cov_new.json > /dev/null 2> gpurun_out/r4r_cov_new.err &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4r_prof_cov -o cov --output-format csv -- python3 -u $GRAFT_REPO_ROOT/bench.py --no-accuracy --reference-check off --shrink off --steps 1 --warmup 0 --config covtype --clip box --max-iter 2000000 > $GRAFT_REPO_ROOT/gpurun_out/r4r_prof_cov.log 2>&1) &&
timeout -k 10 300 $B --config covtype --clip box --max-iter 60000000 --shrink auto --json-out gpurun_out/r4r_covbox_shrink.json > /dev/null 2> gpurun_out/r4r_covbox_shrink.err
rc=$?
tail -4 gpurun_out/r4r_pytest.log
for f in cov_new covbox_shrink; do python3 -c "
import json
d=json.loads(open('gpurun_out/r4r_$f.json').read())
print('$f', d['value'], 'rounds', d['rounds'], 'steps', d['iterations'], 'b', d['b'], 'gap', d['final_gap'], 'us/round', round(1e6*d['value']/max(1,d['rounds']),1))
" 2>/dev/null; done
exit $rc
