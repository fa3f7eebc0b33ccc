# end-of-round check on one MI355X: the GPU suite, smoke, the headline bench,
# and a 2-process rehearsal of the big-shape policy (shrink auto decided over
# the communicator: a capped cache makes the Gram non-resident)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4g_pytest_gpu_full.log 2>&1 &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4g_smoke.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/r4g_bench_n1.json > /dev/null 2> gpurun_out/r4g_bench_n1.err &&
DPSVM_FORCE_DEVICE=0 timeout -k 10 400 python3 -u bench.py --gpus 2 --comm gloo --config covtype --samples 100000 --clip box --max-iter 60000000 --cache-mb 3000 --steps 1 --warmup 0 --no-accuracy --json-out gpurun_out/r4g_shrink2p_auto.json > /dev/null 2> gpurun_out/r4g_shrink2p_auto.err
rc=$?; tail -2 gpurun_out/r4g_pytest_gpu_full.log; tail -2 gpurun_out/r4g_smoke.log
python3 -c "
import json
d=json.loads(open('gpurun_out/r4g_bench_n1.json').read()); print('bench', d['value'], d['rounds'], d['gram_gemm_s'], d['reference_check']['abs_b_diff'])
d=json.loads(open('gpurun_out/r4g_shrink2p_auto.json').read()); print('shrink2p', d['value'], d['n_gpus'], d['converged'], d['iteration'], d['dp_policy'], d['shrink'])
"
exit $rc
