# end-of-round check after the Gram epilogue change: full GPU suite, smoke, headline bench, headline stamps
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4h_pytest_gpu_full.log 2>&1 &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4h_smoke.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/r4h_bench_n1.json > /dev/null 2> gpurun_out/r4h_bench_n1.err &&
timeout -k 10 200 python3 -u bench/ws_stamps.py --out gpurun_out/r4h_stamps_headline.json > /dev/null 2> gpurun_out/r4h_stamps.err
rc=$?; tail -2 gpurun_out/r4h_pytest_gpu_full.log; tail -2 gpurun_out/r4h_smoke.log
python3 -c "
import json
d=json.loads(open('gpurun_out/r4h_bench_n1.json').read()); print('bench', d['value'], d['rounds'], d['gram_gemm_s'], d['reference_check']['abs_b_diff'])
d=json.load(open('gpurun_out/r4h_stamps_headline.json')); print({k: d.get(k) for k in ('rounds','pair_steps','b','solve_us','solve_end_to_next_select_us','round_period_us')})
"
exit $rc
