set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4f_pytest_gpu_full.log 2>&1 &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4f_smoke.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --json-out gpurun_out/r4f_bench_n1.json > /dev/null 2> gpurun_out/r4f_bench_n1.err
rc=$?; tail -4 gpurun_out/r4f_pytest_gpu_full.log; tail -3 gpurun_out/r4f_smoke.log; cat gpurun_out/r4f_bench_n1.json | cut -c1-400; exit $rc
