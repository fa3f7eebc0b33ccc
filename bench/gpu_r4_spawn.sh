set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 > gpurun_out/r4_bench_n1.json 2> gpurun_out/r4_bench_n1.err &&
DPSVM_FORCE_DEVICE=0 timeout -k 10 400 python3 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/r4_bench_spawn2.json 2> gpurun_out/r4_bench_spawn2.err &&
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_failure_gpu.py > gpurun_out/r4_failure_gpu.log 2>&1
