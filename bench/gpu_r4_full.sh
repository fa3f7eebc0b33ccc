set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4_pytest_gpu_full.log 2>&1
rc=$?; tail -8 gpurun_out/r4_pytest_gpu_full.log; exit $rc
