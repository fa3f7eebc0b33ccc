set -o pipefail
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 bench/mfma_swap_probe.hip -o /tmp/mfma_swap_probe 2>/dev/null &&
timeout -k 5 60 /tmp/mfma_swap_probe 4096 49 0 > gpurun_out/r4_mfma_swap_probe.txt &&
timeout -k 5 60 /tmp/mfma_swap_probe 4096 1 0 >> gpurun_out/r4_mfma_swap_probe.txt &&
timeout -k 5 60 /tmp/mfma_swap_probe 4096 49 1 >> gpurun_out/r4_mfma_swap_probe.txt &&
cat gpurun_out/r4_mfma_swap_probe.txt &&
DPSVM_SPLIT_GEMM=4 timeout -k 10 120 python3 bench/gram_ab.py --only split > gpurun_out/r4_gram_v4.txt 2>&1 &&
DPSVM_SPLIT_GEMM=5 timeout -k 10 120 python3 bench/gram_ab.py --only split > gpurun_out/r4_gram_v5.txt 2>&1 &&
tail -1 gpurun_out/r4_gram_v4.txt gpurun_out/r4_gram_v5.txt &&
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ws_gpu.py tests/test_ws_kernels_gpu.py tests/test_split_gemm_gpu.py > gpurun_out/r4_pytest_ws_split.log 2>&1; tail -3 gpurun_out/r4_pytest_ws_split.log
