set -o pipefail
mkdir -p gpurun_out

timeout -k 5 60 bin/mfma_swap_probe 4096 49 0 > gpurun_out/r4_mfma_swap_probe.txt &&
timeout -k 5 60 bin/mfma_swap_probe 4096 1 0 >> gpurun_out/r4_mfma_swap_probe.txt &&
timeout -k 5 60 bin/mfma_swap_probe 4096 49 1 >> gpurun_out/r4_mfma_swap_probe.txt &&
cat gpurun_out/r4_mfma_swap_probe.txt &&
DPSVM_SPLIT_GEMM=4 timeout -k 10 120 python3 bench/gram_ab.py --only split > gpurun_out/r4_gram_v4.txt 2>&1 &&
DPSVM_SPLIT_GEMM=5 timeout -k 10 120 python3 bench/gram_ab.py --only split > gpurun_out/r4_gram_v5.txt 2>&1 &&
tail -1 gpurun_out/r4_gram_v4.txt gpurun_out/r4_gram_v5.txt &&
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ws_gpu.py -k "peer" > gpurun_out/r4_pytest_ws_peer.log 2>&1; tail -15 gpurun_out/r4_pytest_ws_peer.log
