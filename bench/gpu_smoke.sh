#!/bin/bash
# First-light GPU check: native unit tests (device cases) + svmTrain on the
# MNIST-shape headline config.  Run from the repo root on a GPU box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 ./bin/dpsvm_unit --gpu > gpurun_out/unit_gpu.log 2>&1
echo "unit rc=$?" | tee -a gpurun_out/unit_gpu.log
timeout -k 10 300 ./bin/svmTrain -a 784 -x 60000 --synthetic mnist -c 10 -g 0.25 -e 0.001 \
  -m /tmp/mnist_model.txt --metrics-json gpurun_out/mnist_metrics.json --log-every 20000 > gpurun_out/mnist_train.log 2>&1
echo "train rc=$?" | tee -a gpurun_out/mnist_train.log
