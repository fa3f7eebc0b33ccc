#!/bin/bash
# End-of-round GPU evidence on one MI355X: full GPU suite, smoke, default bench (the driver's
# invocation and a 20-step one), svmTrain with the reference's flags (x3), kernel trace of the headline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r3z}
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
echo "pytest rc=$?" > gpurun_out/${T}_status.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
timeout -k 10 120 python bench.py > gpurun_out/${T}_bench_default.json 2> gpurun_out/${T}_bench_default.err || exit 1
timeout -k 10 120 python bench.py --steps 20 --warmup 2 > gpurun_out/${T}_bench_20.json 2> gpurun_out/${T}_bench_20.err || exit 1
for i in 1 2 3; do
  timeout -k 10 60 bin/svmTrain -a 784 -x 60000 --synthetic mnist -c 10 -g 0.25 -e 0.001 -m /tmp/model.txt \
    --metrics-json gpurun_out/${T}_cli_metrics_$i.json > gpurun_out/${T}_cli_$i.log 2>&1 || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/${T}_prof -o run -- python bench.py --steps 3 --reference-check off \
  > gpurun_out/${T}_prof.log 2>&1 || exit 1
echo done >> gpurun_out/${T}_status.txt
