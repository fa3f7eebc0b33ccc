#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
DPSVM_STAMPS=/tmp/st timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-accuracy > gpurun_out/stamps_bench.log 2>&1 || exit $?
python bench/stamps_report.py /tmp/st.rank0 > gpurun_out/stamps.json 2>&1
cat gpurun_out/stamps.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lru -o lru --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-accuracy --cache-lines 20000 > gpurun_out/prof_lru.log 2>&1 || exit $?
timeout -k 10 900 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" | tee -a gpurun_out/pytest_gpu.log
