#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" | tee -a gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench/iter_latency.py --out gpurun_out/iter_latency.jsonl > gpurun_out/iter_latency.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lru -o lru --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-accuracy --cache-lines 20000 > gpurun_out/prof_lru.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --comm rccl > gpurun_out/bench_rccl1.log 2>&1 || exit $?
tail -1 gpurun_out/bench_rccl1.log
