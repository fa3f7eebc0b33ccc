#!/bin/bash
# The other BASELINE.json configs on one MI355X (bench.py presets):
# adult-shape (converges), covtype-shape 581k x 54 cache mode (3M-iteration
# cap of Makefile:77), synthetic 2M x 1024 (capped: per-iteration cost).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name timeout args...
  local name=$1 tmo=$2; shift 2
  timeout -k 10 $tmo python -u bench.py "$@" > gpurun_out/cfg_$name.log 2>&1 || { echo "$name failed rc=$?"; tail -5 gpurun_out/cfg_$name.log; return 1; }
  echo -n "$name: "; grep '^{' gpurun_out/cfg_$name.log | tail -1 | tee gpurun_out/cfg_$name.json
}
run adult 200 --config adult --steps 3 --warmup 1 &&
run synthetic2m 300 --config synthetic-2m --max-iter ${ITERS_2M:-3000} --steps 1 --warmup 0 --no-accuracy &&
run covtype 400 --config covtype --steps 1 --warmup 0 --no-accuracy
