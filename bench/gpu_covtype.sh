#!/bin/bash
# covtype-shape preset (581012 x 54, C=2048): Gram (1.35 TB) does not fit one
# GPU -> fused cache mode with a ~100k-line CLOCK cache.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python bench.py --config covtype --steps 1 --warmup 0 --no-accuracy > gpurun_out/covtype.log 2>&1
rc=$?; echo "covtype rc=$rc"; grep '^{' gpurun_out/covtype.log | tail -1; tail -3 gpurun_out/covtype.log
exit $rc
