# inputs of the 8-GPU plan for covtype / synthetic-2m (one MI355X):
#  - per-kernel time per round at the full shapes (rocprofv3 kernel trace of a
#    capped plain solve): which kernels scale with a rank's rows (f-update
#    passes, miss-row GEMM) and which are redundant on every rank (merge,
#    gather, solve)
#  - the loopback peer exchange's per-round cost at covtype shape
#  - one rank's dense Gram slab at covtype P = 8 (169 GB)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 -u $R/bench.py --no-accuracy --reference-check off --shrink off --steps 1 --warmup 0"
COV="--config covtype --clip box --max-iter 2000000"
SYN="--config synthetic-2m --max-iter 120000"
timeout -k 10 200 $B $COV --json-out $R/gpurun_out/r4b_cov_local.json > /dev/null 2> $R/gpurun_out/r4b_cov_local.err &&
timeout -k 10 200 $B $COV --exchange peer --json-out $R/gpurun_out/r4b_cov_peer.json > /dev/null 2> $R/gpurun_out/r4b_cov_peer.err &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4b_prof_cov -o cov --output-format csv -- python3 -u $R/bench.py --no-accuracy --reference-check off --shrink off --steps 1 --warmup 0 $COV --json-out $R/gpurun_out/r4b_cov_prof.json > $R/gpurun_out/r4b_prof_cov.log 2>&1) &&
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4b_prof_syn -o syn --output-format csv -- python3 -u $R/bench.py --no-accuracy --reference-check off --shrink off --steps 1 --warmup 0 $SYN --json-out $R/gpurun_out/r4b_syn_prof.json > $R/gpurun_out/r4b_prof_syn.log 2>&1) &&
timeout -k 10 300 $B $SYN --json-out $R/gpurun_out/r4b_syn_local.json > /dev/null 2> $R/gpurun_out/r4b_syn_local.err &&
timeout -k 10 200 python3 -u bench/slab_probe.py --P 8 --out gpurun_out/r4b_slab_cov.json > gpurun_out/r4b_slab_cov.log 2>&1
rc=$?
find gpurun_out -name "*kernel_stats.csv" | head
cat gpurun_out/r4b_slab_cov.json 2>/dev/null
exit $rc
