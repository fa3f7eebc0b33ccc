# wide-wave split Gram GEMM (variant 5) vs the persistent LDS-DMA default (4):
# bit-identity tests, then the headline Gram timed (events + rocprof kernel stats)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_split_gemm_gpu.py > gpurun_out/r4w_pytest.log 2>&1 &&
DPSVM_SPLIT_GEMM=4 timeout -k 10 120 python3 -u bench/gram_ab.py --only split --reps 5 > gpurun_out/r4w_gram_v4.log 2>&1 &&
DPSVM_SPLIT_GEMM=5 timeout -k 10 120 python3 -u bench/gram_ab.py --only split --reps 5 > gpurun_out/r4w_gram_v5.log 2>&1 &&
(cd /tmp && DPSVM_SPLIT_GEMM=5 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4w_prof -o w --output-format csv -- python3 -u $GRAFT_REPO_ROOT/bench/gram_ab.py --only split --reps 3 > $GRAFT_REPO_ROOT/gpurun_out/r4w_prof.log 2>&1)
rc=$?
tail -3 gpurun_out/r4w_pytest.log
grep split gpurun_out/r4w_gram_v4.log gpurun_out/r4w_gram_v5.log | head -4
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/r4w_prof/*kernel_stats.csv"):
    for r in list(csv.DictReader(open(f)))[:4]:
        print("  %-50s calls %5s avg_ms %8.3f min_ms %8.3f" % (r["Name"][:50], r["Calls"], float(r["AverageNs"])/1e6, float(r["MinNs"])/1e6))
PY
exit $rc
