#!/bin/bash
# One parametrized GPU-box runner (used through gpurun; replaces the per-
# experiment recipes of round 1).  Every GPU step runs under its own time limit
# and the script stops at the first failure.
#
#   bench/gpu.sh tests [pytest -k EXPR]        pytest -m gpu            -> gpurun_out/pytest_gpu.log
#   bench/gpu.sh bench [bench.py args]         one process, device 0    -> gpurun_out/bench_$TAG.log
#   bench/gpu.sh mp N [bench.py args]          N ranks as N processes sharing device 0 (gloo bootstrap,
#                                              in-kernel peer exchange; rehearsal of the N-GPU run)
#                                                                       -> gpurun_out/mp${N}_$TAG.log
#   bench/gpu.sh prof [bench.py args]          rocprofv3 kernel trace   -> gpurun_out/prof_$TAG/
#   bench/gpu.sh pmc "C1 C2 .." [bench.py args]  one counter pass       -> gpurun_out/pmc_$TAG/
#   bench/gpu.sh py SCRIPT [args]              a python driver script   -> gpurun_out/py_$TAG.log
#   bench/gpu.sh round                         tests + headline bench + kernel-trace profile
#
# Environment: TAG (output name, default "run"), LIMIT (seconds per GPU step, default 600),
# any DPSVM_* variable is passed through to the solver.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-run}
LIMIT=${LIMIT:-600}
task=${1:-round}
shift || true

summary() {  # one-line digest of a bench JSON line
  grep '^{' "$1" | tail -1 | python3 -c "import json,sys
d=json.loads(sys.stdin.read())
it=max(1,d.get('iterations',1))
print(d['n_gpus'],'ranks', d['value'],'s', it,'iters', d.get('n_sv'),'SVs b', d.get('b'), d.get('iteration'), d.get('exchange'), d.get('exchange_mem'), 'geom', d.get('geometry'), round(1e6*d.get('smo_loop_s_max',0)/it,2),'us/iter')"
}

case "$task" in
  tests)
    K=()
    [ -n "$1" ] && K=(-k "$1")
    timeout -k 10 "$LIMIT" python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread "${K[@]}" \
      > gpurun_out/pytest_gpu.log 2>&1
    rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log; exit $rc ;;
  bench)
    timeout -k 10 "$LIMIT" python -u bench.py "$@" > "gpurun_out/bench_$TAG.log" 2>&1
    rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] && summary "gpurun_out/bench_$TAG.log" || tail -20 "gpurun_out/bench_$TAG.log"
    exit $rc ;;
  mp)
    N=$1; shift
    export DPSVM_FORCE_DEVICE=0 DPSVM_XCH_TIMEOUT_S=${DPSVM_XCH_TIMEOUT_S:-30} GPU_MAX_HW_QUEUES=${DPSVM_REHEARSAL_HW_QUEUES:-2}
    timeout -k 10 "$LIMIT" python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" \
      --master-addr 127.0.0.1 --master-port $((29600 + N)) bench.py --gpus "$N" --comm gloo "$@" \
      > "gpurun_out/mp${N}_$TAG.log" 2>&1
    rc=$?; echo "mp$N rc=$rc"; [ $rc -eq 0 ] && summary "gpurun_out/mp${N}_$TAG.log" || tail -20 "gpurun_out/mp${N}_$TAG.log"
    exit $rc ;;
  prof)
    timeout -k 10 "$LIMIT" rocprofv3 --kernel-trace --stats -d "gpurun_out/prof_$TAG" -o run --output-format csv \
      -- python3 bench.py "$@" > "gpurun_out/prof_$TAG.log" 2>&1
    rc=$?; echo "rocprof rc=$rc"
    f=$(find "gpurun_out/prof_$TAG" -name "*kernel_stats.csv" | head -1)
    [ -n "$f" ] && cut -d, -f1-8 "$f" | head -12
    exit $rc ;;
  pmc)
    CTR=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc $CTR -d "gpurun_out/pmc_$TAG" -o run --output-format csv \
      -- python3 bench.py "$@" > "gpurun_out/pmc_$TAG.log" 2>&1
    rc=$?; echo "pmc rc=$rc"; exit $rc ;;
  py)
    S=$1; shift
    timeout -k 10 "$LIMIT" python -u "$S" "$@" > "gpurun_out/py_$TAG.log" 2>&1
    rc=$?; echo "py rc=$rc"; tail -30 "gpurun_out/py_$TAG.log"; exit $rc ;;
  round)
    "$0" tests || exit $?
    TAG=round "$0" bench --steps 3 --warmup 1 || exit $?
    TAG=round "$0" prof --steps 1 --warmup 0 --no-accuracy ;;
  *)
    echo "unknown task $task"; exit 2 ;;
esac
