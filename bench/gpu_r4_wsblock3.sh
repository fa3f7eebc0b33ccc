# 8-round graph blocks (new default) with the one-block switch on 32-round boundaries: ws suites, then the presets
# (expected: the ws_block=32 trajectories of profiles/r4_ws_block_ab.txt, less overshoot after convergence)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ws_gpu.py tests/test_solver_gpu.py > gpurun_out/r4wb3_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4wb3_pytest.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/r4wb3_pytest.log; exit $rc; }
run() {  # tag args...
  local tag=$1; shift
  timeout -k 10 400 python3 -u bench.py "$@" --json-out gpurun_out/r4wb3_${tag}.json > /dev/null 2> gpurun_out/r4wb3_${tag}.err || return 1
  python3 -c "
import json
d=json.loads(open('gpurun_out/r4wb3_${tag}.json').read())
print('$tag', d['value'], 'rounds', d.get('rounds'), 'iters', d.get('iterations'), 'conv', d.get('converged'), 'b', d['b'])
" | tee -a gpurun_out/r4wb3_summary.txt
}
run headline --steps 10 --warmup 2 || exit 1
run headline2 --steps 10 --warmup 2 || exit 1
run parity --config mnist-parity --steps 5 --warmup 1 || exit 1
run makefile --config mnist-makefile --steps 5 --warmup 1 || exit 1
run covbox --config covtype --clip box --max-iter 60000000 --steps 1 --warmup 0 --no-accuracy --reference-check off || exit 1
run syn2m --config synthetic-2m --steps 1 --warmup 0 --no-accuracy --reference-check off || exit 1
