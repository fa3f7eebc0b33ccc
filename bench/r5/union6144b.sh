# 6,144- vs 3,072-row unions after the merge's hash tables went to 8,192 slots (16-bit ranks): kernel tests,
# per-kernel timeline at 6,144, then bench.py alternating
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5w7
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ws_kernels_gpu.py \
  > gpurun_out/r5w7/pytest_kernels.log 2>&1 || { tail -30 gpurun_out/r5w7/pytest_kernels.log; exit 1; }
tail -1 gpurun_out/r5w7/pytest_kernels.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5w7/tl -o run -- python3 -u bench.py --steps 2 --warmup 1 --reference-check off --secondary off --no-accuracy > gpurun_out/r5w7/tl_out.txt 2> gpurun_out/r5w7/tl_err.txt || { tail -5 gpurun_out/r5w7/tl_err.txt; exit 1; }
python3 bench/timeline_gaps.py gpurun_out/r5w7/tl | tail -10
for rep in 1 2; do
  for u in 6144 3072; do
    DPSVM_WS_UNION=$u timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 3 --secondary off \
      > gpurun_out/r5w7/b${u}_$rep.json 2> gpurun_out/r5w7/b${u}_$rep.err || { tail -5 gpurun_out/r5w7/b${u}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r5w7/b${u}_$rep.json').read().strip().splitlines()[-1]); rc=d.get('reference_check') or {}; print('union $u', d['value'], 'rounds', d.get('rounds'), 'it', d.get('iterations'), 'gram', d.get('gram_gemm_s'), 'conv', d.get('converged'), {k: rc.get(k) for k in ('sign_agreement','abs_db','decision_agreement','db')})"
  done
done
