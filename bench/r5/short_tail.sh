# single-round launches once the stop test is predicted within the launch in flight (DPSVM_SHORT_TAIL=0: full
# 8-round graph launches to the end): ws + solver tests, headline / parity / makefile benches alternating,
# kernel-trace tail of the headline
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5st2
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_ws_gpu.py tests/test_solver_gpu.py \
  > gpurun_out/r5st2/pytest.log 2>&1 || { tail -40 gpurun_out/r5st2/pytest.log; exit 1; }
tail -1 gpurun_out/r5st2/pytest.log
for rep in 1 2; do
  for t in 1 0; do
    DPSVM_SHORT_TAIL=$t timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 3 > gpurun_out/r5st2/b${t}_$rep.json 2> gpurun_out/r5st2/b${t}_$rep.err || { tail -5 gpurun_out/r5st2/b${t}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r5st2/b${t}_$rep.json').read().strip().splitlines()[-1]); rc=d['reference_check']; s=d.get('secondary') or {}; print('short_tail $t', d['value'], 'rounds', d['rounds'], 'it', d['iterations'], 'gram', d['gram_gemm_s'], 'b', d['b'], rc['decision_sign_agreement'], 'parity', s.get('value'), s.get('rounds'), s.get('b'))"
  done
done
for t in 1 0; do
  DPSVM_SHORT_TAIL=$t timeout -k 10 240 python3 -u bench.py --config mnist-makefile --steps 5 --warmup 2 > gpurun_out/r5st2/m${t}.json 2> gpurun_out/r5st2/m${t}.err || { tail -5 gpurun_out/r5st2/m${t}.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r5st2/m${t}.json').read().strip().splitlines()[-1]); print('makefile short_tail $t', d['value'], 'rounds', d['rounds'], 'b', d['b'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5st2/tl -o run -- python3 -u bench.py --steps 3 --warmup 1 --reference-check off --secondary off --no-accuracy > gpurun_out/r5st2/tl_out.txt 2> gpurun_out/r5st2/tl_err.txt || { tail -5 gpurun_out/r5st2/tl_err.txt; exit 1; }
echo done
