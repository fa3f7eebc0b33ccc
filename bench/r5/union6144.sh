# 6,144-row unions (128 blocks of 48) for uncoupled ws-dense rounds vs 3,072 (64 x 48): kernel tests, then
# bench.py alternating (DPSVM_WS_UNION=3072 forces the old union)
set -o pipefail
mkdir -p gpurun_out/r5w6
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ws_kernels_gpu.py \
  > gpurun_out/r5w6/pytest_kernels.log 2>&1 || { tail -30 gpurun_out/r5w6/pytest_kernels.log; exit 1; }
tail -2 gpurun_out/r5w6/pytest_kernels.log
for rep in 1 2; do
  for u in 6144 3072; do
    DPSVM_WS_UNION=$u timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 3 --secondary off \
      > gpurun_out/r5w6/b${u}_$rep.json 2> gpurun_out/r5w6/b${u}_$rep.err || { tail -5 gpurun_out/r5w6/b${u}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r5w6/b${u}_$rep.json').read().strip().splitlines()[-1]); print('union $u', d['value'], 'rounds', d.get('rounds'), 'it', d.get('iterations'), 'gram', d.get('gram_gemm_s'), 'conv', d.get('converged'), 'agree', (d.get('reference_check') or {}).get('sign_agreement'), 'db', (d.get('reference_check') or {}).get('abs_db'))"
  done
done
