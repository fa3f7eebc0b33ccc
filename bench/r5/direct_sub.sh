# multi-block solve loading its <= 64-row block (upper triangle, mirrored in LDS) from the resident Gram vs the
# gather kernel (DPSVM_WS_DIRECT_SUB=0): ws tests, then bench.py alternating, then stamps
set -o pipefail
mkdir -p gpurun_out/r5ds2
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ws_kernels_gpu.py tests/test_ws_gpu.py \
  > gpurun_out/r5ds2/pytest.log 2>&1 || { tail -40 gpurun_out/r5ds2/pytest.log; exit 1; }
tail -1 gpurun_out/r5ds2/pytest.log
for rep in 1 2; do
  for d in 1 0; do
    DPSVM_WS_DIRECT_SUB=$d timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 3 --secondary off > gpurun_out/r5ds2/b${d}_$rep.json 2> gpurun_out/r5ds2/b${d}_$rep.err || { tail -5 gpurun_out/r5ds2/b${d}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r5ds2/b${d}_$rep.json').read().strip().splitlines()[-1]); rc=d['reference_check']; print('direct $d', d['value'], 'rounds', d['rounds'], 'it', d['iterations'], 'gram', d['gram_gemm_s'], 'b', d['b'], 'conv', d['converged'], rc['decision_sign_agreement'])"
  done
done
timeout -k 10 300 python3 -u bench/ws_stamps.py --out gpurun_out/r5ds2/stamps.json > gpurun_out/r5ds2/stamps.txt 2>&1 || { tail -5 gpurun_out/r5ds2/stamps.txt; exit 1; }
tail -1 gpurun_out/r5ds2/stamps.txt
