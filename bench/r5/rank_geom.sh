# rank kernel: 16 keys per workgroup (512 workgroups, 32 threads a key) instead of 32 (256, 16 a key): ws kernel
# tests, timeline, bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5rg
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ws_kernels_gpu.py \
  > gpurun_out/r5rg/pytest.log 2>&1 || { tail -30 gpurun_out/r5rg/pytest.log; exit 1; }
tail -1 gpurun_out/r5rg/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5rg/tl -o run -- python3 -u bench.py --steps 3 --warmup 1 --reference-check off --secondary off --no-accuracy > gpurun_out/r5rg/tl_out.txt 2> gpurun_out/r5rg/tl_err.txt || { tail -5 gpurun_out/r5rg/tl_err.txt; exit 1; }
python3 bench/timeline_gaps.py gpurun_out/r5rg/tl | tail -9
for rep in 1 2; do
  timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 3 --secondary off > gpurun_out/r5rg/b_$rep.json 2> gpurun_out/r5rg/b_$rep.err || { tail -5 gpurun_out/r5rg/b_$rep.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r5rg/b_$rep.json').read().strip().splitlines()[-1]); print('bench', d['value'], 'rounds', d['rounds'], 'it', d['iterations'], 'gram', d['gram_gemm_s'], 'b', d['b'])"
done
