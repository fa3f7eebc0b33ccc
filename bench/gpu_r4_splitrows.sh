# single-pass split_rows_kernel: split / ws suites, headline (trajectory must not move), kernel time
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_split_gemm_gpu.py tests/test_ws_gpu.py tests/test_kernels_gpu.py > gpurun_out/r4sr_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4sr_pytest.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/r4sr_pytest.log; exit $rc; }
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/r4sr_headline.json > /dev/null 2> gpurun_out/r4sr_headline.err || exit 1
python3 -c "
import json
d=json.loads(open('gpurun_out/r4sr_headline.json').read())
print('headline', d['value'], 'gram', d['gram_gemm_s'], 'rounds', d['rounds'], 'b', d['b'])"
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4sr_prof -o h --output-format csv -- python3 -u $R/bench.py --steps 2 --warmup 0 --reference-check off --no-accuracy --json-out $R/gpurun_out/r4sr_prof.json > $R/gpurun_out/r4sr_prof.log 2>&1 || exit 1
cd $R && python3 -c "
import csv,glob
f=glob.glob('gpurun_out/r4sr_prof/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'split_rows' in r['Name'] or 'w64' in r['Name']: print(r['Name'][:60], r['Calls'], 'avg us', round(float(r['AverageNs'])/1e3,1))"
