# final-tree validation: full GPU suite, smoke, headline bench (default flags), kernel-trace timeline of the headline,
# covtype box end to end
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5f4
timeout -k 10 1000 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r5f4/pytest.log 2>&1
rc=$?; tail -1 gpurun_out/r5f4/pytest.log; grep -E "FAILED|ERROR" gpurun_out/r5f4/pytest.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5f4/smoke.log 2>&1 || { tail -5 gpurun_out/r5f4/smoke.log; exit 1; }
tail -1 gpurun_out/r5f4/smoke.log
timeout -k 10 300 python3 -u bench.py > gpurun_out/r5f4/bench_default.json 2> gpurun_out/r5f4/bench_default.err || { tail -5 gpurun_out/r5f4/bench_default.err; exit 1; }
tail -1 gpurun_out/r5f4/bench_default.json | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5f4/tl -o run -- python3 -u bench.py --steps 3 --warmup 1 --reference-check off --secondary off --no-accuracy > gpurun_out/r5f4/tl_out.txt 2> gpurun_out/r5f4/tl_err.txt || { tail -5 gpurun_out/r5f4/tl_err.txt; exit 1; }
python3 bench/timeline_gaps.py gpurun_out/r5f4/tl > gpurun_out/r5f4/timeline.txt && tail -12 gpurun_out/r5f4/timeline.txt
C="python3 -u bench.py --no-accuracy --reference-check off --steps 1 --warmup 0 --config covtype --clip box --max-iter 60000000 --log-every 5000000"
timeout -k 10 300 $C --json-out gpurun_out/r5f4/covbox.json > gpurun_out/r5f4/covbox.log 2>&1 || { tail -5 gpurun_out/r5f4/covbox.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r5f4/covbox.json')); print('covbox', d['value'], d['rounds'], d['iterations'], d['b'], d['converged'], d['n_sv'], d['shrink']['phase_log'])"
