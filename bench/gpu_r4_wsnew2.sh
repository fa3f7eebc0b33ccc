# ws_new auto (full replacement from 128 padded features): ws tests, presets
set -o pipefail
mkdir -p gpurun_out
B="python3 -u bench.py --no-accuracy --reference-check off"
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ws_gpu.py tests/test_cli.py > gpurun_out/r4m_pytest.log 2>&1 &&
timeout -k 10 200 $B --steps 5 --warmup 1 --json-out gpurun_out/r4m_headline.json > /dev/null 2> gpurun_out/r4m_headline.err &&
timeout -k 10 200 $B --steps 5 --warmup 1 --config mnist-parity --json-out gpurun_out/r4m_parity.json > /dev/null 2> gpurun_out/r4m_parity.err &&
timeout -k 10 400 $B --steps 1 --warmup 0 --config synthetic-2m --log-every 1000000 --json-out gpurun_out/r4m_syn2m.json > /dev/null 2> gpurun_out/r4m_syn2m.err
rc=$?
tail -2 gpurun_out/r4m_pytest.log
for f in headline parity syn2m; do python3 -c "
import json
d=json.loads(open('gpurun_out/r4m_$f.json').read())
print('$f', d['value'], 'rounds', d['rounds'], 'iters', d['iterations'], 'conv', d['converged'], 'b', d['b'], d['shrink']['phase_log'])
" 2>/dev/null; done
exit $rc
