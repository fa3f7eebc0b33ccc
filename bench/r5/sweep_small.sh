# small coupled problems: ws_rel / ws_new / ws_inner sweep (covtype-shape 7.5k and 20k rows)
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/r5s_sweep_small.jsonl
timeout -k 10 400 python3 -u bench/ws_sweep_small.py --n 7500 --rel 0.1,0.2,0.3,0.5,0.7 --new 96,144,192 --out gpurun_out/r5s_sweep_small.jsonl > gpurun_out/r5s_sweep_small.log 2>&1 || { tail -5 gpurun_out/r5s_sweep_small.log; exit 1; }
timeout -k 10 400 python3 -u bench/ws_sweep_small.py --n 7500 --rel 0.3 --new 144 --inner 100,200,2000 --out gpurun_out/r5s_sweep_small.jsonl >> gpurun_out/r5s_sweep_small.log 2>&1 || { tail -5 gpurun_out/r5s_sweep_small.log; exit 1; }
timeout -k 10 500 python3 -u bench/ws_sweep_small.py --n 20000 --rel 0.1,0.3,0.5 --new 144,192 --out gpurun_out/r5s_sweep_small.jsonl >> gpurun_out/r5s_sweep_small.log 2>&1 || { tail -5 gpurun_out/r5s_sweep_small.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r5s_sweep_small.jsonl'):
    d=json.loads(l); print(d['n'], d['rel'], d['new'], d['inner'], d['fit_s'], d['rounds'], d['steps'], round(d['b'],4), d['converged'])"
