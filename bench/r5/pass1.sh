# wide pass 1 (DPSVM_PASS1=v4: 1024-column groups, 16-B row loads) vs the selection-geometry pass 1 (v1)
set -o pipefail
mkdir -p gpurun_out
for V in v1 v4 v1 v4; do
  DPSVM_PASS1=$V timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --reference-check off --no-accuracy --json-out gpurun_out/r5p1_$V.json > gpurun_out/r5p1_$V.log 2>&1 || { tail -20 gpurun_out/r5p1_$V.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5p1_$V.json')); print('$V', d['value'], d['gram_gemm_s'], d['rounds'], d['iterations'], d['converged'], d['b'])" | tee -a gpurun_out/r5p1_summary.txt
done
DPSVM_PASS1=v4 timeout -k 10 300 python3 -u bench/ws_stamps.py --out gpurun_out/r5p1_stamps_v4.json > /dev/null 2> gpurun_out/r5p1_stamps_v4.err || exit 1
DPSVM_PASS1=v1 timeout -k 10 300 python3 -u bench/ws_stamps.py --out gpurun_out/r5p1_stamps_v1.json > /dev/null 2> gpurun_out/r5p1_stamps_v1.err || exit 1
python3 -c "
import json
for v in ('v1','v4'):
    d=json.load(open(f'gpurun_out/r5p1_stamps_{v}.json')); print(v, d['round_period_us'], d.get('merge_phases_us'), {k: d[k] for k in d if 'us' in k and not isinstance(d[k], dict)})" | tee -a gpurun_out/r5p1_summary.txt
