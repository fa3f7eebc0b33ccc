set -o pipefail
for I in 96 128 192 0; do
  timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --reference-check off --no-accuracy --ws-inner $I > gpurun_out/i.log 2>&1 || { echo "I=$I failed"; tail -5 gpurun_out/i.log; exit 1; }
  grep '^{' gpurun_out/i.log | tail -1 | python3 -c "import json,sys
d=json.loads(sys.stdin.read()); print('inner=$I', d['value'], 'steps', d['iterations'], 'rounds', d['rounds'], d['converged'])" | tee -a gpurun_out/isweep.txt
done
