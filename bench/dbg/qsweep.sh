set -o pipefail
for Q in 128 160 192; do
  timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --reference-check off --no-accuracy --ws-blocks 8 --ws-size $Q > gpurun_out/q.log 2>&1 || { echo "Q=$Q failed"; tail -5 gpurun_out/q.log; exit 1; }
  grep '^{' gpurun_out/q.log | tail -1 | python3 -c "import json,sys
d=json.loads(sys.stdin.read()); print('q=$Q', d['value'], 'steps', d['iterations'], 'rounds', d['rounds'], d['converged'])" | tee -a gpurun_out/qsweep.txt
done
