# auto block count from the kernel's coupling: uncoupled (headline) -> 64 x 48, coupled -> 32 x 96
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/r5k_ab.txt
for k in 1 2; do
  for env in auto 32; do
    for cfg in mnist mnist-parity mnist-makefile; do
      if [ $env = auto ]; then E=""; else E="DPSVM_WS_AUTO_BLOCKS=$env"; fi
      env $E timeout -k 10 300 python3 -u bench.py --config $cfg --steps 10 --warmup 3 --secondary off --json-out gpurun_out/r5k_b.json > gpurun_out/r5k_b.log 2>&1 || { tail -5 gpurun_out/r5k_b.log; exit 1; }
      python3 -c "
import json; d=json.load(open('gpurun_out/r5k_b.json')); rc=d.get('reference_check') or {}
print('blocks=$env', '$cfg', d['value'], 'start', d['ws_blocks']['start'], 'rounds', d['rounds'], 'conv', d['converged'], 'agree', rc.get('decision_sign_agreement'), 'db', rc.get('abs_b_diff'))" >> gpurun_out/r5k_ab.txt
    done
  done
done
cat gpurun_out/r5k_ab.txt
