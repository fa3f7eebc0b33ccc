# wide pass 1 with 2048-column workgroups (two partitions of 512 threads: 8-KiB row pieces) vs 1024 (default):
# pass-1 probe at the headline shape, then bench.py alternating (DPSVM_P1_COLS)
set -o pipefail
mkdir -p gpurun_out/r5pc
for c in 1024 2048; do
  DPSVM_P1_COLS=$c timeout -k 10 400 python3 -u bench/pass1_probe.py --cols 60000 --changed 6144 --ks 4,6,8,12 --wide --reps 12 > gpurun_out/r5pc/probe_$c.jsonl 2> gpurun_out/r5pc/probe_$c.err || { tail -3 gpurun_out/r5pc/probe_$c.err; exit 1; }
  echo "cols $c"; cat gpurun_out/r5pc/probe_$c.jsonl | cut -c1-220
done
for rep in 1 2; do
  for c in 2048 1024; do
    DPSVM_P1_COLS=$c timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 3 --secondary off > gpurun_out/r5pc/b${c}_$rep.json 2> gpurun_out/r5pc/b${c}_$rep.err || { tail -5 gpurun_out/r5pc/b${c}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r5pc/b${c}_$rep.json').read().strip().splitlines()[-1]); rc=d['reference_check']; print('cols $c', d['value'], 'rounds', d['rounds'], 'it', d['iterations'], 'gram', d['gram_gemm_s'], 'b', d['b'], 'conv', d['converged'], rc['decision_sign_agreement'])"
  done
done
