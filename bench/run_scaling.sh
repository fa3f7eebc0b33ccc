#!/bin/bash
# 1/2/4/8-GPU strong-scaling sweep on one MI355X node. `bench.py --gpus N`
# starts its N ranks itself (one process per GPU over torch.distributed.run,
# 127.0.0.1 rendezvous, RCCL over xGMI) and fails non-zero unless N ranks ran.
# Usage: bench/run_scaling.sh [config] [steps] [warmup]     (config: bench.py --config)
# Replaces the reference's `mpirun -np P --hostfile hf` recipes (Makefile:74-86, hf).
set -o pipefail
cd "$(dirname "$0")/.."
CFG=${1:-mnist}; STEPS=${2:-3}; WARM=${3:-1}
OUT=${OUT:-gpurun_out/scaling_${CFG}.jsonl}
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
NGPU=$(python3 -c "import torch;print(torch.cuda.device_count())")
for N in 1 2 4 8; do
  [ "$N" -le "$NGPU" ] || break
  timeout -k 10 1800 python3 bench.py --config "$CFG" --gpus "$N" --steps "$STEPS" --warmup "$WARM" \
    | grep '^{' | tail -1 >> "$OUT" || exit $?
  tail -1 "$OUT"
done
python3 - "$OUT" <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.strip()]
t1 = next((r["value"] for r in rows if r["n_gpus"] == 1), None)
for r in rows:
    eff = (t1 / (r["n_gpus"] * r["value"])) if t1 else float("nan")
    print(f"N={r['n_gpus']}  {r['value']:.4f} s  iters={r['iterations']}  dp={r.get('dp_policy')}  "
          f"strong-scaling eff={eff:.2f}")
PY
