#!/bin/bash
# 1/2/4/8-GPU strong-scaling sweep on one MI355X node (one process per GPU,
# torch.distributed bootstrap, RCCL over xGMI for the per-iteration keys).
# Usage: bench/run_scaling.sh [config] [steps] [warmup]     (config: bench.py --config)
# Replaces the reference's `mpirun -np P --hostfile hf` recipes (Makefile:74-86, hf).
set -o pipefail
cd "$(dirname "$0")/.."
CFG=${1:-mnist}; STEPS=${2:-3}; WARM=${3:-1}
OUT=${OUT:-gpurun_out/scaling_${CFG}.jsonl}
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
NGPU=$(python3 -c "import torch;print(torch.cuda.device_count())")
PORT=$((29500 + RANDOM % 1000))
for N in 1 2 4 8; do
  [ "$N" -le "$NGPU" ] || break
  if [ "$N" -eq 1 ]; then
    timeout -k 10 1800 python3 bench.py --config "$CFG" --gpus 1 --steps "$STEPS" --warmup "$WARM" | tail -1 >> "$OUT" || exit $?
  else
    timeout -k 10 1800 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
      --master-port $((PORT + N)) bench.py --config "$CFG" --gpus "$N" --steps "$STEPS" --warmup "$WARM" \
      | grep '^{' | tail -1 >> "$OUT" || exit $?
  fi
  tail -1 "$OUT"
done
python3 - "$OUT" <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.strip()]
t1 = next((r["value"] for r in rows if r["n_gpus"] == 1), None)
for r in rows:
    eff = (t1 / (r["n_gpus"] * r["value"])) if t1 else float("nan")
    print(f"N={r['n_gpus']}  {r['value']:.4f} s  iters={r['iterations']}  strong-scaling eff={eff:.2f}")
PY
