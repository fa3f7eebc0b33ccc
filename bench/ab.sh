#!/bin/bash
# A/B runner: one bench.py run per line of a spec file, "label | bench.py args"
# or "label | bench.py args | VAR=value ..." (DPSVM_* A/B switches for that run),
# each under its own time limit; a one-line digest per run goes to
# gpurun_out/ab_$TAG.txt (full JSON lines to gpurun_out/ab_$TAG.jsonl).
# Stops at the first failing run.
#   bench/ab.sh SPEC_FILE          (LIMIT: seconds per run, default 300)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-ab}
LIMIT=${LIMIT:-300}
SPEC=$1
out=gpurun_out/ab_$TAG.txt
: > "$out"
: > "gpurun_out/ab_$TAG.jsonl"
while IFS='|' read -r label args envs; do
  label=$(echo "$label" | xargs)
  [ -z "$label" ] && continue
  case "$label" in \#*) continue ;; esac
  log="gpurun_out/ab_${TAG}_${label}.log"
  # shellcheck disable=SC2086
  timeout -k 10 "$LIMIT" env $envs python -u bench.py $args > "$log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "$label FAILED rc=$rc" | tee -a "$out"
    tail -20 "$log"
    exit $rc
  fi
  grep '^{' "$log" | tail -1 >> "gpurun_out/ab_$TAG.jsonl"
  grep '^{' "$log" | tail -1 | LABEL="$label" python3 -c "import json,os,sys
d=json.loads(sys.stdin.read()); r=d.get('reference_check') or {}; w=d.get('ws_blocks') or {}
print(os.environ['LABEL'], d['value'], 's steps', d['iterations'], 'rounds', d['rounds'], 'conv', d['converged'],
      'gap', round(d['final_gap'] or 0, 6), 'b', round(d['b'], 6), 'nsv', d['n_sv'], 'acc', d['train_accuracy'],
      'P', w.get('start'), '->', w.get('end'), 'P1@', w.get('one_block_from_round'), 'damped', w.get('damped_rounds'),
      'gram', d.get('gram_gemm_s'), 'ref|db|', r.get('abs_b_diff'), 'agree', r.get('decision_sign_agreement'),
      d.get('iteration'), d.get('engine_note'))" | tee -a "$out"
done < "$SPEC"
