# model-level agreement of two trajectories on the big configs (held-out rows of the same generator)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u bench/parity_big.py --config covtype-box --alt '{"shrink": "off"}' --out gpurun_out/r5q_parity_big.jsonl > gpurun_out/r5q_cov.log 2>&1 || { tail -20 gpurun_out/r5q_cov.log; exit 1; }
grep "^\[parity\]" gpurun_out/r5q_cov.log | cut -c1-400
timeout -k 10 900 python3 -u bench/parity_big.py --config covtype-box --alt '{"ws_block": 32}' --out gpurun_out/r5q_parity_big.jsonl > gpurun_out/r5q_cov32.log 2>&1 || { tail -20 gpurun_out/r5q_cov32.log; exit 1; }
grep "^\[parity\]" gpurun_out/r5q_cov32.log | cut -c1-400
timeout -k 10 900 python3 -u bench/parity_big.py --config synthetic-2m --alt '{"shrink": "off"}' --out gpurun_out/r5q_parity_big.jsonl > gpurun_out/r5q_s2m.log 2>&1 || { tail -20 gpurun_out/r5q_s2m.log; exit 1; }
grep "^\[parity\]" gpurun_out/r5q_s2m.log | cut -c1-400
python3 -c "
import json
for l in open('gpurun_out/r5q_parity_big.jsonl'):
    d=json.loads(l); print(d['config'], d['alt']['knobs'], 'agree', d['decision_sign_agreement'], 'db', d['abs_b_diff'], 'acc', d['base']['holdout_accuracy'], d['alt']['holdout_accuracy'], 'nsv', d['base']['n_sv'], d['alt']['n_sv'], 'svdiff', d['sv_set_symmetric_diff'], 't', d['base']['fit_time_s'], d['alt']['fit_time_s'])"
