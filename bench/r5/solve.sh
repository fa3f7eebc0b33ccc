# ws_solve with register-resident alphas: full GPU suite (bit-identity tests), pair-step stamps
set -o pipefail
mkdir -p gpurun_out
bash bench/r5/suite.sh || exit $?
timeout -k 10 300 python3 -u bench/ws_stamps.py --data covtype --samples 7500 --features 54 --C 2048 --gamma 0.03125 --clip box --ws-blocks 1 --out gpurun_out/r5v_stamps_cov7500.json > /dev/null 2> gpurun_out/r5v_stamps_cov7500.err || exit 1
timeout -k 10 300 python3 -u bench/ws_stamps.py --out gpurun_out/r5v_stamps_headline.json > /dev/null 2> gpurun_out/r5v_stamps_headline.err || exit 1
python3 -c "
import json
for k in ('cov7500','headline'):
    d=json.load(open(f'gpurun_out/r5v_stamps_{k}.json')); print(k, d['rounds'], d['pair_steps'], d['fit_time_s'], d['solve_per_step_us'], d['solve_us'], d['round_period_us'], d['b'])"
