# 8-rank one-GPU rehearsal with 2 hardware queues per process + stamps; then 2 / 4 again for the table
set -o pipefail
mkdir -p gpurun_out
for N in 8 4 2; do
  rm -f /tmp/st$N.rank*
  DPSVM_STAMPS=/tmp/st$N DPSVM_FORCE_DEVICE=0 timeout -k 10 400 python3 -u bench.py --gpus $N --dp shard --steps 3 --warmup 1 --no-accuracy --reference-check off --json-out gpurun_out/r5r_mp$N.json > gpurun_out/r5r_mp$N.log 2>&1 || { tail -20 gpurun_out/r5r_mp$N.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5r_mp$N.json')); print('$N ranks', d['value'], d['ws_exchange'], repr(d['engine_note']), d['config']['parallelism'], d['rounds'], d['converged'], d['b'])"
  python3 bench/shard_stamps.py /tmp/st$N $N --out gpurun_out/r5r_stamps_mp$N.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($N, d['exchange_consumer_us_per_round'], d['median_over_ranks'])"
done
python3 bench/project_shard.py gpurun_out/r5r_projection_inputs.json --rehearsal 2:gpurun_out/r5r_stamps_mp2.json --rehearsal 4:gpurun_out/r5r_stamps_mp4.json --rehearsal 8:gpurun_out/r5r_stamps_mp8.json > gpurun_out/r5r_projection.txt; tail -6 gpurun_out/r5r_projection.txt
