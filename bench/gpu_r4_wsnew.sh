# rows replaced per one-block round (ws_new, default 3/4 of ws_size): full
# replacement on the one-block problems with >= 128 features (mnist-parity
# after its fallback to one block, adult with solver=ws)
set -o pipefail
mkdir -p gpurun_out
B="python3 -u bench.py --no-accuracy --reference-check off"
for cfg in "mnist-parity" "adult --solver ws"; do
  tag=$(echo $cfg | cut -d' ' -f1)
  timeout -k 10 200 $B --steps 3 --warmup 1 --config $cfg --ws-new 192 --json-out gpurun_out/r4n_${tag}_new192.json > /dev/null 2> gpurun_out/r4n_${tag}_new192.err || exit $?
  timeout -k 10 200 $B --steps 3 --warmup 1 --config $cfg --json-out gpurun_out/r4n_${tag}_def.json > /dev/null 2> gpurun_out/r4n_${tag}_def.err || exit $?
done
for f in mnist-parity_new192 mnist-parity_def adult_new192 adult_def; do python3 -c "
import json
d=json.loads(open('gpurun_out/r4n_$f.json').read())
print('$f', d['value'], 'rounds', d['rounds'], 'iters', d['iterations'], 'conv', d['converged'], 'b', d['b'], d['ws_blocks'])
"; done
