# ws_block 32 (default) vs 8 on the other presets: mnist-parity, mnist-makefile, adult, covtype box (full), synthetic-2m
set -o pipefail
mkdir -p gpurun_out
run() {  # tag wb args...
  local tag=$1 wb=$2; shift 2
  timeout -k 10 400 python3 -u bench.py --ws-block $wb "$@" --json-out gpurun_out/r4wb2_${tag}_$wb.json > /dev/null 2> gpurun_out/r4wb2_${tag}_$wb.err || return 1
  python3 -c "
import json
d=json.loads(open('gpurun_out/r4wb2_${tag}_$wb.json').read())
print('$tag ws_block=$wb', d['value'], 'rounds', d.get('rounds'), 'iters', d.get('iterations'), 'conv', d.get('converged'), 'b', d['b'])
" | tee -a gpurun_out/r4wb2_summary.txt
}
for wb in 32 8; do run parity $wb --config mnist-parity --steps 5 --warmup 1 || exit 1; done
for wb in 32 8; do run makefile $wb --config mnist-makefile --steps 5 --warmup 1 || exit 1; done
for wb in 32 8; do run adult $wb --config adult --steps 3 --warmup 1 --no-accuracy || exit 1; done
for wb in 32 8; do run covbox $wb --config covtype --clip box --max-iter 60000000 --steps 1 --warmup 0 --no-accuracy --reference-check off || exit 1; done
for wb in 32 8; do run syn2m $wb --config synthetic-2m --steps 1 --warmup 0 --no-accuracy --reference-check off || exit 1; done
