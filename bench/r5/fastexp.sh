# (historical: the A/B switch / code this script exercised was removed after its measurement; see profiles/)
# recompute rounds: libm expf (the Gram's bits) vs the hardware exp, covtype 581k x 54 one block, 1M pair steps
set -o pipefail
mkdir -p gpurun_out
for E in libm fast; do
  DPSVM_RECOMPUTE_EXP=$E timeout -k 10 400 python3 -u bench/ws_stamps.py --data covtype --samples 581012 --features 54 --C 2048 --gamma 0.03125 --clip box --ws-blocks 1 --max-iter 1000000 --out gpurun_out/r5e_$E.json > /dev/null 2> gpurun_out/r5e_$E.err || { tail -5 gpurun_out/r5e_$E.err; exit 1; }
  echo "$E $(cat gpurun_out/r5e_$E.json)"
done
