# inputs of the 8-GPU plan for covtype / synthetic-2m (one MI355X): round
# anatomy by in-kernel stamps at the full shapes (local and loopback peer
# exchange), one rank's dense Gram slab at covtype P = 8
set -o pipefail
mkdir -p gpurun_out
S="python3 -u bench/ws_stamps.py"
COV="--data covtype --samples 581012 --features 54 --C 2048 --gamma 0.03125 --clip box --max-iter 2000000"
timeout -k 10 200 $S $COV --out gpurun_out/r4b_stamps_covbox.json > /dev/null 2> gpurun_out/r4b_stamps_covbox.err &&
timeout -k 10 200 $S $COV --exchange peer --out gpurun_out/r4b_stamps_covbox_peer.json > /dev/null 2> gpurun_out/r4b_stamps_covbox_peer.err &&
timeout -k 10 300 $S --data uniform --samples 2000000 --features 1024 --C 1 --gamma 0.0009765625 --max-iter 150000 --out gpurun_out/r4b_stamps_syn2m.json > /dev/null 2> gpurun_out/r4b_stamps_syn2m.err &&
timeout -k 10 200 python3 -u bench/slab_probe.py --P 8 --out gpurun_out/r4b_slab_cov.json > gpurun_out/r4b_slab_cov.log 2>&1
rc=$?
cat gpurun_out/r4b_*.json
exit $rc
