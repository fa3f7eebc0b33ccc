# rocprofv3 kernel stats of the final headline (bench.py --steps 3 --warmup 1)
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4k_prof -o headline --output-format csv -- python3 -u $R/bench.py --steps 3 --warmup 1 --json-out $R/gpurun_out/r4k_bench.json > $R/gpurun_out/r4k_prof.log 2>&1
rc=$?; cd $R; ls gpurun_out/r4k_prof; exit $rc
