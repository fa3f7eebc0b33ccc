# PMC of the headline's round kernels (final tree): bytes fetched from HBM / MALL per kernel (TCC FETCH_SIZE; a pass of
# its own), bench.py --steps 1 --warmup 0
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5pmc
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/r5pmc/f -o run -- python3 -u bench.py --steps 1 --warmup 0 --reference-check off --secondary off --no-accuracy > gpurun_out/r5pmc/out.txt 2> gpurun_out/r5pmc/err.txt || { tail -5 gpurun_out/r5pmc/err.txt; exit 1; }
ls gpurun_out/r5pmc/f
