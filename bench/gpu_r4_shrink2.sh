# shrinking with the whole-problem solver set up untimed (ShrinkingSolver):
# covtype box + synthetic-2m under the defaults, a sub-problem tolerance A/B
# on covtype box, then the 8-GPU plan inputs (bench/gpu_r4_big.sh)
set -o pipefail
mkdir -p gpurun_out
B="python3 -u bench.py --no-accuracy --reference-check off"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ws_gpu.py tests/test_cli.py -k "shrink" > gpurun_out/r4s2_pytest.log 2>&1 &&
timeout -k 10 300 $B --config covtype --clip box --max-iter 60000000 --steps 1 --warmup 0 --log-every 5000000 --verbose > gpurun_out/r4s2_covbox_auto.json 2> gpurun_out/r4s2_covbox_auto.err &&
timeout -k 10 300 $B --config covtype --clip box --max-iter 60000000 --ws-rel 0.1 --steps 1 --warmup 0 --log-every 5000000 --verbose > gpurun_out/r4s2_covbox_rel01.json 2> gpurun_out/r4s2_covbox_rel01.err &&
timeout -k 10 400 $B --config synthetic-2m --steps 1 --warmup 0 --log-every 1000000 --verbose > gpurun_out/r4s2_syn2m_auto.json 2> gpurun_out/r4s2_syn2m_auto.err
rc=$?
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r4s2_*.json")):
    try:
        d=json.loads(open(f).read().strip().split("\n")[-1])
    except Exception as e:
        print(f, "unreadable", e); continue
    print(f, d["value"], "rounds", d.get("rounds"), "iters", d.get("iterations"), "conv", d.get("converged"),
          "gap", d.get("final_gap"), "b", d.get("b"), "nsv", d.get("n_sv"), d.get("iteration"), d.get("shrink"))
PY
grep -h "shrink phase" gpurun_out/r4s2_*.err
tail -3 gpurun_out/r4s2_pytest.log
[ $rc -eq 0 ] && bash bench/gpu_r4_big.sh
