# shrink=auto (library / CLI / bench default) on the big configs, 1 MI355X:
# headline unchanged (auto keeps the resident-Gram path), covtype box to
# convergence, covtype-ref (Makefile:77, 500k rows, the reference's 3M cap),
# synthetic-2m; auto vs off A/B on the same box
set -o pipefail
mkdir -p gpurun_out
B="python3 -u bench.py --no-accuracy --reference-check off"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ws_gpu.py tests/test_cli.py -k "small_cache or production_engines or shrink" > gpurun_out/r4sh_pytest.log 2>&1 &&
timeout -k 10 300 $B --steps 3 --warmup 1 > gpurun_out/r4sh_headline.json 2> gpurun_out/r4sh_headline.err &&
timeout -k 10 300 $B --config covtype --clip box --max-iter 60000000 --steps 1 --warmup 0 --log-every 5000000 --verbose > gpurun_out/r4sh_covbox_auto.json 2> gpurun_out/r4sh_covbox_auto.err &&
timeout -k 10 300 $B --config covtype --clip box --max-iter 60000000 --shrink off --steps 1 --warmup 0 --log-every 5000000 > gpurun_out/r4sh_covbox_off.json 2> gpurun_out/r4sh_covbox_off.err &&
timeout -k 10 200 $B --config covtype-ref --steps 1 --warmup 0 --log-every 5000000 --verbose > gpurun_out/r4sh_covref_auto.json 2> gpurun_out/r4sh_covref_auto.err &&
timeout -k 10 200 $B --config covtype-ref --shrink off --steps 1 --warmup 0 --log-every 5000000 > gpurun_out/r4sh_covref_off.json 2> gpurun_out/r4sh_covref_off.err &&
timeout -k 10 400 $B --config synthetic-2m --steps 1 --warmup 0 --log-every 1000000 --verbose > gpurun_out/r4sh_syn2m_auto.json 2> gpurun_out/r4sh_syn2m_auto.err &&
timeout -k 10 400 $B --config synthetic-2m --shrink off --steps 1 --warmup 0 --log-every 1000000 > gpurun_out/r4sh_syn2m_off.json 2> gpurun_out/r4sh_syn2m_off.err
rc=$?
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r4sh_*.json")):
    try:
        d=json.loads(open(f).read().strip().split("\n")[-1])
    except Exception as e:
        print(f, "unreadable", e); continue
    print(f, d["value"], "rounds", d.get("rounds"), "iters", d.get("iterations"), "conv", d.get("converged"),
          "gap", d.get("final_gap"), "b", d.get("b"), "nsv", d.get("n_sv"), d.get("iteration"), d.get("shrink"))
PY
grep -h "shrink phase" gpurun_out/r4sh_*.err
tail -3 gpurun_out/r4sh_pytest.log
exit $rc
