set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_ws_gpu.py -k "peer" > gpurun_out/r4m_pytest_peer.log 2>&1 &&
timeout -k 10 400 python3 bench/shard_projection.py --out gpurun_out/r4m_shard_inputs.json > gpurun_out/r4m_shard_inputs.log 2>&1 &&
DPSVM_FORCE_DEVICE=0 timeout -k 10 400 python3 bench.py --gpus 2 --dp shard --steps 5 --warmup 1 > gpurun_out/r4m_shard2.json 2> gpurun_out/r4m_shard2.err &&
DPSVM_FORCE_DEVICE=0 timeout -k 10 400 python3 bench.py --gpus 4 --dp shard --steps 5 --warmup 1 > gpurun_out/r4m_shard4.json 2> gpurun_out/r4m_shard4.err &&
DPSVM_FORCE_DEVICE=0 timeout -k 10 400 python3 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/r4m_auto2.json 2> gpurun_out/r4m_auto2.err
rc=$?
tail -2 gpurun_out/r4m_pytest_peer.log
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r4m_*.json")):
    try:
        d=json.loads(open(f).read().strip().split("\n")[-1])
    except Exception as e:
        print(f, "unreadable", e); continue
    if "value" in d:
        print(f, d["value"], d["n_gpus"], d.get("exchange"), d.get("dp_policy"), d.get("rounds"), d.get("iterations"), d.get("shard_check"), d.get("dp_autotune"))
    else:
        print(f, {k: d[k] for k in ("local","peer_loopback","rccl_one_rank") if k in d})
PY
exit $rc
