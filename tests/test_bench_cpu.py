"""bench.py contract (JSON line) on the CPU path with a small problem."""
import json
import os
import sys

from conftest import ROOT, run


def test_bench_json_contract():
    r = run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--samples", "1500",
             "--steps", "1", "--warmup", "0"])
    assert r.returncode == 0, r.stderr
    line = [l for l in r.stdout.strip().split("\n") if l.startswith("{")][-1]
    out = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in out
    assert out["higher_is_better"] is False and out["scaling"] == "strong" and out["n_gpus"] == 1
    assert out["converged"] and out["config"]["parallelism"] == "dp1"
    # a reduced problem is not the reference's published config: no baseline ratio
    assert out["vs_baseline"] is None and "1500x" in out["metric"]


def test_graft_entry_build():
    sys.path.insert(0, ROOT)
    import __graft_entry__ as ge

    ge.build()


def test_bench_multirank_launch_contract():
    """The driver's N > 1 launch (torch.distributed.run, one process per rank,
    127.0.0.1 rendezvous), rehearsed on the CPU path with 4 gloo ranks: exactly
    one JSON line (rank 0), n_gpus / parallelism follow the rank count."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    r = run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
             "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
             "--gpus", "4", "--device", "cpu", "--samples", "1500", "--steps", "1", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.strip().split("\n") if l.startswith("{")]
    assert len(lines) == 1, lines
    out = json.loads(lines[0])
    assert out["n_gpus"] == 4 and out["config"]["parallelism"] == "dp4-shard" and out["converged"]
    assert out["dp_autotune"]["shard_s"] == out["value"] and out["dp_autotune"]["chosen"] == "shard"
    assert out["steps"] == 1 and out["warmup"] == 1 and out["value"] > 0
    # per-rank setup diagnostics at N > 1 (exchange self test, union, communicator)
    assert [d["timed"]["rank"] for d in out["rank_setup"]] == [0, 1, 2, 3]
    for d in out["rank_setup"]:
        assert {"comm", "exchange", "xch_selftest", "union", "n_local"} <= set(d["timed"])


def test_bench_spawns_its_own_ranks():
    """``bench.py --gpus N`` without a launcher starts the N ranks itself
    (torch.distributed.run child, never an exec) and relays rank 0's line."""
    r = run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu", "--samples", "2000",
             "--steps", "1", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.strip().split("\n") if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2-shard" and out["converged"]
    assert out["launcher"].startswith("bench.py spawned")


def test_bench_refuses_missing_devices_and_rank_mismatch():
    # --device cuda with fewer visible devices than --gpus: a clear non-zero exit, no silent downgrade
    env = dict(os.environ)
    env.pop("DPSVM_FORCE_DEVICE", None)
    r = run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cuda",
             "--samples", "500"], env=env)
    assert r.returncode == 2 and "visible device" in r.stderr
    # launched with a different rank count than --gpus: refused
    env["WORLD_SIZE"], env["RANK"], env["LOCAL_RANK"] = "1", "0", "0"
    r = run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu",
             "--samples", "500"], env=env)
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stderr + r.stdout)


def test_bench_presets_and_shrink_flag():
    """BASELINE configs as bench presets: covtype-ref is Makefile:77's run_cover
    recipe (500,000 rows, C=2048, gamma=0.03125, eps 1e-3, 3M cap); shrink is
    auto by default (on only where the whole Gram is not resident, GPU) and
    accepts on / off."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    a = bench.parse(["--config", "covtype-ref"])
    assert (a.samples, a.features, a.C, a.gamma, a.eps, a.max_iter) == (500000, 54, 2048.0, 0.03125, 1e-3, 3000000)
    assert a.shrink == "auto" and a.engines == "production"
    assert bench.parse(["--shrink", "off"]).shrink == "off"
    full = bench.parse(["--config", "covtype"])
    assert full.samples == 581012 and full.data == a.data == "covtype"
