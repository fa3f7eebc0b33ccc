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
