#!/usr/bin/env python3
"""Cache-mode statistics for a bench preset: X passes, misses, speculative
rows and us/iteration per speculation width (capped iteration count).
  python bench/cache_stats.py --config covtype --max-iter 300000 --spec 0,8,14"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="covtype")
    ap.add_argument("--max-iter", type=int, default=300000)
    ap.add_argument("--spec", default="0,8,14")
    ap.add_argument("--lines", type=int, default=0)
    a = ap.parse_args()
    import torch  # noqa: F401
    import bench
    from dpsvm_amd import SVCConfig
    from dpsvm_amd._native import load
    from dpsvm_amd.utils.datasets import synthetic

    p = bench.PRESETS[a.config]
    C = load()
    X, y = synthetic(p["data"], n=p["samples"], d=p["features"], seed=0)
    for spec in [int(v) for v in a.spec.split(",")]:
        cfg = SVCConfig(C=p["C"], gamma=p["gamma"], eps=p["eps"], max_iter=a.max_iter, cache_lines=a.lines,
                        spec_rows=spec)
        s = C.GpuSolver(cfg.to_native(X.shape[1]), None, 0)
        si = s.setup(X, X.shape[0], y)
        t0 = time.perf_counter()
        _, info = s.solve()
        wall = time.perf_counter() - t0
        print(json.dumps({"config": a.config, "variant": si["iteration"], "lines": si["cache_lines"], "spec": spec,
                          "iters": info["iters"], "t_solve_s": round(info["t_solve"], 3), "wall_s": round(wall, 3),
                          "us_per_iter": round(1e6 * info["t_solve"] / max(1, info["iters"]), 3),
                          "x_passes": info["x_passes"], "rows_computed": info["rows_computed"],
                          "misses": info["cache_misses"], "hits": info.get("cache_hits"),
                          "spec_rows": info["spec_rows"]}), flush=True)
        del s


if __name__ == "__main__":
    main()
