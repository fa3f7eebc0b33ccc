#!/usr/bin/env python3
"""Per-iteration latency anatomy of the device-resident SMO loop.

Prints (JSON lines):
  * launch floor: us per kernel of a hipGraph chain of dependent empty kernels
    (the MI355X 'boundary' cost) for several grid sizes;
  * SMO loop: us per iteration for the dense fused kernel, the fused cache-mode
    kernel and the cache-mode rows + step + finalize chain, on the MNIST-shape headline problem,
    for several graph block sizes.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=60000)
    ap.add_argument("--features", type=int, default=784)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch  # noqa: F401  (single HIP runtime)
    from dpsvm_amd import SVCConfig
    from dpsvm_amd._native import load
    from dpsvm_amd.utils.datasets import synthetic

    C = load()
    lines = []
    for blocks in (1, 64, 235, 256, 1024):
        us = C.launch_floor_us(blocks, 256, 64, 50)
        lines.append({"what": "launch_floor", "blocks": blocks, "us_per_kernel": round(us, 3)})
    X, y = synthetic("mnist", n=a.samples, d=a.features, seed=0)
    modes = (("dense", {"persist": "off"}), ("dense-persist", {"persist": "on"}), ("lru", {"cache_lines": 20000}),
             ("lru-chain", {"cache_lines": 20000}))
    for mode, extra in modes:
        if mode == "lru-chain":
            os.environ["DPSVM_LRU_KERNELS"] = "3"  # rows/step/finalize chain (A/B)
        for gb in ((64,) if mode == "lru-chain" else (16, 64, 256)):
            if mode == "dense-persist":
                extra = dict(extra, persist_block=gb * 32)
            cfg = SVCConfig(C=10.0, gamma=0.25, eps=1e-3, graph_block=gb, **extra)
            s = C.GpuSolver(cfg.to_native(X.shape[1]), None, 0)
            si = s.setup(X, X.shape[0], y)
            s.solve()  # warm (graph build, caches)
            t0 = time.perf_counter()
            alpha, info = s.solve()
            wall = time.perf_counter() - t0
            lines.append({"what": "smo_loop", "mode": mode, "graph_block": gb, "iters": info["iters"],
                          "t_solve_s": round(info["t_solve"], 4), "wall_s": round(wall, 4),
                          "us_per_iter": round(1e6 * info["t_solve"] / max(1, info["iters"]), 3),
                          "x_passes": info["x_passes"], "rows_computed": info["rows_computed"],
                          "misses": info["cache_misses"], "spec_rows": info.get("spec_rows"),
                          "iteration": si["iteration"]})
            del s
    out = "\n".join(json.dumps(l) for l in lines)
    print(out)
    if a.out:
        with open(a.out, "w") as f:
            f.write(out + "\n")


if __name__ == "__main__":
    main()
