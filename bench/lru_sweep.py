#!/usr/bin/env python3
"""Cache-mode sweep on the MNIST-shape problem: speculation width x iteration
variant (fused one-launch kernel vs rows/step/finalize chain) x cache size.
Prints one JSON line per run (us/iteration, X passes, misses, speculative rows)."""
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
    ap.add_argument("--lines", default="20000")
    ap.add_argument("--spec", default="0,4,8,14")
    ap.add_argument("--variants", default="fused,chain")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch  # noqa: F401
    from dpsvm_amd import SVCConfig
    from dpsvm_amd._native import load
    from dpsvm_amd.utils.datasets import synthetic

    C = load()
    X, y = synthetic("mnist", n=a.samples, d=a.features, seed=0)
    out = []
    for variant in a.variants.split(","):
        if variant == "chain":
            os.environ["DPSVM_LRU_KERNELS"] = "3"
        else:
            os.environ.pop("DPSVM_LRU_KERNELS", None)
        for lines in [int(v) for v in a.lines.split(",")]:
            for spec in [int(v) for v in a.spec.split(",")]:
                cfg = SVCConfig(C=10.0, gamma=0.25, eps=1e-3, cache_lines=lines, spec_rows=spec)
                s = C.GpuSolver(cfg.to_native(X.shape[1]), None, 0)
                si = s.setup(X, X.shape[0], y)
                t0 = time.perf_counter()
                _, info = s.solve()
                wall = time.perf_counter() - t0
                rec = {"variant": si["iteration"], "lines": lines, "spec": spec, "iters": info["iters"],
                       "t_solve_s": round(info["t_solve"], 4), "wall_s": round(wall, 4),
                       "us_per_iter": round(1e6 * info["t_solve"] / max(1, info["iters"]), 3),
                       "x_passes": info["x_passes"], "rows_computed": info["rows_computed"],
                       "misses": info["cache_misses"], "hits": info.get("cache_hits"), "spec_rows": info["spec_rows"]}
                print(json.dumps(rec), flush=True)
                out.append(rec)
                del s
    if a.out:
        with open(a.out, "w") as f:
            f.write("\n".join(json.dumps(r) for r in out) + "\n")


if __name__ == "__main__":
    main()
