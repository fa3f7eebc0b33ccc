#!/usr/bin/env python3
"""Working-set parameter sweep on a small coupled problem (the covtype-shape
shrunk phases: one block per round, second-order pair choice): ws_rel
(sub-problem tolerance relative to the global gap), ws_new (rows replaced per
round), ws_inner (pair steps per round at most).  One JSON line per setting.

  python bench/ws_sweep_small.py --n 7500 [--rel 0.1,0.3] [--new 96,144] [--inner 0,2000]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--data", default="covtype")
    ap.add_argument("--n", type=int, default=7500)
    ap.add_argument("--d", type=int, default=54)
    ap.add_argument("--C", type=float, default=2048.0)
    ap.add_argument("--gamma", type=float, default=0.03125)
    ap.add_argument("--clip", default="box")
    ap.add_argument("--q", default="192")
    ap.add_argument("--rel", default="0.3")
    ap.add_argument("--new", default="0")
    ap.add_argument("--inner", default="0")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from dpsvm_amd import SVC
    from dpsvm_amd.utils.datasets import synthetic

    X, y = synthetic(a.data, n=a.n, d=a.d)
    for q in [int(v) for v in a.q.split(",")]:
        for rel in [float(v) for v in a.rel.split(",")]:
            for nw in [int(v) for v in a.new.split(",")]:
                for inner in [int(v) for v in a.inner.split(",")]:
                    clf = SVC(C=a.C, gamma=a.gamma, eps=1e-3, clip=a.clip, device="cuda", solver="ws", ws_size=q,
                              ws_rel=rel, ws_new=nw, ws_inner=inner, ws_blocks=1, shrink="off", max_iter=50_000_000)
                    clf.fit(X, y)
                    line = json.dumps({"data": a.data, "n": a.n, "q": q, "rel": rel, "new": nw, "inner": inner,
                                       "fit_s": round(clf.fit_time_, 4), "rounds": int(clf.n_rounds_),
                                       "steps": int(clf.n_iter_), "b": float(clf.b_), "n_sv": int(clf.n_support_),
                                       "converged": bool(clf.converged_)})
                    print(line, flush=True)
                    if a.out:
                        with open(a.out, "a") as f:
                            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
