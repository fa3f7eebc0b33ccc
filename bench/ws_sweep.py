#!/usr/bin/env python3
"""Working-set engine parameter sweep on the headline problem (one process):
ws_size (q), ws_new (rows replaced per round), ws_rel (sub-problem tolerance
relative to the global gap).  Prints one line per setting: solve seconds
(median of 3), rounds, pair steps, b.

  python bench/ws_sweep.py [--q 192] [--new 120,144,168] [--rel 0.2,0.3,0.5]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--q", default="192")
    ap.add_argument("--new", default="0")
    ap.add_argument("--rel", default="0.3")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from dpsvm_amd import SVC
    from dpsvm_amd.utils.datasets import synthetic

    X, y = synthetic("mnist", n=60000, d=784)
    for q in [int(v) for v in a.q.split(",")]:
        for nw in [int(v) for v in a.new.split(",")]:
            for rel in [float(v) for v in a.rel.split(",")]:
                clf = SVC(C=10.0, gamma=0.25, eps=1e-3, device="cuda", solver="ws", ws_size=q, ws_new=nw, ws_rel=rel)
                ts = []
                for _ in range(a.reps):
                    clf.fit(X, y)
                    ts.append(clf.fit_time_)
                print(f"q {q} new {nw} rel {rel}: {statistics.median(ts):.4f} s  rounds {clf.n_rounds_} "
                      f"steps {clf.n_iter_} b {clf.b_:.6f} conv {clf.converged_}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
