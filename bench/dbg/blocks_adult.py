"""multi-block rounds on coupled problems: stop status, steps, rounds, final gap per P and clip"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
from dpsvm_amd import SVC
from dpsvm_amd.utils.datasets import synthetic
X, y = synthetic("adult", n=3000, seed=2)
for clip in ("independent", "box"):
    for P in (1, 2, 4, 8):
        for q in (192, 64):
            w = SVC(C=1.0, gamma=0.05, eps=1e-3, clip=clip, device="cuda", solver="ws", ws_blocks=P, ws_size=q,
                    max_iter=60000).fit(X, y)
            s = w.stats_
            yy = np.where(y > 0, 1.0, -1.0)
            print(clip, "P", P, "q", q, "status", w.status_, "steps", w.n_iter_, "rounds", w.n_rounds_,
                  "gap", s.get("b_lo", 0) - s.get("b_hi", 0), "sum(ay)", float(np.sum(w.alpha_ * yy)), flush=True)
