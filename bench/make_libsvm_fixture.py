#!/usr/bin/env python3
"""LIBSVM (scikit-learn's libsvm, CPU) reference for the covtype-shape parity
test (tests/test_parity_gpu.py): trains sklearn.svm.SVC on the first N rows of
the deterministic synthetic covtype-shape set and stores its support-vector
count, intercept and decision values on M held-out rows of the same generator.

  python bench/make_libsvm_fixture.py [--n 20000] [--holdout 2000] [--C 2048]

The reference's README claims SV-count parity with LibSVM (README.md:27); its
covtype recipe is Makefile:77 (C=2048, gamma=0.03125, eps 1e-3).  The fixture is
generated here (no LIBSVM binary is run on the GPU box) and checked in.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20000)
    ap.add_argument("--holdout", type=int, default=2000)
    ap.add_argument("--C", type=float, default=2048.0)
    ap.add_argument("--gamma", type=float, default=0.03125)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "tests", "data", "libsvm_covtype20k.json"))
    a = ap.parse_args()
    from sklearn.svm import SVC

    from dpsvm_amd.utils.datasets import synthetic

    X, y = synthetic("covtype", n=a.n + a.holdout, seed=a.seed)
    Xt, yt, Xh, yh = X[:a.n], y[:a.n], X[a.n:], y[a.n:]
    t0 = time.time()
    m = SVC(C=a.C, gamma=a.gamma, kernel="rbf", tol=1e-3, cache_size=4000).fit(Xt, yt)
    dt = time.time() - t0
    dh = m.decision_function(Xh)
    # sklearn's classes_ are [-1, 1]: decision > 0 -> +1 (ours: sum alpha y K - b)
    rec = {"generator": "synthetic('covtype', n=N + holdout, seed)", "n": a.n, "holdout": a.holdout,
           "seed": a.seed, "C": a.C, "gamma": a.gamma, "tol": 1e-3, "sklearn_fit_s": round(dt, 2),
           "n_support": int(m.n_support_.sum()), "intercept": float(m.intercept_[0]),
           "n_bounded": int(np.sum(np.abs(m.dual_coef_) >= a.C * (1 - 1e-6))),
           "train_accuracy": float(np.mean(m.predict(Xt) == yt)),
           "holdout_accuracy": float(np.mean(np.where(dh > 0, 1.0, -1.0) == yh)),
           "holdout_decision": [round(float(v), 5) for v in dh]}
    with open(a.out, "w") as f:
        json.dump(rec, f)
    print({k: v for k, v in rec.items() if k != "holdout_decision"})
    return 0


if __name__ == "__main__":
    sys.exit(main())
