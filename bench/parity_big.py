#!/usr/bin/env python3
"""Model-level agreement between two trajectories of one big configuration
(VERDICT round 4, item 5): the default solve and an alternative (shrinking off,
another graph-block size, ...), compared on held-out rows of the same
deterministic generator — decision-sign agreement, held-out accuracy, support
vectors, b — plus each run's training time.  One JSON line per comparison.

  python bench/parity_big.py --config covtype-box [--alt '{"shrink": "off"}'] [--holdout 5000]

Configs: covtype-box (581,012 x 54, C=2048, gamma=0.03125, box clipping, to tol 1e-3),
covtype-ref (Makefile:77: 500,000 rows, the reference's independent clipping,
3M-step cap), synthetic-2m (2,000,000 x 1024, C=1, gamma=1/1024).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CONFIGS = {
    "covtype-box": dict(data="covtype", n=581012, d=54, C=2048.0, gamma=0.03125, clip="box", max_iter=60_000_000),
    "covtype-ref": dict(data="covtype", n=500000, d=54, C=2048.0, gamma=0.03125, clip="independent",
                        max_iter=3_000_000),
    "synthetic-2m": dict(data="uniform", n=2000000, d=1024, C=1.0, gamma=1.0 / 1024, clip="independent",
                         max_iter=3_000_000),
    "covtype-200k": dict(data="covtype", n=200000, d=54, C=2048.0, gamma=0.03125, clip="box", max_iter=60_000_000),
}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="covtype-box", choices=sorted(CONFIGS))
    ap.add_argument("--base", default="{}", help="SVC knobs of the default run (JSON)")
    ap.add_argument("--alt", default='{"shrink": "off"}', help="SVC knobs of the alternative run (JSON)")
    ap.add_argument("--holdout", type=int, default=5000)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from dpsvm_amd import SVC
    from dpsvm_amd.utils.datasets import synthetic

    c = CONFIGS[a.config]
    X, y = synthetic(c["data"], n=c["n"], d=c["d"], seed=0)
    # held-out rows: the generator's rows n .. n + holdout (prefix-stable: rows are seeded by index)
    Xh, yh = synthetic(c["data"], n=c["n"] + a.holdout, d=c["d"], seed=0, row0=c["n"], rows=a.holdout)
    runs = {}
    for tag, knobs in (("base", json.loads(a.base)), ("alt", json.loads(a.alt))):
        kw = dict(C=c["C"], gamma=c["gamma"], eps=1e-3, clip=c["clip"], max_iter=c["max_iter"], device="cuda")
        kw.update(knobs)
        t0 = time.perf_counter()
        clf = SVC(**kw).fit(X, y)
        wall = time.perf_counter() - t0
        d = np.asarray(clf.decision_function(Xh))
        runs[tag] = {"knobs": knobs, "fit_time_s": round(float(clf.fit_time_), 3), "wall_s": round(wall, 2),
                     "converged": bool(clf.converged_), "pair_steps": int(clf.n_iter_),
                     "rounds": int(getattr(clf, "n_rounds_", 0) or 0), "n_sv": int(clf.n_support_),
                     "n_bounded": int(np.sum(clf.alpha_ >= c["C"] * (1 - 1e-6))), "b": float(clf.b_),
                     "sum_alpha_y": float((clf.alpha_.astype(np.float64) * np.where(y > 0, 1.0, -1.0)).sum()),
                     "holdout_accuracy": float(np.mean(np.where(d >= 0, 1.0, -1.0) == yh)),
                     "engine_note": clf.setup_info_.get("engine_note", "")}
        runs[tag]["_d"] = d
        runs[tag]["_sv"] = clf.alpha_ > 0
        print(f"[parity] {tag}: {json.dumps({k: v for k, v in runs[tag].items() if not k.startswith('_')})}",
              file=sys.stderr, flush=True)
        del clf
    db, da = runs["base"].pop("_d"), runs["alt"].pop("_d")
    sb, sa = runs["base"].pop("_sv"), runs["alt"].pop("_sv")
    res = {"config": a.config, **{k: v for k, v in CONFIGS[a.config].items()}, "holdout_rows": a.holdout,
           "base": runs["base"], "alt": runs["alt"],
           "decision_sign_agreement": float(np.mean(np.sign(db) == np.sign(da))),
           "decision_max_abs_diff": float(np.max(np.abs(db - da))),
           "decision_median_abs_diff": float(np.median(np.abs(db - da))),
           "sv_set_symmetric_diff": int(np.sum(sb ^ sa)), "abs_b_diff": abs(runs["base"]["b"] - runs["alt"]["b"])}
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        with open(a.out, "a") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
