"""Adaptive split Gram vs the three-product Gram (docs/DESIGN.md §13) on the
headline shape (MNIST-shape 60000 x 784, gamma 0.25): the symmetric Gram and
one rank's P = 8 slab K(60000, 7500).

Per case: median wall ms of the Gram call (CUDA events; includes the operand
split, ~0.07 ms, and for the adaptive Gram the log2-norm pass), hot tiles /
tiles, max |K_adaptive - K_three_product| (must be <= tau) and both kernels'
max error vs float64 on a 1024-row block.  Run under
`rocprofv3 --kernel-trace --stats` for the per-kernel split (h1 pass vs the
hot-tile pass).  --data mnist-parity: structured rows (gram_adapt auto would
refuse them; the probe forces it to show what that costs).
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dpsvm_amd.ops import kernels as K  # noqa: E402
from dpsvm_amd.utils.datasets import synthetic  # noqa: E402


def timed(fn, reps):
    ts = []
    for _ in range(reps + 1):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        out = fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts[1:])), out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=60000)
    ap.add_argument("--data", default="mnist")
    ap.add_argument("--gamma", type=float, default=0.25)
    ap.add_argument("--tau", type=float, default=2.0 ** -22)
    ap.add_argument("--slab", type=int, default=7500)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cases", default="sym,slab")
    ap.add_argument("--adaptive-only", action="store_true", help="skip the three-product Gram (A/B sweeps)")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    X, _ = synthetic(args.data, n=args.n, seed=1)
    x = torch.from_numpy(X).cuda()
    res = {"n": args.n, "d": X.shape[1], "data": args.data, "gamma": args.gamma, "tau": args.tau}
    sub = np.random.default_rng(0).choice(args.n, 1024, replace=False)
    subt = torch.from_numpy(sub).cuda()
    a64 = X[sub].astype(np.float64)
    for case in args.cases.split(","):
        b = None if case == "sym" else x[: args.slab].contiguous()
        ta, ka = timed(lambda: K.rbf_gram(x, b, args.gamma, split=True, cold_tau=args.tau), args.reps)
        tiles, hot = K.gram_adapt_last()
        if args.adaptive_only:
            res[case] = {"ms_adaptive": ta, "tiles": tiles, "hot_tiles": hot}
            print(case, json.dumps(res[case]), flush=True)
            continue
        t3, k3 = timed(lambda: K.rbf_gram(x, b, args.gamma, split=True), args.reps)
        diff = (ka - k3).abs().max().item()
        bx = X if case == "sym" else X[: args.slab]
        b64 = bx.astype(np.float64)
        d2 = (a64 * a64).sum(1)[:, None] + (b64 * b64).sum(1)[None, :] - 2 * a64 @ b64.T
        ref = np.exp(-args.gamma * np.maximum(d2, 0))
        e3 = float(np.abs(k3[subt].double().cpu().numpy() - ref).max())
        ea = float(np.abs(ka[subt].double().cpu().numpy() - ref).max())
        res[case] = {"ms_three_product": t3, "ms_adaptive": ta, "tiles": tiles, "hot_tiles": hot,
                     "max_diff": diff, "within_tau": diff <= args.tau, "err64_three_product": e3,
                     "err64_adaptive": ea}
        print(case, json.dumps(res[case]), flush=True)
        del k3, ka
        torch.cuda.empty_cache()
    print(json.dumps(res))
    if args.out:
        with open(args.out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
