"""A/B of the two Gram GEMMs on the headline shape (MNIST-shape 60000 x 784,
gamma 0.25): the f32-input MFMA kernel (rbf_gemm.hip) and the fp16 split-operand
kernel (rbf_gemm_split.hip), symmetric mode as the dense engines run it.

Prints per-kernel wall times (CUDA events around the launch, the split one
including its split_rows pass), TFLOP/s counted as f32 work of the computed
tiles, and the accuracy of both against float64 on a 2048-row block.
Run under `rocprofv3 --kernel-trace --stats` for the per-kernel split.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dpsvm_amd._native import load  # noqa: E402
from dpsvm_amd.utils.datasets import synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=60000)
    ap.add_argument("--d", type=int, default=784)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default="")
    ap.add_argument("--only", default="", choices=["", "f32", "split"])
    args = ap.parse_args()
    C = load()
    X, _ = synthetic("mnist", n=args.n, seed=1)
    n, d = X.shape
    dp = (d + 15) // 16 * 16
    rows = (n + 255) // 256 * 256 + 512
    x = torch.zeros(rows, dp, device="cuda")
    x[:n, :d] = torch.from_numpy(X).cuda()
    s = torch.cuda.current_stream().cuda_stream
    xsq = torch.zeros(rows, device="cuda")
    C.k_row_sqnorm(x.data_ptr(), rows, dp, dp, xsq.data_ptr(), s)
    ld = (n + 127) // 128 * 128
    out = torch.empty((n, ld), device="cuda")
    res = {"n": n, "d": d}
    tiles = (n + 127) // 128
    flops = 2.0 * 128 * 128 * dp * tiles * (tiles + 1) / 2  # upper tiles incl. the diagonal
    sub = np.random.default_rng(0).choice(n, 2048, replace=False)
    for name, fn in (("f32", C.k_rbf_gram), ("split", C.k_rbf_gram_split)):
        if args.only and name != args.only:
            continue
        ts = []
        for r in range(args.reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn(x.data_ptr(), xsq.data_ptr(), n, x.data_ptr(), xsq.data_ptr(), n, dp, 0.25, out.data_ptr(), ld, True, s)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        t = min(ts[1:])
        got = out[torch.from_numpy(sub).cuda()][:, :n].double().cpu().numpy()
        a = X[sub].astype(np.float64)
        b = X.astype(np.float64)
        d2 = (a * a).sum(1)[:, None] + (b * b).sum(1)[None, :] - 2 * a @ b.T
        ref = np.exp(-0.25 * np.maximum(d2, 0))
        err = np.abs(got - ref)
        res[name] = {"ms": t * 1e3, "tflops_f32_equiv": flops / t / 1e12, "max_abs_err": float(err.max()),
                     "mean_abs_err": float(err.mean())}
        print(name, json.dumps(res[name]), flush=True)
    print(json.dumps(res))
    if args.out:
        with open(args.out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
