#!/usr/bin/env python3
"""One rank's Gram slab K(all n rows, n / P owned columns) at a big shape, the
non-symmetric split-operand MFMA GEMM a sharded ws-dense rank runs in its
timed region (rbf_gemm_split.hip) — measured on one MI355X with the output
preallocated (the kernel alone, event-timed), for the P whose slab fits.

  python bench/slab_probe.py --samples 581012 --features 54 --gamma 0.03125 --P 8
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--data", default="covtype")
    ap.add_argument("--samples", type=int, default=581012)
    ap.add_argument("--features", type=int, default=54)
    ap.add_argument("--gamma", type=float, default=0.03125)
    ap.add_argument("--P", default="8")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch

    from dpsvm_amd._native import load
    from dpsvm_amd.ops.kernels import _pad_rows_cols, _stream
    from dpsvm_amd.utils.datasets import synthetic

    C = load()
    X, _ = synthetic(a.data, n=a.samples, d=a.features, seed=0)
    xt = torch.tensor(X, device="cuda")
    ap_, dp = _pad_rows_cols(xt)
    asq = torch.zeros(ap_.shape[0], device="cuda")
    C.k_row_sqnorm(ap_.data_ptr(), ap_.shape[0], dp, dp, asq.data_ptr(), _stream(xt))
    free, total = torch.cuda.mem_get_info()
    res = {"n": a.samples, "d": a.features, "free_gb": round(free / 2**30, 1), "slab": {}}
    for P in [int(v) for v in a.P.split(",")]:
        cols = (a.samples + P - 1) // P
        ld = (cols + 127) // 128 * 128
        gb = a.samples * ld * 4 / 2**30
        if a.samples * ld * 4 > free - (8 << 30):
            res["slab"][P] = {"gb": round(gb, 1), "fits": False}
            continue
        out = torch.empty((a.samples, ld), device="cuda")
        bp, _ = _pad_rows_cols(xt[:cols])  # padded like the op's B operand (zero rows past cols)
        bsq = torch.zeros(bp.shape[0], device="cuda")
        C.k_row_sqnorm(bp.data_ptr(), bp.shape[0], dp, dp, bsq.data_ptr(), _stream(xt))
        ts = []
        for _ in range(a.reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            C.k_rbf_gram_split(ap_.data_ptr(), asq.data_ptr(), a.samples, bp.data_ptr(), bsq.data_ptr(), cols, dp,
                               float(a.gamma), out.data_ptr(), ld, False, _stream(xt))
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 1e3)
        ok = bool(torch.isfinite(out[:: max(1, a.samples // 64), :cols]).all().item())
        res["slab"][P] = {"gb": round(gb, 1), "fits": True, "s": round(min(ts[1:]), 5), "finite": ok,
                          "TBps_write": round(a.samples * ld * 4 / min(ts[1:]) / 1e12, 2)}
        del out
        torch.cuda.empty_cache()
        print(json.dumps(res), flush=True)
    line = json.dumps(res)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
