"""Interleaved A/B of split Gram GEMM variants in ONE process (guide §5.4 rule 24).

Shapes: the headline's symmetric Gram (60000^2 x 784) and one rank's slab at
P ranks (A = all 60000 rows, B = 60000 / P rows, non-symmetric: what a sharded
ws-dense rank computes in its timed region).  Each round times every variant
once (CUDA events around the launch, the operand split included); prints the
median / min per variant and whether each variant's output is bit-identical to
the first one's (the split kernels must agree bit for bit: operand-swap
symmetry, docs/DESIGN.md §8b).

    python bench/gram_variants.py --variants 5,6 --rounds 7 [--slab 8]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dpsvm_amd._native import load  # noqa: E402
from dpsvm_amd.utils.datasets import synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=60000)
    ap.add_argument("--variants", default="5,6")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--slab", type=int, default=0, help="P: also time the n x n/P slab (0: symmetric only)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    C = load()
    X, _ = synthetic("mnist", n=a.n, seed=1)
    n, d = X.shape
    dp = (d + 15) // 16 * 16
    rows = (n + 255) // 256 * 256 + 512
    x = torch.zeros(rows, dp, device="cuda")
    x[:n, :d] = torch.from_numpy(X).cuda()
    s = torch.cuda.current_stream().cuda_stream
    xsq = torch.zeros(rows, device="cuda")
    C.k_row_sqnorm(x.data_ptr(), rows, dp, dp, xsq.data_ptr(), s)
    variants = [int(v) for v in a.variants.split(",")]
    shapes = [("sym", n, True)]
    if a.slab > 1:
        shapes.append((f"slab{a.slab}", (n + a.slab - 1) // a.slab, False))
    res = {}
    for name, nb, sym in shapes:
        ld = (nb + 127) // 128 * 128
        outs = {v: torch.empty((n, ld), device="cuda") for v in variants}
        times = {v: [] for v in variants}
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for r in range(a.rounds + 1):
            for v in variants:
                C.k_set_split_gemm_variant(v)
                torch.cuda.synchronize()
                ev0.record()
                C.k_rbf_gram_split(x.data_ptr(), xsq.data_ptr(), n, x.data_ptr(), xsq.data_ptr(), nb, dp, 0.25,
                                   outs[v].data_ptr(), ld, sym, s)
                ev1.record()
                torch.cuda.synchronize()
                if r > 0:
                    times[v].append(ev0.elapsed_time(ev1))
        C.k_set_split_gemm_variant(0)
        base = outs[variants[0]]
        for v in variants:
            o = outs[v]
            if sym:  # the symmetric kernels write both triangles
                same = bool(torch.equal(o[:, :n], base[:, :n]))
            else:
                same = bool(torch.equal(o[:, :nb], base[:, :nb]))
            t = np.array(times[v])
            res[f"{name}/v{v}"] = {"median_ms": float(np.median(t)), "min_ms": float(t.min()),
                                   "bit_identical_to_v%d" % variants[0]: same}
            print(name, v, json.dumps(res[f"{name}/v{v}"]), flush=True)
        del outs
        torch.cuda.empty_cache()
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
