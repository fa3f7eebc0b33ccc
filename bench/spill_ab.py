#!/usr/bin/env python3
"""Host spill tier vs recompute, per problem shape (one MI355X).

A kernel-row line of an n-row problem is n floats.  A pinned-host spill tier
would bring an evicted line back over PCIe (n x 4 B); the working-set cache
engine instead recomputes the round's missing rows with one MFMA row GEMM
(2 n d FLOP per row, rbf_rows_indexed).  Measured here for the BASELINE
shapes:
  * fetch: hipMemcpy of pinned host memory -> device, one line and a batch of
    64 lines (the bandwidth a spill tier could reach at best);
  * recompute: rbf_rows_indexed for 64 / 192 missing rows of the shape (time
    per row).
Prints one JSON line (--out writes it too).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [("covtype-581k", 581012, 54), ("mnist-200k", 200000, 784), ("synthetic-2m", 2000000, 1024)]


def timeit(fn, reps=5):
    import torch

    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return min(ts)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch

    from dpsvm_amd.ops import kernels as K

    out = {}
    for name, n, d in SHAPES:
        r = {"n": n, "d": d, "line_MB": round(n * 4 / 2**20, 2)}
        host = torch.empty((64, n), dtype=torch.float32).pin_memory()
        dev = torch.empty((64, n), dtype=torch.float32, device="cuda")
        t1 = timeit(lambda: dev[0].copy_(host[0], non_blocking=True))
        t64 = timeit(lambda: dev.copy_(host, non_blocking=True))
        r["fetch_one_line_us"] = round(t1 * 1e6, 1)
        r["fetch_per_line_us_batch64"] = round(t64 / 64 * 1e6, 1)
        r["pcie_GBps"] = round(64 * n * 4 / t64 / 1e9, 1)
        del host, dev
        from dpsvm_amd._native import load

        C = load()
        xp, dp = K._pad_rows_cols(torch.rand(n, d, device="cuda"), row_mult=512)
        xsq = torch.zeros(xp.shape[0], device="cuda")
        C.k_row_sqnorm(xp.data_ptr(), xp.shape[0], dp, dp, xsq.data_ptr(), K._stream(xp))
        ld = (n + 127) // 128 * 128
        for m in (64, 192):
            rows = torch.arange(0, n, n // m, dtype=torch.int32, device="cuda")[:m].contiguous()
            lines = torch.arange(m, dtype=torch.int32, device="cuda")
            outl = torch.empty((m, ld), device="cuda")
            tr = timeit(lambda: C.k_rbf_rows_indexed(xp.data_ptr(), xsq.data_ptr(), n, dp, rows.data_ptr(), m,
                                                     1.0 / d, outl.data_ptr(), ld, lines.data_ptr(),
                                                     K._stream(xp)), reps=3)
            r[f"recompute_per_row_us_{m}rows"] = round(tr / m * 1e6, 2)
            del outl
        del xp, xsq
        r["fetch_over_recompute"] = round(r["fetch_per_line_us_batch64"] / r["recompute_per_row_us_192rows"], 1)
        out[name] = r
        torch.cuda.empty_cache()
        print(name, json.dumps(r), flush=True)
    line = json.dumps(out)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
