"""The ws-cache miss-row GEMM alone (rbf_rows_split_glds_kernel) at the
synthetic-2m round shape: m = 189 indexed rows against all n = 2,000,000 rows of
a d = 1024 split-operand X (operands split once), event-timed per launch.  The
B panel (8.2 GB of split operands) is streamed from HBM once per launch; the
report gives ms, the B stream's TB/s and the share of the split MFMA peak
(3 products x 2 m n d flops at 2.5 PFLOP/s dense f16).

    DPSVM_ROWS_BRING=3 python bench/rows_probe.py   # the round-5 B ring depth
    python bench/rows_probe.py [--n 2000000] [--d 1024] [--m 189] [--reps 7]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dpsvm_amd._native import load  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2_000_000)
    ap.add_argument("--d", type=int, default=1024)
    ap.add_argument("--m", type=int, default=189)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--out", default="")
    ap.add_argument("--stamps", action="store_true", help="one more launch of the stamps build: where a tile's time goes")
    a = ap.parse_args()
    C = load()
    n, d, m = a.n, a.d, a.m
    dp = (d + 15) // 16 * 16
    rows_alloc = (n + 511) // 512 * 512
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.zeros(rows_alloc, dp, device="cuda")
    x[:n, :d] = torch.rand(n, d, device="cuda", generator=g)
    s = torch.cuda.current_stream().cuda_stream
    xsq = torch.zeros(rows_alloc, device="cuda")
    C.k_row_sqnorm(x.data_ptr(), rows_alloc, dp, dp, xsq.data_ptr(), s)
    rng = np.random.default_rng(1)
    rows = torch.from_numpy(rng.choice(n, size=m, replace=False).astype(np.int32)).cuda()
    lines = torch.arange(m, dtype=torch.int32, device="cuda")
    ld = (n + 127) // 128 * 128
    out = torch.empty(m, ld, device="cuda")
    torch.cuda.synchronize()
    ms = C.k_rows_split_bench(x.data_ptr(), xsq.data_ptr(), n, dp, rows.data_ptr(), m, 1.0 / d, out.data_ptr(), ld,
                              lines.data_ptr(), a.reps + 1, s)[1:]
    med = float(np.median(ms))
    b_bytes = n * ((dp + 31) // 32) * 128  # split B panel: 128 B per row and 32-k block
    flops = 3 * 2.0 * m * n * ((dp + 31) // 32 * 32)
    # spot check against float64 on a few entries
    xr = x[:n, :d]
    sel = rows[:4].long()
    cols = torch.arange(0, n, max(1, n // 4096), device="cuda")[:4096]
    ref = torch.exp(-(1.0 / d) * torch.cdist(xr[sel].double(), xr[cols].double()) ** 2)
    err = float((out[:4, cols].double() - ref).abs().max())
    res = {"n": n, "d": d, "m": m, "ring": os.environ.get("DPSVM_ROWS_BRING", "3"), "persist": os.environ.get("DPSVM_ROWS_PERSIST", "1"), "ms_median": round(med, 4),
           "ms_min": round(float(min(ms)), 4), "b_stream_TBps": round(b_bytes / med / 1e9, 2),
           "split_peak_share": round(flops / (med * 1e-3) / 2.5e15, 3), "max_abs_err_vs_f64": err}
    if a.stamps:
        tiles = (n + 127) // 128  # one tile row (m <= 192)
        st = torch.zeros(tiles * 8, dtype=torch.int64, device="cuda")
        C.k_set_rows_stamps(st.data_ptr())
        C.k_rows_split_bench(x.data_ptr(), xsq.data_ptr(), n, dp, rows.data_ptr(), m, 1.0 / d, out.data_ptr(), ld,
                             lines.data_ptr(), 1, s)
        C.k_set_rows_stamps(0)
        v = st.view(-1, 8).cpu().numpy().astype(np.int64)
        v = v[(v[:, 0] > 0) & (v[:, 4] >= v[:, 0])]
        pro, loop, epi, drain = np.diff(v[:, :5], axis=1).T
        tot = v[:, 4] - v[:, 0]
        clk = float(np.median(tot / np.maximum(1, v[:, 6] - v[:, 5]) * 0.1))
        nkb = (dp + 31) // 32
        floor = nkb * 36 * 32  # 12 waves x 12 MFMAs a k block over 4 SIMDs, 32 cycles each
        span = (v[:, 6].max() - v[:, 5].min()) / 100.0
        res["stamps"] = {"workgroups": int(len(v)), "clock_ghz": round(clk, 3),
                         "cycles_median": {"prologue": float(np.median(pro)), "k_loop": float(np.median(loop)),
                                           "epilogue_issue": float(np.median(epi)), "drain": float(np.median(drain)),
                                           "total": float(np.median(tot))},
                         "k_loop_mfma_floor": floor, "k_loop_mfma_eff": round(floor / float(np.median(loop)), 3),
                         "span_us": round(span, 1),
                         "mean_wg_in_flight": round(((v[:, 6] - v[:, 5]).sum() / 100.0) / max(span, 1e-9), 1)}
    print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "a") as fh:
            fh.write(json.dumps(res) + "\n")


if __name__ == "__main__":
    main()
