"""Where a wide-wave Gram tile's time goes: per-workgroup s_memtime stamps of
rbf_gemm_split_w64_kernel (the NT = 3 diagnostics build of the same kernel,
C.k_set_gram_stamps): entry -> first k block landed (prologue: row data + the
first LDS-DMA) -> k loop done -> stores issued (epilogue math + store issue)
-> stores done, and s_memrealtime at entry / end (100 MHz) for the clock and
the number of workgroups in flight over the kernel's span.

The k loop's MFMA floor per tile is nkb x 48 MFMAs x 32 cycles per SIMD
(2 waves x 24 v_mfma_f32_32x32x16_f16 per 32-k block), so loop / floor is the
loop's MFMA efficiency in shader cycles.

    python bench/gram_stamps.py [--n 60000] [--slab 8]
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


def analyse(st, nkb, kernel_ms):
    st = st.astype(np.int64)
    ok = (st[:, 0] > 0) & (st[:, 4] >= st[:, 0])
    st = st[ok]
    # (the persistent kernel stamps per tile: [0] tile start, [1] first block
    # landed, [2] k loop done, [3] = [4] stores issued; no drain stamp)
    pro, loop, epi, drain = (np.diff(st[:, :5], axis=1)).T
    total = st[:, 4] - st[:, 0]
    clk_ghz = float(np.median(total / np.maximum(1, st[:, 6] - st[:, 5]) * 0.1))  # memtime ticks per 10 ns
    floor = nkb * 48 * 32
    span_us = (st[:, 6].max() - st[:, 5].min()) / 100.0
    busy_us = (st[:, 6] - st[:, 5]).sum() / 100.0
    med = lambda v: float(np.median(v))  # noqa: E731
    # persistent kernel: tile L is step L // 256 of its workgroup (drift check:
    # do later steps run slower k loops?)
    idx = np.nonzero(ok)[0]
    step = idx // 256
    by_step = {}
    for lo, hi in ((0, 1), (1, 10), (10, 100), (100, 10**9)):
        m = (step >= lo) & (step < hi)
        if m.any():
            by_step[f"{lo}-{hi if hi < 10**9 else 'end'}"] = med(loop[m])
    return {
        "k_loop_cycles_by_step": by_step,
        "workgroups": int(len(st)), "clock_ghz_median": round(clk_ghz, 3),
        "cycles_median": {"prologue": med(pro), "k_loop": med(loop), "epilogue_store_issue": med(epi),
                          "store_drain": med(drain), "total": med(total)},
        "share_of_tile": {k: round(med(v) / med(total), 3) for k, v in
                          (("prologue", pro), ("k_loop", loop), ("epilogue_store_issue", epi), ("store_drain", drain))},
        "k_loop_mfma_floor_cycles": floor, "k_loop_mfma_efficiency": round(floor / med(loop), 3),
        "tile_mfma_efficiency": round(floor / med(total), 3),
        "span_us": round(span_us, 1), "kernel_ms_events": round(kernel_ms, 3),
        "mean_workgroups_in_flight": round(busy_us / max(span_us, 1e-9), 1),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=60000)
    ap.add_argument("--slab", type=int, default=0, help="P: also the n x n/P slab")
    ap.add_argument("--variant", type=int, default=0, help="split GEMM variant (6 w64 tiles, 7 persistent)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    C = load()
    X, _ = synthetic("mnist", n=a.n, seed=1)
    n, d = X.shape
    dp = (d + 15) // 16 * 16
    nkb = (dp + 31) // 32
    rows = (n + 255) // 256 * 256 + 512
    x = torch.zeros(rows, dp, device="cuda")
    x[:n, :d] = torch.from_numpy(X).cuda()
    s = torch.cuda.current_stream().cuda_stream
    xsq = torch.zeros(rows, device="cuda")
    C.k_row_sqnorm(x.data_ptr(), rows, dp, dp, xsq.data_ptr(), s)
    res = {}
    shapes = [("sym", n, True)] + ([(f"slab{a.slab}", (n + a.slab - 1) // a.slab, False)] if a.slab > 1 else [])
    for name, nb, sym in shapes:
        ld = (nb + 127) // 128 * 128
        out = torch.empty((n, ld), device="cuda")
        tiles = ((n + 255) // 256) * ((nb + 127) // 128)
        stamps = torch.zeros(tiles * 8, dtype=torch.int64, device="cuda")
        C.k_set_split_gemm_variant(a.variant)
        C.k_rbf_gram_split(x.data_ptr(), xsq.data_ptr(), n, x.data_ptr(), xsq.data_ptr(), nb, dp, 0.25,
                           out.data_ptr(), ld, sym, s)  # warm
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        C.k_set_gram_stamps(stamps.data_ptr())
        torch.cuda.synchronize()
        ev0.record()
        C.k_rbf_gram_split(x.data_ptr(), xsq.data_ptr(), n, x.data_ptr(), xsq.data_ptr(), nb, dp, 0.25,
                           out.data_ptr(), ld, sym, s)
        ev1.record()
        torch.cuda.synchronize()
        C.k_set_gram_stamps(0)
        C.k_set_split_gemm_variant(0)
        st = stamps.view(-1, 8).cpu().numpy()
        res[name] = analyse(st, nkb, ev0.elapsed_time(ev1))
        print(name, json.dumps(res[name]), flush=True)
        del out, stamps
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
