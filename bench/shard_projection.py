#!/usr/bin/env python3
"""Inputs of the sharded multi-GPU projection, measured on ONE MI355X
(docs/DESIGN.md "Sharded headline: projection").

  1. the headline solve as run by the library default (ws-dense, adaptive
     multi-block rounds): time, Gram GEMM, rounds;
  2. the same solve with every per-round collective issued through a one-rank
     RCCL communicator (force_collectives, captured in the round graph): the
     launch cost of the three collectives per round without any transfer;
  3. one rank's Gram slab K(all n rows, n / P owned columns) for P = 1, 2, 4, 8
     (the non-symmetric split-operand MFMA GEMM a sharded rank runs, incl. the
     fp16 split of its operands);
  4. the round anatomy from in-kernel stamps (DPSVM_STAMPS): which phases are
     per-rank redundant (merge, gather, solve) and which scale with n / P (the
     two f-update passes).

Prints one JSON line; --out writes it too.  Every number here is a one-GPU
measurement; the projection itself (bench/project_shard.py) is arithmetic on
them plus an explicitly assumed xGMI collective latency.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=60000)
    ap.add_argument("--features", type=int, default=784)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    stamp_path = os.path.join(tempfile.mkdtemp(), "ws_stamps")
    import torch

    from dpsvm_amd import SVC
    from dpsvm_amd._native import load
    from dpsvm_amd.ops import kernels as K
    from dpsvm_amd.utils.datasets import synthetic

    C = load()
    X, y = synthetic("mnist", n=a.samples, d=a.features, seed=0)
    kw = dict(C=10.0, gamma=0.25, eps=1e-3, device="cuda")
    out = {"n": a.samples, "d": a.features}

    def best(fn):
        ts = []
        r = None
        for _ in range(a.reps):
            r = fn()
            ts.append(r.fit_time_)
        return min(ts), r

    t_loc, loc = best(lambda: SVC(**kw).fit(X, y))
    out["local"] = {"s": round(t_loc, 6), "gram_s": round(float(loc.stats_["t_gram"]), 6), "rounds": loc.n_rounds_,
                    "steps": loc.n_iter_, "engine": loc.setup_info_["iteration"],
                    "blocks": [int(loc.stats_.get("ws_blocks", 1)), int(loc.stats_.get("ws_blocks_end", 1))]}
    comm = C.rccl_comm(C.rccl_unique_id(), 0, 1, 0)
    t_rc, rc = best(lambda: SVC(force_collectives=True, **kw).fit(X, y, comm=comm))
    out["rccl_one_rank"] = {"s": round(t_rc, 6), "rounds": rc.n_rounds_, "steps": rc.n_iter_,
                            "same_trajectory": bool(rc.n_iter_ == loc.n_iter_ and np.array_equal(rc.alpha_, loc.alpha_)),
                            "extra_us_per_round": round(1e6 * (t_rc - t_loc) / max(1, rc.n_rounds_), 2)}
    del comm
    # the multi-block rounds over the in-kernel peer exchange at world 1
    # (loopback: every push lands in the own receive buffer, the collect kernels
    # and the solve poll it): the exchange's per-round kernel cost without xGMI
    t_px, px = best(lambda: SVC(exchange="peer", xch_timeout_s=60.0, **kw).fit(X, y))
    out["peer_loopback"] = {"s": round(t_px, 6), "rounds": px.n_rounds_, "steps": px.n_iter_,
                            "exchange": px.setup_info_.get("exchange"),
                            "blocks": int(px.stats_.get("ws_blocks", 1)),
                            "same_trajectory": bool(px.n_iter_ == loc.n_iter_ and np.array_equal(px.alpha_, loc.alpha_)),
                            "extra_us_per_round": round(1e6 * (t_px - t_loc) / max(1, px.n_rounds_), 2)}

    # one rank's Gram slab: K(all rows, n / P columns), non-symmetric GEMM
    # (the adaptive Gram when the local solve ran it, docs/DESIGN.md §13: every rank applies the same rule)
    xt = torch.tensor(X, device="cuda")
    tau = 2.0 ** -22 if loc.setup_info_.get("gram") == "split-f16-adaptive" else 0.0
    out["gram_slab_mode"] = "adaptive" if tau else "three-product"
    slabs = {}
    for P in (1, 2, 4, 8):
        cols = xt[: (a.samples + P - 1) // P]
        K.rbf_gram(xt, cols, 0.25, split=True, cold_tau=tau)  # warm
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            K.rbf_gram(xt, cols, 0.25, split=True, cold_tau=tau)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        slabs[P] = round(min(ts), 6)
    out["gram_slab_s"] = slabs
    torch.cuda.empty_cache()

    # round anatomy (stamps; 10 ns ticks)
    os.environ["DPSVM_STAMPS"] = stamp_path
    st = SVC(**kw).fit(X, y)
    del os.environ["DPSVM_STAMPS"]
    raw = np.fromfile(stamp_path + ".rank0", dtype=np.uint64).reshape(4096, 24).astype(np.int64)
    R = min(st.n_rounds_, 4096)
    s = raw[2:R]
    # (stamp 8, the gather kernel's exit, is absent when the solve loads its
    # block itself: direct sub-Gram at world 1)
    s = s[(s[:, [0, 1, 2, 3, 4, 6, 7]] > 0).all(axis=1)]
    us = lambda v: float(np.round(np.median(v) * 0.01, 2))  # noqa: E731
    out["round_us"] = {
        "period": us(np.diff(s[:, 6])),
        # the candidate rank kernel (stamp 21) + the merge: redundant on every rank
        "merge": us(s[:, 2] - s[:, 21]) if (s[:, 21] > 0).all() else us(s[:, 2] - s[:, 1]),
        "gather": us(s[:, 8] - s[:, 2]) if (s[:, 8] > 0).all() else 0.0,
        "load_subgram": us(s[:, 3] - s[:, 0]),
        "solve": us(s[:, 4] - s[:, 3]),
        "select_pass2": us(s[:, 7] - s[:, 6]),
        "select_pass1_wg0": us(s[:, 23] - s[:, 22]) if (s[:, 22] > 0).all() else None,
        "pass1_start_to_pass2_start": us(s[:, 6] - s[:, 22]) if (s[:, 22] > 0).all() else None,
        "steps_per_round": float(np.median(s[:, 5])),
    }
    line = json.dumps(out)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
