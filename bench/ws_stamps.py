#!/usr/bin/env python3
"""Phase anatomy of the working-set engine from in-kernel s_memrealtime stamps
(DPSVM_STAMPS; 100 MHz).  Ring slot r holds, in time order: ws_select
workgroup 0 entry/f updated/exit (6, 10, 7: the f update + candidates before round r),
ws_gather workgroup 0 entry (1), merged (2), exit (8), ws_solve entry (0),
sub-Gram loaded (3), sub-problem solved (4), pair steps (5).

  python bench/ws_stamps.py [--samples N] [--features D] [...]
"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--data", default="mnist")
    ap.add_argument("--samples", type=int, default=60000)
    ap.add_argument("--features", type=int, default=784)
    ap.add_argument("--C", type=float, default=10.0)
    ap.add_argument("--gamma", type=float, default=0.25)
    ap.add_argument("--ws-size", type=int, default=192)
    ap.add_argument("--ws-new", type=int, default=0)
    ap.add_argument("--ws-rel", type=float, default=0.3)
    ap.add_argument("--ws-blocks", type=int, default=0, help="0: the library default (adaptive multi-block)")
    ap.add_argument("--max-iter", type=int, default=10**7)
    ap.add_argument("--cache-lines", type=int, default=0)
    ap.add_argument("--force-cache", action="store_true")
    ap.add_argument("--exchange", default="auto", help="peer: the in-kernel exchange at world 1 (loopback)")
    ap.add_argument("--clip", default="independent", choices=["independent", "box"])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    path = os.path.join(tempfile.mkdtemp(), "ws_stamps")
    os.environ["DPSVM_STAMPS"] = path
    from dpsvm_amd import SVC
    from dpsvm_amd.utils.datasets import synthetic

    X, y = synthetic(a.data, n=a.samples, d=a.features)
    clf = SVC(C=a.C, gamma=a.gamma, eps=1e-3, device="cuda", solver="ws", ws_size=a.ws_size, ws_new=a.ws_new,
              ws_rel=a.ws_rel, ws_blocks=a.ws_blocks, max_iter=a.max_iter, cache_lines=a.cache_lines, force_cache=a.force_cache,
              exchange=a.exchange, xch_timeout_s=60.0, clip=a.clip, shrink="off").fit(X, y)
    raw = np.fromfile(path + ".rank0", dtype=np.uint64).reshape(4096, 24).astype(np.int64)
    rounds = min(clf.n_rounds_, 4096)
    s = raw[2:rounds]
    # direct sub-Gram loads (blocks of <= 64 rows at world 1): no ws_gather launch, so no stamp 8
    direct = not (s[:, 8] > 0).any()
    if direct:
        s = s.copy()
        s[:, 8] = s[:, 2]  # "gather end" = merged: gather_end_to_solve becomes merged-to-solve
    ok = (s[:, [0, 1, 2, 3, 4, 6, 7, 8]] > 0).all(axis=1)
    us = lambda v: np.round(np.median(v) * 0.01, 2)  # noqa: E731  (10 ns ticks -> us)
    s = s[ok]
    nxt = np.roll(raw[:, 6], -1)[2:rounds][ok]
    res = {
        "rounds": clf.n_rounds_, "pair_steps": clf.n_iter_, "fit_time_s": round(clf.fit_time_, 4),
        "b": float(clf.b_), "n_sv": int(clf.n_support_), "engine": clf.setup_info_["iteration"],
        "rows_computed": int(clf.stats_.get("rows_computed", 0)),
        "steps_per_round_median": float(np.median(s[:, 5])),
        "select_wg0_us": us(s[:, 7] - s[:, 6]),
        "select_fupdate_us": us(s[:, 10] - s[:, 6]),
        "select_candidates_us": us(s[:, 7] - s[:, 10]),
        "select_end_to_gather_us": us(s[:, 1] - s[:, 7]),
        "merge_us": us(s[:, 2] - s[:, 1]),
        **({"rank_and_merge_us": us(s[:, 2] - s[:, 21])} if a.ws_blocks != 1 else {}),
        "merge_phases_us": ({"lists_and_stop_test": us(s[:, 11] - s[:, 1]), "radix_thresholds": us(s[:, 12] - s[:, 11]),
                             "class_compaction": us(s[:, 13] - s[:, 12]), "hash_dedup": us(s[:, 14] - s[:, 13]),
                             "previous_set": us(s[:, 2] - s[:, 14])} if a.ws_blocks == 1 else
                            {"rank_kernel_to_merge": us(s[:, 1] - s[:, 21]), "sorted_loads_hash_init": us(s[:, 20] - s[:, 1]),
                             "to_sorted_keys": us(s[:, 11] - s[:, 1]), "stop_test_hash_insert": us(s[:, 12] - s[:, 11]),
                             "dedup_compaction": us(s[:, 13] - s[:, 12]), "previous_union": us(s[:, 14] - s[:, 13]),
                             "block_assignment": us(s[:, 2] - s[:, 14])}),
        "gather_rows_us": us(s[:, 8] - s[:, 2]),
        **({"merged_to_gather_entry_us": us(s[:, 9] - s[:, 2]), "gather_kernel_us": us(s[:, 8] - s[:, 9])}
           if (s[:, 9] > 0).all() else {}),
        "gather_end_to_solve_us": us(s[:, 0] - s[:, 8]),
        "load_subgram_us": us(s[:, 3] - s[:, 0]),
        **({"subgram": "direct (ws_solve loads its block; gather_* = merged -> solve)"} if direct else {}),
        "solve_us": us(s[:, 4] - s[:, 3]),
        "solve_per_step_us": float(np.round(np.median((s[:, 4] - s[:, 3]) / np.maximum(1, s[:, 5])) * 0.01, 3)),
        "solve_end_to_next_select_us": us(nxt - s[:, 4]),
        "round_period_us": us(np.diff(s[:, 6])),
    }
    if clf.setup_info_.get("ws_rows") == "recompute":  # ws_recompute.hip: select = the fused pass (6 -> 7)
        res["ws_rows"] = "recompute"
        for k in ("select_fupdate_us", "select_candidates_us"):
            res.pop(k, None)
    if (s[:, 15] > 0).all():  # multi-block peer exchange: the two collect kernels (workgroup 0)
        res["exchange"] = clf.setup_info_.get("exchange")
        res["peer_phases_us"] = {
            "pass2_end_to_collect_cand": us(s[:, 15] - s[:, 7]),
            "collect_cand_wg0": us(s[:, 16] - s[:, 15]),
            "collect_cand_to_rank": us(s[:, 21] - s[:, 16]),
            "pass1_wg0": us(s[:, 23] - s[:, 22]),
            "pass1_to_collect_part": us(s[:, 17] - s[:, 23]),
            "collect_part_wg0": us(s[:, 19] - s[:, 17]),
            "collect_part_to_pass2": us(s[:, 6] - s[:, 19]),
        }
    if (s[:, 18] > 0).any():  # experimental per-phase core-clock cycle sums (s_memtime)
        st = np.maximum(1, s[:, 5])
        res["cycles_per_step"] = {k: float(np.median(s[:, 12 + i] / st)) for i, k in enumerate(
            ["reduce", "argpos", "lds", "pair", "fupdate", "set_alpha"])}
        res["cycles_per_step"]["loop_total"] = float(np.median(s[:, 18] / st))
    line = json.dumps(res)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
