#!/usr/bin/env python3
"""Summarise DPSVM_STAMPS in-kernel timestamps of the fused SMO iteration.

Slots (s_memrealtime, 100 MHz): 0 entry, 1 pair known (first round trip +
wave reduction), 2 eta/alpha update done (second round trip), 3 row loop done,
4 keys stored (end).  Workgroup 0 and workgroup G-1 of each iteration.
Usage: DPSVM_STAMPS=/tmp/st python bench.py ...; python bench/stamps_report.py /tmp/st.rank0
"""
import json
import sys

import numpy as np

RING, SLOTS = 4096, 12


LRU_ORDER = [0, 1, 8, 9, 10, 2, 3, 4, 5, 6, 7]  # slot order in time
LRU_PHASES = ["alpha", "need_slots", "spec_cands", "spec_rank", "rows_chosen", "victims", "plan", "fill", "commit",
              "f_update_keys"]


def main_lru(path):
    """smo_fused_lru slots: 0 entry, 1 alpha update, 2 rows chosen, 3 victims,
    4 plan done, 5 lines filled, 6 commit, 7 end; split by fill time (X pass)."""
    a = np.fromfile(path, dtype=np.uint64).reshape(RING, 2, SLOTS).astype(np.int64)
    ok = (a[:, :, 0] > 0).all(1) & (a[:, :, 7] > 0).all(1)
    a = a[ok]
    out = {"samples": int(len(a))}
    for b, name in ((0, "wg0"), (1, "wglast")):
        t = a[:, b, LRU_ORDER].copy()
        # slots 9/10 are only stamped in speculating iterations: carry the previous time
        for c in range(1, t.shape[1]):
            t[:, c] = np.where(t[:, c] >= t[:, c - 1], t[:, c], t[:, c - 1])
        d = np.diff(t, axis=1) * 10.0
        fill = d[:, LRU_PHASES.index("fill")]
        for tag, sel in (("pass", fill > 3000), ("nopass", fill <= 3000)):
            if sel.sum() == 0:
                continue
            out[f"{name}_{tag}"] = {"n": int(sel.sum()),
                                    **{ph + "_ns": float(np.median(d[sel, i])) for i, ph in enumerate(LRU_PHASES)},
                                    "total_ns": float(np.median((a[sel, b, 7] - a[sel, b, 0]) * 10.0))}
    period = np.diff(a[:, 0, 0]) * 10.0
    out["iter_period_ns_median"] = float(np.median(period[period > 0]))
    print(json.dumps(out, indent=1))


PERSIST_PHASES = ["poll", "alpha_update", "f_update", "key_reduce", "publish", "to_next_poll"]


def main_persist(path):
    """smo_persist slots: 0 poll start, 1 pair known, 2 alpha update, 3 f
    update, 4 keys reduced, 5 published; ring index = iteration."""
    a = np.fromfile(path, dtype=np.uint64).reshape(RING, 2, SLOTS).astype(np.int64)[:, :, :6]
    out = {}
    for b, name in ((0, "wg0"), (1, "wglast")):
        t = a[:, b, :]
        ok = (t > 0).all(1)
        d = np.diff(t, axis=1) * 10.0
        nxt = (np.roll(t[:, 0], -1) - t[:, 5]) * 10.0  # next iteration's poll start - this publish
        okn = ok & np.roll(ok, -1)
        out[name] = {ph + "_ns": float(np.median(d[ok, i])) for i, ph in enumerate(PERSIST_PHASES[:5])}
        out[name]["to_next_poll_ns"] = float(np.median(nxt[okn]))
        per = np.diff(t[:, 0]) * 10.0
        out[name]["period_ns"] = float(np.median(per[(per > 0) & ok[1:] & ok[:-1]]))
    print(json.dumps(out, indent=1))


def main(path):
    a = np.fromfile(path, dtype=np.uint64).reshape(RING, 2, SLOTS).astype(np.int64)
    ok = (a[:, 0, 0] > 0) & (a[:, 0, 4] > 0) & (a[:, 1, 4] > 0)
    a = a[ok]
    out = {}
    for b, name in ((0, "wg0"), (1, "wglast")):
        d = np.diff(a[:, b, :5], axis=1) * 10.0  # ns
        out[name] = {
            "entry->pair_ns": float(np.median(d[:, 0])),
            "pair->update_ns": float(np.median(d[:, 1])),
            "update->rows_ns": float(np.median(d[:, 2])),
            "rows->end_ns": float(np.median(d[:, 3])),
            "entry->end_ns": float(np.median((a[:, b, 4] - a[:, b, 0]) * 10.0)),
        }
    # kernel-to-kernel: entry of iteration t+1 minus end of iteration t (workgroup 0),
    # only for consecutive ring slots
    it0 = a[:, 0, 0]
    nxt = it0[1:] - a[:-1, 0, 4]
    period = np.diff(it0) * 10.0
    out["iter_period_ns_median"] = float(np.median(period[period > 0]))
    out["end_to_next_entry_ns_median"] = float(np.median(nxt[nxt > 0] * 10.0))
    out["wg_skew_entry_ns_median"] = float(np.median((a[:, 1, 0] - a[:, 0, 0]) * 10.0))
    out["samples"] = int(len(a))
    print(json.dumps(out, indent=1))


PLRU_PHASES = ["poll", "pair_to_plan", "fill", "f_update", "keys_publish"]


def main_plru(path):
    """smo_persist_lru slots: 0 poll start, 1 pair known, 2 plan broadcast,
    3 lines filled, 4 f update, 5 published, 6 rows filled; split by fills."""
    a = np.fromfile(path, dtype=np.uint64).reshape(RING, 2, SLOTS).astype(np.int64)
    out = {}
    for b, name in ((0, "wg0"), (1, "wglast")):
        t = a[:, b, :6]
        ok = (t > 0).all(1)
        rows = a[:, b, 6]
        d = np.diff(t, axis=1) * 10.0
        per = np.diff(t[:, 0]) * 10.0
        for tag, sel in (("fill", ok & (rows > 0)), ("hit", ok & (rows == 0))):
            if sel.sum() == 0:
                continue
            out[f"{name}_{tag}"] = {"n": int(sel.sum()),
                                    **{ph + "_ns": float(np.median(d[sel, i])) for i, ph in enumerate(PLRU_PHASES)}}
            pp = per[sel[:-1] & ok[1:] & (per > 0)]
            if len(pp):
                out[f"{name}_{tag}"]["period_ns"] = float(np.median(pp))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "--plru":
        main_plru(sys.argv[1])
        sys.exit(0)
    if len(sys.argv) > 2 and sys.argv[2] == "--lru":
        main_lru(sys.argv[1])
    elif len(sys.argv) > 2 and sys.argv[2] == "--persist":
        main_persist(sys.argv[1])
    else:
        main(sys.argv[1])
