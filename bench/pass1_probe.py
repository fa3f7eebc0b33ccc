#!/usr/bin/env python3
"""Pass-1 (multi-block f update) kernel time at the per-rank shapes of the
sharded headline: a rank of P owns n = 60000 / P columns of every Gram row and
a round changes up to 6,144 rows (the default union: 128 blocks x 48).  Times ws_select pass 1 alone
(event-timed, repeated: it only reads the state) on crafted state through the
ws_select probe, for several list-slice counts ks (pass-1 workgroups per
selection group), to see whether the G = ceil(n / 256) workgroups of the
selection geometry can drive the memory system at small n.

  python bench/pass1_probe.py [--rows 60000] [--reps 20] [--out file.jsonl]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=60000, help="Gram rows (lines) of the shard")
    ap.add_argument("--cols", default="7500,15000,30000", help="columns per rank (60000 / P)")
    ap.add_argument("--ks", default="1,2,4,8,16")
    ap.add_argument("--changed", type=int, default=6144)
    ap.add_argument("--blocks", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--wide", action="store_true", help="the wide pass 1 (ws_pass1_v4_kernel, the default)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from dpsvm_amd._native import load

    C = load()
    rng = np.random.default_rng(0)
    blocks, q = a.blocks, a.changed // a.blocks
    out = []
    for n in [int(v) for v in a.cols.split(",")]:
        L = a.rows
        gram = np.full((L, n), 0.5, dtype=np.float32)
        f = rng.standard_normal(n).astype(np.float32)
        y = np.where(rng.random(n) < 0.5, -1.0, 1.0).astype(np.float32)
        alpha = (rng.random(n) * 5).astype(np.float32)
        dalpha = np.zeros(n, dtype=np.float32)
        lines = rng.permutation(L)[: blocks * q].astype(np.int32)
        coef = (rng.standard_normal(blocks * q) * 1e-2).astype(np.float32)
        nab = np.full(blocks, q, dtype=np.int32)
        for ks in [int(v) for v in a.ks.split(",")]:
            r = C.k_ws_select(gram.reshape(-1), L, n, f, alpha, y, dalpha, lines, coef, nab, blocks, blocks, blocks, q,
                              10.0, 1, ks=ks, reps=a.reps, wide=a.wide)
            t = np.array(r["pass1_us"][2:])
            rec = {"cols": n, "rows": L, "changed": int(blocks * q), "G": int(r["G"]), "ks": ks,
                   "wide": bool(a.wide), "p1G": int(r["p1G"]), "workgroups": int(r["p1G"]) * ks, "pass1_us_median": round(float(np.median(t)), 2),
                   "pass1_us_min": round(float(t.min()), 2),
                   "GBps": round(blocks * q * n * 4 / (float(np.median(t)) * 1e-6) / 1e9, 1)}
            print(json.dumps(rec), flush=True)
            out.append(rec)
        del gram
    if a.out:
        with open(a.out, "w") as fo:
            for rec in out:
                fo.write(json.dumps(rec) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
