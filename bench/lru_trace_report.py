#!/usr/bin/env python3
"""Duration histogram of the fused cache kernel from a rocprofv3 kernel trace:
separates X-pass launches from pass-free ones, reports gaps between launches."""
import csv
import json
import sys

import numpy as np


def main(path, name="smo_fused_lru"):
    rows = [r for r in csv.DictReader(open(path)) if name in r["Kernel_Name"]]
    st = np.array([int(r["Start_Timestamp"]) for r in rows], dtype=np.int64)
    en = np.array([int(r["End_Timestamp"]) for r in rows], dtype=np.int64)
    d = (en - st) / 1000.0
    gaps = (st[1:] - en[:-1]) / 1000.0
    cut = 20.0
    out = {"launches": int(len(d)), "mean_us": float(d.mean()),
           "pass_launches": int((d > cut).sum()), "pass_median_us": float(np.median(d[d > cut])) if (d > cut).any() else None,
           "nopass_median_us": float(np.median(d[d <= cut])) if (d <= cut).any() else None,
           "gap_median_us": float(np.median(gaps)), "gap_mean_us": float(gaps.mean()),
           "period_mean_us": float((en[-1] - st[0]) / 1000.0 / len(d))}
    print(json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:])
