#!/usr/bin/env python3
"""Per-kernel statistics from a rocprofv3 SQLite result (rocpd *_results.db):
calls, total / mean / min time, share of GPU time.  Kernel names are shortened
to the function name and its template arguments.

  python bench/rocpd_stats.py gpurun_out/prof/run_results.db [--top 25] [--csv out.csv]
"""
import argparse
import re
import sqlite3
import sys


def short(name: str) -> str:
    name = re.sub(r"\(.*\)$", "", name)  # parameter list
    name = re.sub(r"^(void )?(dpsvm::)?(dev::)?", "", name)
    return name.replace("dpsvm::dev::", "")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--csv", default=None)
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    name_col = "name" if "name" in cols else "kernel_name"
    rows = db.execute(f"select {name_col}, start, end from kernels").fetchall()
    agg = {}
    for n, s, e in rows:
        k = short(n)
        d = (e - s) * 1e-3  # ns -> us
        c, t, mn = agg.get(k, (0, 0.0, float("inf")))
        agg[k] = (c + 1, t + d, min(mn, d))
    total = sum(v[1] for v in agg.values())
    out = sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]
    lines = ["kernel,calls,total_us,mean_us,min_us,pct"]
    for k, (c, t, mn) in out:
        lines.append(f"\"{k}\",{c},{t:.1f},{t / c:.2f},{mn:.2f},{100 * t / total:.1f}")
    text = "\n".join(lines)
    print(text)
    if a.csv:
        with open(a.csv, "w") as f:
            f.write(text + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
