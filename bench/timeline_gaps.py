#!/usr/bin/env python3
"""Per-solve GPU timeline from a rocprofv3 --kernel-trace CSV: the solves are
split at the Gram GEMM launches; for each, the wall span from the first kernel
to the last, the summed kernel time, and the largest gaps between consecutive
kernels (host-side or launch overhead)."""
import csv
import glob
import os
import sys


def main(root):
    f = glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    solves, cur = [], []
    for r in rows:
        name = r["Kernel_Name"]
        if "split_rows_kernel" in name and cur:  # each solve starts with the operand split
            solves.append(cur)
            cur = []
        cur.append(r)
    solves.append(cur)
    for i, s in enumerate(solves):
        t0, t1 = int(s[0]["Start_Timestamp"]), int(s[-1]["End_Timestamp"])
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in s)
        gaps = []
        for a, b in zip(s, s[1:]):
            g = int(b["Start_Timestamp"]) - int(a["End_Timestamp"])
            gaps.append((g, a["Kernel_Name"].split("(")[0][-40:], b["Kernel_Name"].split("(")[0][-40:]))
        gaps.sort(reverse=True)
        tot_gap = sum(max(0, g[0]) for g in gaps)
        print(f"solve {i}: {len(s)} kernels, span {(t1 - t0) / 1e6:.3f} ms, kernel busy {busy / 1e6:.3f} ms, "
              f"gaps {tot_gap / 1e6:.3f} ms")
        for g in gaps[:6]:
            print(f"   gap {g[0] / 1e3:8.1f} us  {g[1]} -> {g[2]}")
    # per-kernel totals of the last solve
    agg = {}
    for r in solves[-1]:
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("dpsvm::dev::", "")
        c, t = agg.get(k, (0, 0))
        agg[k] = (c + 1, t + int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    print("last solve, per kernel:")
    for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"   {k[:52]:52s} {c:4d} x  {t / 1e6:7.3f} ms  ({t / 1e3 / c:8.1f} us each)")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
