#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs per kernel (sums over dispatches).

MFMA work: SQ_INSTS_VALU_MFMA_MOPS_F32 x 512 = f32 MFMA FLOPs (rocprofv3's
MfmaFlopsF32); achieved TFLOP/s uses the dispatch durations of the same run
(counter collection serialises dispatches)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root):
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        agg = defaultdict(lambda: defaultdict(float))
        dur = defaultdict(dict)
        for r in csv.DictReader(open(f)):
            short = r.get("Kernel_Name", "?").split("(")[0].replace("dpsvm::dev::", "").replace("void ", "")
            agg[short][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[short][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        print(f"== {os.path.relpath(f, root)}")
        for k, cs in agg.items():
            ns = sum(dur[k].values())
            line = ", ".join(f"{c}={v:.4g}" for c, v in sorted(cs.items()))
            extra = f"  [{len(dur[k])} dispatches, {ns / 1e6:.3f} ms"
            if cs.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0) > 0 and ns > 0:
                fl = cs["SQ_INSTS_VALU_MFMA_MOPS_F32"] * 512
                extra += f", f32 MFMA {fl / 1e12:.3f} TFLOP = {fl / ns / 1e3:.1f} TFLOP/s ({100 * fl / ns / 1e3 / 157.3:.0f}% of 157.3)"
            for c in ("FETCH_SIZE", "WRITE_SIZE"):  # KiB over the kernel's serialised dispatches
                if cs.get(c, 0) > 0 and ns > 0:
                    extra += f", {c} {cs[c] / 1024 ** 2:.2f} GiB = {cs[c] * 1024 / ns:.0f} GB/s"
            print(f"  {k}: {line}{extra}]")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
