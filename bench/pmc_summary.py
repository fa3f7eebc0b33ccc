#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs per kernel (sums over dispatches)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root):
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        agg = defaultdict(lambda: defaultdict(float))
        calls = defaultdict(set)
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "?")
            short = k.split("(")[0].replace("dpsvm::dev::", "").replace("void ", "")
            agg[short][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[short].add(r.get("Dispatch_Id", ""))
        print(f"== {os.path.relpath(f, root)}")
        for k, cs in agg.items():
            line = ", ".join(f"{c}={v:.4g}" for c, v in sorted(cs.items()))
            extra = ""
            if "SQ_VALU_MFMA_BUSY_CYCLES" in cs and "GRBM_GUI_ACTIVE" in cs and cs["GRBM_GUI_ACTIVE"] > 0:
                # MFMA busy per CU-cycle: busy cycles are summed over the chip's CUs (256)
                extra = f"  [MFMA busy ~{100.0 * cs['SQ_VALU_MFMA_BUSY_CYCLES'] / (cs['GRBM_GUI_ACTIVE'] * 256):.1f}% of CU-cycles]"
            print(f"  {k} (dispatches {len(calls[k])}): {line}{extra}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
