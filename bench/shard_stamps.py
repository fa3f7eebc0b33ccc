#!/usr/bin/env python3
"""Per-rank round anatomy of a sharded run from in-kernel stamps (DPSVM_STAMPS;
each rank writes <path>.rank<r>): the peer exchange's consumer phases — the
candidate collect kernel (stamps 15 -> 16), the line-search partials collect
(17 -> 19), the solve's sub-Gram poll + LDS load (0 -> 3) — and the round
period, medians over rounds 2 .. R.

Run the sharded solve with stamps, e.g. (every rank on one GPU: a ONE-GPU
measurement — the ranks' kernels share the device, so the consumers' waits
include the other ranks' work, an upper bound of the exchange cost on 8 GPUs):

  DPSVM_STAMPS=/tmp/st DPSVM_FORCE_DEVICE=0 python bench.py --gpus 8 --dp shard --steps 1 --warmup 0
  python bench/shard_stamps.py /tmp/st 8 [--out file.json]
"""
import argparse
import json
import os
import sys

import numpy as np

RING, SLOTS = 4096, 24  # kStampRing rounds x (2 x kStampSlots) u64 per round


def rank_phases(path: str, rounds: int) -> dict:
    raw = np.fromfile(path, dtype=np.uint64).reshape(RING, SLOTS).astype(np.int64)
    s = raw[2:min(rounds, RING)]
    ok = (s[:, [0, 3, 6, 15, 16]] > 0).all(axis=1)
    s = s[ok]
    us = lambda v: round(float(np.median(v)) * 0.01, 2)  # noqa: E731  (10 ns ticks)
    out = {"rounds_used": int(len(s)),
           "round_period_us": us(np.diff(s[:, 6])),
           "collect_cand_us": us(s[:, 16] - s[:, 15]),
           "solve_poll_load_us": us(s[:, 3] - s[:, 0]),
           "solve_us": us(s[:, 4] - s[:, 3])}
    if (s[:, 17] > 0).all() and (s[:, 19] > 0).all():
        out["collect_part_us"] = us(s[:, 19] - s[:, 17])
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("ranks", type=int)
    ap.add_argument("--rounds", type=int, default=RING)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    per = [rank_phases(f"{a.path}.rank{r}", a.rounds) for r in range(a.ranks) if os.path.exists(f"{a.path}.rank{r}")]
    keys = [k for k in per[0] if k.endswith("_us")]
    res = {"ranks": len(per), "one_gpu_measurement": True,
           "median_over_ranks": {k: round(float(np.median([p[k] for p in per if k in p])), 2) for k in keys},
           "max_over_ranks": {k: round(float(np.max([p[k] for p in per if k in p])), 2) for k in keys},
           "per_rank": per}
    # the exchange's consumer cost per round: both collects + the solve's poll/load
    m = res["median_over_ranks"]
    res["exchange_consumer_us_per_round"] = round(m["collect_cand_us"] + m.get("collect_part_us", 0.0)
                                                  + m["solve_poll_load_us"], 2)
    line = json.dumps(res)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
