#!/usr/bin/env python3
"""PROJECTION (not a measurement) of covtype (581k x 54, box) and synthetic-2m
(2M x 1024) at 1/2/4/8 MI355X under the multi-GPU policy bench.py runs
(--gpus N: shrink=auto agreed over the ranks, each phase a multi-rank solve
with dp=auto: rows sharded when the phase's Gram does not fit one GPU,
replicated when it does), from one-GPU measurements:

  * per-kernel time per round at the full shape (rocprofv3 kernel trace of a
    capped plain solve, profiles/r4_big_inputs/*_kernel_stats.csv): the
    f-update/selection pass (ws_select) and the miss-row GEMM
    (rbf_gemm_split / rbf_rows_split_glds) work on a rank's rows and divide by
    P; the merge, gather and sub-problem solve run redundantly on every rank;
    the remainder of the measured round period (launch gaps) stays;
  * the in-kernel peer exchange's own per-round cost at the same shape, loopback
    at world 1 (profiles/r4_big_inputs/runs.jsonl: peer vs local);
  * the shrinking phases of the one-GPU run (rows, rounds, seconds:
    profiles/r4_big_configs_final_1gpu.jsonl phase_log);
  * ASSUMED: X us extra latency per exchange point of a store crossing xGMI
    (3 points per round) — the one input no single GPU can measure.

A whole-problem phase at P ranks: rounds x (redundant + rows / P + gaps +
exchange(P)); a shrunk phase whose Gram fits one GPU runs replicated (dp=auto):
its one-GPU time.  The trajectory (rounds) is the one-GPU one: sharded solves
are bit-identical to one rank (tests/test_ws_gpu.py peer-exchange tests).

  python bench/project_big.py
"""
import csv
import json
import sys

INP = "profiles/r4_big_inputs"
HBM_GRAM_BYTES = 0.8 * 288e9  # a phase's Gram "fits one GPU" (dp=auto replicate) below this (cache_frac 0.8)


def kernel_round_us(path, rounds):
    """{class: us per round} from a rocprofv3 kernel_stats.csv"""
    out = {"rows": 0.0, "redundant": 0.0, "other": 0.0}
    for r in csv.DictReader(open(path)):
        name, tot = r["Name"], float(r["TotalDurationNs"]) / 1e3
        if "ws_select" in name or "rbf_gemm_split_kernel" in name or "rbf_rows_split" in name:
            out["rows"] += tot / rounds
        elif any(k in name for k in ("ws_solve", "ws_merge", "ws_gather", "ws_rank", "ws_xcollect")):
            out["redundant"] += tot / rounds
        else:
            out["other"] += tot / rounds
    return out


def runs():
    """profiles/r4_big_inputs/runs.jsonl, in order: covtype capped solve with the
    loopback peer exchange and its local twin (the same kernels: their
    difference is the exchange's cost), covtype local with the round-4 ROWS
    kernel, synthetic-2m local (same), the covtype P = 8 slab probe"""
    return [json.loads(line) for line in open(f"{INP}/runs.jsonl") if line.strip()]


def main() -> int:
    rs = runs()
    cov_peer, cov_local_old, cov_local, syn_local = rs[0], rs[1], rs[2], rs[3]
    slab = rs[4]["slab"]["8"]
    assert cov_peer["exchange"] == "loopback" and cov_local_old["exchange"] == "none"
    fin = [json.loads(line) for line in open("profiles/r4_big_configs_final_1gpu.jsonl") if line.strip()]
    cov_shr = next(r for r in fin if r["preset"] == "covtype" and r["shrink"]["on"])
    syn_shr = next(r for r in fin if r["preset"] == "synthetic-2m" and r["shrink"]["on"])
    ext = 1e6 * (cov_peer["value"] - cov_local_old["value"]) / cov_local_old["rounds"]
    print(f"measured loopback peer-exchange cost at covtype shape: {ext:.1f} us/round "
          f"({cov_peer['value']:.3f} vs {cov_local_old['value']:.3f} s, {cov_local_old['rounds']} rounds)")
    print(f"measured covtype dense Gram slab at P = 8 (K(581012 rows, 72627 columns), {slab['gb']} GB): "
          f"{slab['s']} s - the P = 8 whole-problem phase may run ws-dense; projected as ws-cache "
          f"(its miss-row GEMM / P): an upper bound")
    cov_run, syn_run = cov_local, syn_local
    shapes = []
    for name, run, stats, shr, n, d in (
            ("covtype box 581k x 54", cov_run, f"{INP}/covtype_box_2M_steps_kernel_stats.csv", cov_shr, 581012, 54),
            ("synthetic-2m 2M x 1024", syn_run, f"{INP}/synthetic2m_120k_steps_kernel_stats.csv", syn_shr, 2000000,
             1024)):
        k = kernel_round_us(stats, run["rounds"])
        period = 1e6 * run["value"] / run["rounds"]
        gaps = max(0.0, period - k["rows"] - k["redundant"] - k["other"])
        print(f"{name}: measured round {period:.1f} us = rows {k['rows']:.1f} (/P) + redundant {k['redundant']:.1f} "
              f"+ other {k['other']:.2f} + gaps {gaps:.1f}")
        shapes.append((name, k, gaps, period, shr, n))
    print("PROJECTION, seconds (ASSUMED xGMI store-to-poll latency X per exchange point, 3 per round)")
    print(f"{'shape':<26} {'X us':>5} | " + " | ".join(f"P={p:<2d}" for p in (1, 2, 4, 8)) + " | policy at P > 1")
    for name, k, gaps, period, shr, n in shapes:
        phases = [p.split() for p in shr["shrink"]["phase_log"].split(";")]
        for X in (2, 4, 8):
            row = []
            for P in (1, 2, 4, 8):
                t = 0.0
                for ph in phases:
                    rows_ph, rounds_ph, sec = int(ph[0]), int(ph[2]), float(ph[3])
                    if P == 1 or rows_ph * rows_ph * 4.0 <= HBM_GRAM_BYTES:
                        t += sec  # one GPU, or replicated (dp=auto: the phase's Gram fits): one-GPU time
                        continue
                    per1 = 1e6 * sec / rounds_ph  # this phase's measured round, split as the full shape's
                    f_rows = k["rows"] / period
                    per = per1 * (1 - f_rows) + per1 * f_rows / P + ext + 3 * X
                    t += rounds_ph * per * 1e-6
                row.append(t)
            pol = " + ".join(("shard" if int(ph[0]) ** 2 * 4.0 > HBM_GRAM_BYTES else "replicate") for ph in phases)
            print(f"{name:<26} {X:>5} | " + " | ".join(f"{v:6.2f}" for v in row) + f" | shrink phases: {pol}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
