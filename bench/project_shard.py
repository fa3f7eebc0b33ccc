#!/usr/bin/env python3
"""PROJECTION (not a measurement) of the sharded headline solve at 1/2/4/8
MI355X, from the one-GPU measurements of bench/shard_projection.py plus an
explicitly ASSUMED cost of the per-round collectives over xGMI.

Per round, a rank of P:
  * runs the merge, the sub-Gram gather / load and the P-block solve
    redundantly (identical on every rank: the measured one-GPU times);
  * runs the two f-update passes over its n / P rows (measured time / P);
  * pays the launch gaps of the round graph (measured);
  * waits for three collectives: the candidate all-gather (tiny), the sum
    all-reduce of the P sub-Grams + members' f (blocks x (q^2 + 192) floats),
    the line-search partials all-gather (tiny) — ASSUMED latency L each plus
    the all-reduce's ring traffic 2 (P - 1) / P x bytes at an ASSUMED bus
    bandwidth B.
plus the rank's Gram slab K(all rows, n / P columns) (measured at P = 1..8).
The rounds are the one-GPU count (the trajectory is bit-identical at any
rank count: tests/test_ws_gpu.py sharded-vs-replicated tests).

  python bench/project_shard.py [inputs.json] [pass1_probe.jsonl]

With a pass-1 probe file (bench/pass1_probe.py: the multi-block f-update pass 1
measured alone at a rank's shard shape, 60000 x 60000 / P, with the workgroup
split the solver picks, ws_pass1_splits) pass 1 at P > 1 is that measurement
instead of the one-rank time / P — pass 1 does not divide by P (few selection
groups per rank: profiles/r3_pass1_probe.txt).
"""
import json
import sys

PASS1_US = 50.0   # f-update pass 1 at P = 1 when the inputs carry no stamp of it (round-2 value)
UNION = 6144      # rows per round (device_state.hpp kWsMaxAll); blocks of UNION / blocks rows, <= 192


def pass1_splits(G: int) -> int:
    return max(1, min(16, 256 // max(1, G)))  # kernels ws_pass1_splits


def pass1_v4_splits(p1G: int) -> int:
    return max(1, min(32, 256 // max(1, p1G)))  # kernels ws_pass1_v4_splits


def probe_pass1(path):
    """{P: pass-1 us} at the shard shapes of the probe, with the solver's split:
    the wide pass 1 (the default since round 5) when the probe holds it, else
    the selection-geometry pass 1"""
    wide, sel = {}, {}  # P -> (|ks - the solver's split|, us): the probed split nearest the solver's
    for line in open(path):
        r = json.loads(line)
        if r["rows"] != 60000:
            continue
        P = 60000 // r["cols"]
        if r.get("wide"):
            d = abs(r["ks"] - pass1_v4_splits(r["p1G"]))
            if P not in wide or d < wide[P][0]:
                wide[P] = (d, r["pass1_us_median"])
        else:
            d = abs(r["ks"] - pass1_splits(r["G"]))
            if P not in sel or d < sel[P][0]:
                sel[P] = (d, r["pass1_us_median"])
    return {P: v[1] for P, v in (wide or sel).items()}


def main() -> int:
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("inputs", nargs="?", default="profiles/r3_shard_projection_inputs_1gpu.json")
    ap.add_argument("probe", nargs="?", default=None)
    ap.add_argument("--rehearsal", action="append", default=[],
                    help="P:path of a bench/shard_stamps.py JSON of a P-rank run sharing ONE GPU: its measured "
                         "exchange consumer cost per round replaces the assumed xGMI latency for that P")
    a = ap.parse_args()
    path = a.inputs
    probe = probe_pass1(a.probe) if a.probe else {}
    reh = {}
    for spec in a.rehearsal:
        P, f = spec.split(":", 1)
        reh[int(P)] = json.load(open(f))
    m = json.load(open(path))
    r = m["round_us"]
    rounds = m["local"]["rounds"]
    blocks = m["local"]["blocks"][0]
    q = min(192, UNION // max(1, blocks)) if blocks > 1 else 192
    ar_bytes = blocks * (q * q + 192) * 4
    fixed = r["merge"] + r["gather"] + r["load_subgram"] + r["solve"]
    pass1 = r.get("pass1_start_to_pass2_start") or PASS1_US
    rows_part = pass1 + r["select_pass2"]
    if probe:
        print(f"  pass 1 measured at the shard shapes (bench/pass1_probe.py): {probe} us; one rank {pass1:.1f} us")
    gaps = max(0.0, r["period"] - fixed - rows_part)
    print(f"inputs: {path}")
    print(f"  measured: rounds {rounds}, round period {r['period']} us = redundant {fixed:.1f} (merge, gather, "
          f"load, solve) + row passes {rows_part:.1f} + launch gaps {gaps:.1f}; one-rank RCCL launch cost "
          f"{m['rccl_one_rank']['extra_us_per_round']} us/round")
    print(f"  measured Gram slab (s): {m['gram_slab_s']};  local solve {m['local']['s']} s")
    print(f"  sub-Gram all-reduce: {ar_bytes / 1e6:.2f} MB per round")
    print("PROJECTION (assumed xGMI collective cost: latency L per collective, all-reduce bus bandwidth B)")
    print(f"{'L us':>6} {'B GB/s':>7} | " + " | ".join(f"P={p:<2d} s" for p in (1, 2, 4, 8)))
    for L, B in ((5, 100), (10, 64), (20, 40)):
        row = []
        for P in (1, 2, 4, 8):
            gram = m["gram_slab_s"][str(P)]
            if P == 1:
                row.append(m["local"]["s"])
                continue
            coll = 3 * L + 2 * (P - 1) / P * ar_bytes / (B * 1e3)  # bytes / (GB/s) -> us
            p1 = probe.get(P, pass1 / P)
            per_round = fixed + p1 + r["select_pass2"] / P + gaps + coll
            row.append(gram + rounds * per_round * 1e-6)
        print(f"{L:>6} {B:>7} | " + " | ".join(f"{v:.4f}  " for v in row))
    px = m.get("peer_loopback")
    if px:
        # the default at world > 1: no collective per round.  MEASURED on one GPU:
        # the exchange's kernel cost per round (loopback: pushes, two collect
        # launches, the solve's polled loads).  ASSUMED: the extra latency of a
        # store crossing xGMI before the consumer's poll sees it (three exchange
        # points per round: candidates, sub-Gram rows, partials) and the link
        # bandwidth for the pushed bytes (each rank sends its owned share of the
        # P sub-Grams to every peer: ~ entries / P x (P - 1) x 8 B per link set)
        ext = px["extra_us_per_round"]
        sub_entries = blocks * q * q
        print(f"PEER EXCHANGE (default): measured loopback cost {ext} us/round "
              f"(same trajectory: {px['same_trajectory']}); ASSUMED xGMI store-to-poll latency X per exchange point "
              f"(3 per round) and per-GPU injection bandwidth W for the pushed granules")
        print(f"{'X us':>6} {'W GB/s':>7} | " + " | ".join(f"P={p:<2d} s" for p in (1, 2, 4, 8)))
        for X, W in ((2, 300), (4, 150), (8, 64)):
            row = []
            for P in (1, 2, 4, 8):
                if P == 1:
                    row.append(m["local"]["s"])
                    continue
                sent = sub_entries / P * (P - 1) * 8  # bytes a rank pushes to its peers
                xfer = 3 * X + sent / (W * 1e3)
                p1 = probe.get(P, pass1 / P)
                per_round = fixed + p1 + r["select_pass2"] / P + gaps + max(0.0, ext) + xfer
                row.append(m["gram_slab_s"][str(P)] + rounds * per_round * 1e-6)
            print(f"{X:>6} {W:>7} | " + " | ".join(f"{v:.4f}  " for v in row))
    if reh:
        # MEASURED on ONE GPU with P ranks sharing it (bench/shard_stamps.py): the
        # exchange consumers' time per round (candidate collect, partials collect,
        # the solve's sub-Gram poll + load) — they wait for every rank's pushes,
        # and on one device also for the other ranks' kernels: an upper bound of
        # the exchange cost across P GPUs
        print("PEER EXCHANGE, consumer cost per round MEASURED in one-GPU rehearsals (upper bound; no assumed latency)")
        row = []
        for P in (1, 2, 4, 8):
            if P == 1:
                row.append(f"{m['local']['s']:.4f}")
                continue
            if P not in reh:
                row.append("   -   ")
                continue
            exch = reh[P]["exchange_consumer_us_per_round"]
            p1 = probe.get(P, pass1 / P)
            per_round = fixed - r["load_subgram"] + p1 + r["select_pass2"] / P + gaps + exch
            row.append(f"{m['gram_slab_s'][str(P)] + rounds * per_round * 1e-6:.4f}")
        print(f"{'':>14} | " + " | ".join(f"P={p} {v}" for p, v in zip((1, 2, 4, 8), row)))
        for P, d in sorted(reh.items()):
            print(f"  P={P}: consumer cost {d['exchange_consumer_us_per_round']} us/round "
                  f"(median over {d['ranks']} ranks: {d['median_over_ranks']})")
    return 0


if __name__ == "__main__":
    sys.exit(main())
