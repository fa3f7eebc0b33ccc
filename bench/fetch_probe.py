"""FETCH_SIZE pinned against a known-bytes stream.

`run`: under `rocprofv3 --kernel-trace --pmc FETCH_SIZE`, (1) two known-bytes
streams over a 2 GiB buffer, each byte read exactly once (8x the 256 MB Infinity
Cache: every line comes from HBM), three dispatches each: stream_read
(microbench.hip, 16-B loads) and row_sqnorm (setup_kernels.hip, 4-B loads);
(2) one headline solve (MNIST-shape 60000 x 784, C=10, gamma=0.25, ws-dense):
the split Gram GEMM and the rounds' pass 1.

`report DIR`: per kernel, FETCH_SIZE (KiB summed over dispatches, as rocprofv3
reports it) against the probe's known bytes gives the counter's scale on this
device; the Gram's and pass 1's fetched bytes and rates are then reported in
true bytes (counter / scale).  FETCH_SIZE counts what the L2s fetch over the
fabric (Infinity Cache hits included), so for a kernel whose lines are re-read
through the MALL it is an upper bound of its HBM bytes.

    rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/fetch -o run -- \\
        python3 bench/fetch_probe.py run
    python3 bench/fetch_probe.py report gpurun_out/fetch
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE_ROWS, PROBE_D, PROBE_REPS = 262144, 2048, 3  # 2 GiB of fp32, read once per dispatch


def run():
    sys.path.insert(0, ROOT)
    import torch

    from dpsvm_amd import SVC
    from dpsvm_amd._native import load
    from dpsvm_amd.utils.datasets import synthetic

    C = load()
    s = torch.cuda.current_stream().cuda_stream
    nbytes = PROBE_ROWS * PROBE_D * 4
    x = torch.empty(nbytes // 4, device="cuda")  # contents irrelevant: no fill kernel in the profile
    out = torch.empty(PROBE_ROWS, device="cuda")
    for _ in range(PROBE_REPS):  # 16-B loads, each chunk once (the shape of pass 1 / the GEMMs' LDS-DMA)
        C.k_stream_read(x.data_ptr(), nbytes, out.data_ptr(), 2048, s)
    for _ in range(PROBE_REPS):  # 4-B loads, one wave per 8-KiB row
        C.k_row_sqnorm(x.data_ptr(), PROBE_ROWS, PROBE_D, PROBE_D, out.data_ptr(), s)
    torch.cuda.synchronize()
    del x, out
    torch.cuda.empty_cache()
    X, y = synthetic("mnist", n=60000, seed=0)
    clf = SVC(C=10.0, gamma=0.25, eps=1e-3, device="cuda").fit(X, y)
    print(json.dumps({"probe_bytes_per_dispatch": nbytes, "probe_dispatches": PROBE_REPS,
                      "headline_rounds": clf.n_rounds_, "headline_converged": bool(clf.converged_),
                      "iteration": clf.setup_info_["iteration"]}))


def _short(name):
    return name.split("(")[0].replace("void ", "").replace("dpsvm::dev::", "").strip()


def report(root):
    files = sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True))
    assert files, f"no counter_collection.csv under {root}"
    kib = defaultdict(float)
    ns = defaultdict(dict)
    per = defaultdict(lambda: defaultdict(float))  # kernel -> dispatch -> KiB
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != "FETCH_SIZE":
                continue
            k = _short(r.get("Kernel_Name", "?"))
            kib[k] += float(r["Counter_Value"])
            per[k][r["Dispatch_Id"]] += float(r["Counter_Value"])
            ns[k][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    logical_per = PROBE_ROWS * PROBE_D * 4
    scales = {}
    print(f"# FETCH_SIZE vs known-bytes streams ({logical_per / 2**30:.0f} GiB per dispatch, each byte read once,"
          f" 8x the Infinity Cache): the counter's scale per access shape")
    for name, label in (("stream_read_kernel", "16-B loads (pass-1 / LDS-DMA shape)"),
                        ("row_sqnorm_kernel", "4-B loads, one wave per 8-KiB row")):
        k = next((k for k in kib if k.startswith(name)), None)
        if k is None:
            continue
        # the probe's dispatches: the PROBE_REPS largest (the solver's setup runs row_sqnorm on X too)
        ids = sorted(per[k], key=lambda i: -per[k][i])[:PROBE_REPS]
        logical = logical_per * len(ids)
        counted = sum(per[k][i] for i in ids) * 1024
        scales[name] = counted / logical
        t = sum(ns[k][i] for i in ids) / 1e6
        print(f"probe {name} ({label}): logical {logical / 1e9:.3f} GB in {t:.3f} ms ({logical / t / 1e9:.2f} TB/s),"
              f" FETCH_SIZE x 1 KiB = {counted / 1e9:.3f} GB -> scale {scales[name]:.3f}")
    scale = scales.get("stream_read_kernel") or next(iter(scales.values()))
    print(f"# kernels in true bytes with the 16-B stream's scale {scale:.3f} (FETCH_SIZE counts L2 fills over the"
          f" fabric: Infinity Cache hits included)")
    print(f"{'kernel':48s} {'calls':>5s} {'counter GB':>11s} {'true GB':>9s} {'time ms':>9s} {'true TB/s':>9s}")
    for k in sorted(kib, key=lambda k: -kib[k]):
        if kib[k] * 1024 < 1e7:
            continue
        t = sum(ns[k].values()) / 1e6
        c = kib[k] * 1024 / 1e9
        tb = c / scale
        print(f"{k[:48]:48s} {len(ns[k]):5d} {c:11.3f} {tb:9.3f} {t:9.3f} {tb / t if t > 0 else 0:9.2f}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "report":
        report(sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/fetch")
    else:
        run()
