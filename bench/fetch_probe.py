"""FETCH_SIZE pinned against a known-bytes stream.

`run`: under `rocprofv3 --kernel-trace --pmc FETCH_SIZE`, (1) the row_sqnorm
kernel (setup_kernels.hip) over a 2 GiB fp32 matrix, each byte read exactly once
(8x the 256 MB Infinity Cache: every line comes from HBM), three dispatches;
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
    x = torch.rand(PROBE_ROWS, PROBE_D, device="cuda")
    out = torch.empty(PROBE_ROWS, device="cuda")
    for _ in range(PROBE_REPS):
        C.k_row_sqnorm(x.data_ptr(), PROBE_ROWS, PROBE_D, PROBE_D, out.data_ptr(), s)
    torch.cuda.synchronize()
    ref = (x.double() ** 2).sum(1).float()
    assert torch.allclose(out, ref, rtol=1e-4), "probe kernel wrong"
    del x, out, ref
    torch.cuda.empty_cache()
    X, y = synthetic("mnist", n=60000, seed=0)
    clf = SVC(C=10.0, gamma=0.25, eps=1e-3, device="cuda").fit(X, y)
    print(json.dumps({"probe_bytes_per_dispatch": PROBE_ROWS * PROBE_D * 4, "probe_dispatches": PROBE_REPS,
                      "headline_rounds": clf.n_rounds_, "headline_converged": bool(clf.converged_),
                      "iteration": clf.setup_info_["iteration"]}))


def _short(name):
    return name.split("(")[0].replace("void ", "").replace("dpsvm::dev::", "").strip()


def report(root):
    files = sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True))
    assert files, f"no counter_collection.csv under {root}"
    kib = defaultdict(float)
    ns = defaultdict(dict)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != "FETCH_SIZE":
                continue
            k = _short(r.get("Kernel_Name", "?"))
            kib[k] += float(r["Counter_Value"])
            ns[k][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    probe = next(k for k in kib if k.startswith("row_sqnorm_kernel"))
    n_probe = len(ns[probe])
    logical = PROBE_ROWS * PROBE_D * 4 * n_probe
    counted = kib[probe] * 1024
    scale = counted / logical
    print(f"# FETCH_SIZE vs a known-bytes stream (row_sqnorm over {PROBE_ROWS} x {PROBE_D} fp32, {n_probe} dispatches,"
          f" each byte read once, 8x the Infinity Cache)")
    print(f"probe: logical {logical / 1e9:.3f} GB, FETCH_SIZE x 1 KiB = {counted / 1e9:.3f} GB -> scale {scale:.3f}"
          f" (counter / true bytes)")
    print(f"{'kernel':48s} {'calls':>5s} {'counter GB':>11s} {'true GB':>9s} {'time ms':>9s} {'true TB/s':>9s}")
    for k in sorted(kib, key=lambda k: -kib[k]):
        t = sum(ns[k].values()) / 1e6
        c = kib[k] * 1024 / 1e9
        tb = c / scale
        print(f"{k[:48]:48s} {len(ns[k]):5d} {c:11.3f} {tb:9.3f} {t:9.3f} {tb / t if t > 0 else 0:9.2f}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "report":
        report(sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/fetch")
    else:
        run()
