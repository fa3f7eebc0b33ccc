"""Persistent-engine run for rocprofv3 --pmc diagnostics (bench/gpu_tlb_pmc.sh notes):
prints OK <engine> <iterations> or ERR <message>."""
import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
from dpsvm_amd import SVC
from dpsvm_amd.utils.datasets import synthetic
big = len(sys.argv) > 1 and sys.argv[1] == "mnist"
X, y = synthetic("mnist", n=60000, seed=0) if big else synthetic("blobs", n=4000, d=16, seed=1, sep=1.0)
try:
    kw = dict(C=10.0, gamma=0.25) if big else dict(C=1.0, gamma=0.1)
    c = SVC(device="cuda", persist=os.environ.get("PERSIST", "on"), verbose=True, **kw).fit(X, y)
    print("OK", c.setup_info_["iteration"], c.n_iter_)
except Exception as e:
    print("ERR", e)
