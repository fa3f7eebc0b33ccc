"""Debug: ws-cache exact-gradient gap on well-separated blobs at several n."""
import sys, os
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dpsvm_amd import SVC
from dpsvm_amd.utils.datasets import synthetic


def gap_of(X, y, alpha, C_, g):
    n = X.shape[0]
    yy = torch.tensor(np.where(y > 0, 1.0, -1.0), device="cuda", dtype=torch.float64)
    a = torch.tensor(alpha, device="cuda", dtype=torch.float64)
    Xd = torch.tensor(X, device="cuda", dtype=torch.float64)
    sv = torch.nonzero(a > 0).flatten()
    coef = a[sv] * yy[sv]
    f = torch.empty(n, device="cuda", dtype=torch.float64)
    for i in range(0, n, 1 << 16):
        k = torch.exp(-g * torch.cdist(Xd[i:i + (1 << 16)], Xd[sv]) ** 2)
        f[i:i + (1 << 16)] = k @ coef - yy[i:i + (1 << 16)]
    up = ((a == 0) & (yy == 1)) | ((a == C_) & (yy != 1)) | ((a > 0) & (a < C_))
    lo = ((a == 0) & (yy != 1)) | ((a == C_) & (yy == 1)) | ((a > 0) & (a < C_))
    return float(f[lo].max() - f[up].min()), f


for arg in sys.argv[1:]:
    n, extra = int(arg.split(":")[0]), arg.split(":")[1:] 
    X, y = synthetic("blobs", n=n, d=8, seed=3, sep=10.0)
    kw = dict(C=1.0, gamma=0.125, eps=1e-3, device="cuda", max_iter=200000)
    if "cache" in extra:
        kw.update(force_cache=True, cache_lines=4000)
    for solver in ("ws", "smo"):
        s = SVC(solver=solver, **kw).fit(X, y)
        gap, f = gap_of(X, y, s.alpha_, 1.0, 0.125)
        print(n, extra, solver, s.setup_info_["iteration"], s.setup_info_["rows_per_group"], "conv", s.converged_,
              "iters", s.n_iter_, "rounds", s.n_rounds_, "b", round(s.b_, 5), "nsv", s.n_support_,
              "bhi", s.stats_.get("b_hi"), "blo", s.stats_.get("b_lo"), "EXACT GAP", round(gap, 5), flush=True)
