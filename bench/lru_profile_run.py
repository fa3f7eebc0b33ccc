#!/usr/bin/env python3
"""One cache-mode solve (for rocprofv3 kernel traces / DPSVM_STAMPS).
usage: lru_profile_run.py [spec=14] [max_iter=20000] [data=mnist] [n=60000] [lines=20000] [C] [gamma]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
from dpsvm_amd import SVCConfig  # noqa: E402
from dpsvm_amd._native import load  # noqa: E402
from dpsvm_amd.utils.datasets import synthetic  # noqa: E402

argv = sys.argv[1:] + [None] * 8
spec = int(argv[0] or 14)
max_iter = int(argv[1] or 20000)
data = argv[2] or "mnist"
n = int(argv[3] or 60000)
lines = int(argv[4] or 20000)
Cc = float(argv[5] or (2048.0 if data == "covtype" else 10.0))
gamma = float(argv[6] or (0.03125 if data == "covtype" else 0.25))
C = load()
X, y = synthetic(data, n=n, seed=0)
cfg = SVCConfig(C=Cc, gamma=gamma, eps=1e-3, cache_lines=lines, spec_rows=spec, max_iter=max_iter)
s = C.GpuSolver(cfg.to_native(X.shape[1]), None, 0)
print(s.setup(X, X.shape[0], y))
_, info = s.solve()
print({k: info[k] for k in ("iters", "t_solve", "x_passes", "rows_computed", "cache_misses", "spec_rows")})
print("us/iter", 1e6 * info["t_solve"] / max(1, info["iters"]))
