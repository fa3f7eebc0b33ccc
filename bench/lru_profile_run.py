#!/usr/bin/env python3
"""One cache-mode solve (for rocprofv3 kernel traces): MNIST shape, 20k lines."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
from dpsvm_amd import SVCConfig  # noqa: E402
from dpsvm_amd._native import load  # noqa: E402
from dpsvm_amd.utils.datasets import synthetic  # noqa: E402

spec = int(sys.argv[1]) if len(sys.argv) > 1 else 14
max_iter = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
C = load()
X, y = synthetic("mnist", n=60000, seed=0)
cfg = SVCConfig(C=10.0, gamma=0.25, eps=1e-3, cache_lines=20000, spec_rows=spec, max_iter=max_iter)
s = C.GpuSolver(cfg.to_native(X.shape[1]), None, 0)
print(s.setup(X, X.shape[0], y))
_, info = s.solve()
print({k: info[k] for k in ("iters", "t_solve", "x_passes", "rows_computed", "cache_misses", "spec_rows")})
