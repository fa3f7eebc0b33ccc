"""Dataset helpers: CSV / LIBSVM loading and the deterministic synthetic
generators of the reference's benchmark shapes (no datasets ship with the
reference — .MISSING_LARGE_BLOBS — and there is no network).

All heavy lifting is native (mmap + parallel from_chars parse; row-seeded
generators identical on every rank).
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np

from .._native import load

# name -> (n, d) of the reference's recorded configs (Makefile:74-86, BASELINE.json)
SHAPES = {
    "mnist": (60000, 784),          # MNIST even/odd, README.md:23
    "mnist-parity": (60000, 784),
    "mnist-test": (10000, 784),     # Makefile:80
    "adult": (32561, 123),          # a9a, Makefile:86
    "adult-test": (16281, 123),     # Makefile:83
    "covtype": (581012, 54),        # BASELINE.json; Makefile:77 used 500000
    "synthetic-2m": (2000000, 1024),
}


def synthetic(name: str = "mnist", n: Optional[int] = None, d: Optional[int] = None, seed: int = 0,
              row0: int = 0, rows: int = -1, sep: float = 2.0) -> Tuple[np.ndarray, np.ndarray]:
    """Generate (X float32 [rows, d], y float32 +/-1).

    name: mnist (pixel-like [0,1], ~19% nonzero, random labels — the BASELINE
    headline shape), mnist-parity (digit-like prototypes, label = parity),
    adult (123 binary one-hot features), covtype (10 continuous + 44 binary),
    blobs (two gaussians, centres +/- sep/2), uniform (dense [0,1)).
    ``row0``/``rows`` generate only a slice (a rank's shard) — identical to the
    same rows of the full set.
    """
    C = load()
    base = name.replace("-test", "")
    if n is None:
        n = SHAPES.get(name, (10000, 0))[0]
    if d is None:
        d = SHAPES.get(name, (0, 0))[1] or C.synth_default_d(base)
    return C.make_synthetic(base, int(n), int(d), int(seed), int(row0), int(rows), float(sep))


def read_csv(path: str, n: int = 0, d: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """Dense CSV 'label,f1..fd' (parse.cpp:10-43 semantics: first n rows)."""
    return load().read_csv(path, int(n), int(d), 0)


def read_csv_rows(path: str, row0: int, rows: int, d: int) -> Tuple[np.ndarray, np.ndarray]:
    return load().read_csv_rows(path, int(row0), int(rows), int(d))


def write_csv(path: str, X, y) -> None:
    load().write_csv(path, np.ascontiguousarray(X, dtype=np.float32), np.ascontiguousarray(y, dtype=np.float32))


def read_libsvm(path: str, d: int, n: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """Sparse LIBSVM text -> dense; feature k (1-based) -> column k-1."""
    return load().read_libsvm(path, int(d), int(n))
