"""The adaptive split Gram's element rule (docs/DESIGN.md §13, split_cold in
kernels/split_util.hpp), checked on the CPU: the split-operand arithmetic is
emulated in float64 (rows scaled by 2^s, fp16 hi / lo planes as
split_rows_kernel builds them) and every pair the rule calls cold must have
|K_one_product - K_three_product| <= tau.  This pins the bound's derivation
(the constants come from the native module, `split_cold_consts`); the GPU
tests (test_gram_adapt_gpu.py) pin the kernels' bits against it.
Reference: the kernel values the Gram replaces, svmTrain.cu:212-249.
"""
import math

import numpy as np
import pytest

TAU = 2.0 ** -22


def _consts(gamma, tau):
    from dpsvm_amd._native import load

    return load().split_cold_consts(gamma, tau)


def _split(x):
    """split_rows_kernel: largest |x| scaled into [2^14, 2^15), h = fp16, l = fp16(rest)."""
    m = np.abs(x).max(axis=1)
    e = np.zeros(len(x), dtype=np.int64)
    nz = m > 0
    e[nz] = np.frexp(m[nz])[1]
    s = np.where(nz, 15 - e, 0)
    xs = np.ldexp(x.astype(np.float32), s[:, None].astype(np.int32)).astype(np.float32)
    h = xs.astype(np.float16)
    l = (xs - h.astype(np.float32)).astype(np.float16)
    return h.astype(np.float64), l.astype(np.float64), s


def _pairs(x, gamma, tau):
    h, l, s = _split(x)
    sc = np.ldexp(1.0, -(s[:, None] + s[None, :]))
    dot1 = (h @ h.T) * sc
    dot3 = (h @ h.T + h @ l.T + l @ h.T) * sc
    sq = (x.astype(np.float64) ** 2).sum(1)
    d1 = np.maximum(sq[:, None] + sq[None, :] - 2 * dot1, 0)
    d3 = np.maximum(sq[:, None] + sq[None, :] - 2 * dot3, 0)
    k1, k3 = np.exp(-gamma * d1), np.exp(-gamma * d3)
    c0, c1 = _consts(gamma, tau)
    r = 0.5 * np.log2(np.maximum(sq, 1e-300))
    sr = r[:, None] + r[None, :]
    t1 = -gamma * d1 * math.log2(math.e)
    cold = (sr <= c1) & (t1 <= c0 - sr)
    return cold, np.abs(k1 - k3), k3


def _mnist_like(n, seed):
    rng = np.random.default_rng(seed)
    x = np.where(rng.random((n, 784)) < 0.19, rng.random((n, 784)), 0.0).astype(np.float32)
    dup = rng.choice(n, 8, replace=False)
    x[dup[4:]] = np.clip(x[dup[:4]] + 0.01 * rng.standard_normal((4, 784)), 0, 1).astype(np.float32)
    return x


@pytest.mark.parametrize("data,gamma", [("mnist", 0.25), ("mnist", 0.02), ("gauss", 0.01), ("wide", 1e-3)])
def test_split_cold_rule_bound_holds(data, gamma):
    rng = np.random.default_rng(7)
    if data == "mnist":
        x = _mnist_like(600, 3)
    elif data == "gauss":
        x = rng.standard_normal((500, 300)).astype(np.float32)
    else:  # rows of very different scales
        x = (rng.standard_normal((500, 128)) * np.exp(rng.uniform(-6, 6, (500, 1)))).astype(np.float32)
    cold, diff, k3 = _pairs(x, gamma, TAU)
    assert diff[cold].max(initial=0.0) <= TAU
    # (how many pairs are cold depends on the data: none for mnist at gamma 0.02, K ~ 0.2 everywhere)


def test_split_cold_rule_separates_the_headline_shape():
    """MNIST-shape rows at gamma 0.25: every off-diagonal pair but the
    near-duplicates is cold (the one-product pass keeps them); the
    near-duplicates and the diagonal are hot."""
    x = _mnist_like(600, 5)
    cold, diff, k3 = _pairs(x, 0.25, TAU)
    off = ~np.eye(len(x), dtype=bool)
    assert cold[off].mean() > 0.99
    assert (~cold[k3 > 1e-3]).all()
    assert diff[cold].max() <= TAU


def test_split_cold_consts():
    g = 0.25
    c0, c1 = _consts(g, TAU)
    e = 4.5 * 2.0 ** -11 * g
    assert c1 == pytest.approx(-math.log2(e), rel=1e-6)
    assert c0 == pytest.approx(math.log2(TAU) - math.log2(1.72 * e) - 0.01, rel=1e-6)
