"""Adaptive split Gram (rbf_gemm_split.hip: rbf_gemm_split_h1s_kernel + the
w64p hot-tile pass; docs/DESIGN.md §13): the one-product value where
split_cold proves it within tau of the three-product one, the three-product
value elsewhere.  Checked here against the three-product kernel (every element
within tau), against float64 (within the split GEMM's own bound), across
tilings (the symmetric Gram and its column slabs store the same bits) and in a
solve (same b / decisions as the three-product Gram).
Reference: the kernel rows these replace, svmTrain.cu:212-249 (cuBLAS Sgemv + exp).
"""
import numpy as np
import pytest
import torch

from dpsvm_amd.utils.datasets import synthetic

pytestmark = pytest.mark.gpu

TAU = 2.0 ** -22


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dpsvm_amd.ops import kernels

    return kernels


def _data(n, seed=0, dups=12):
    """MNIST-shape rows (every off-diagonal K tiny) plus near-duplicates of a
    few rows far apart in the order, so some off-diagonal tiles hold hot
    elements (K near 1) and most do not."""
    X, _ = synthetic("mnist", n=n, seed=seed)
    X = X.copy()
    rng = np.random.default_rng(seed)
    src = rng.choice(n // 2, dups, replace=False)
    dst = n // 2 + rng.choice(n // 2, dups, replace=False)
    X[dst] = np.clip(X[src] + 0.01 * rng.standard_normal(X[src].shape).astype(np.float32), 0, 1)
    return X


def _ref64(a, b, gamma):
    a = a.astype(np.float64)
    b = b.astype(np.float64)
    d2 = (a * a).sum(1)[:, None] + (b * b).sum(1)[None, :] - 2 * a @ b.T
    return np.exp(-gamma * np.maximum(d2, 0))


@pytest.mark.parametrize("n,d", [(3000, 784), (2333, 300), (1500, 1024)])
def test_adaptive_gram_within_tau_of_three_product(K, n, d):
    X = _data(n)
    if d != X.shape[1]:
        X = np.ascontiguousarray(np.resize(X, (n, d)))
    x = torch.from_numpy(X).cuda()
    g = 0.25 * 784 / d
    k3 = K.rbf_gram(x, None, g, split=True)
    assert K.gram_adapt_last() == (-1, -1)
    ka = K.rbf_gram(x, None, g, split=True, cold_tau=TAU)
    tiles, hot = K.gram_adapt_last()
    assert tiles > 0 and 0 < hot < tiles, (tiles, hot)
    diff = (ka - k3).abs()
    assert torch.isfinite(ka).all()
    assert diff.max().item() <= TAU, diff.max().item()
    assert torch.equal(ka.diagonal(), k3.diagonal())
    # hot elements (the near-duplicates) keep the three-product bits
    big = k3 > 1e-3
    assert torch.equal(ka[big], k3[big])
    # symmetric bit for bit (the rule reads only symmetric quantities)
    assert torch.equal(ka, ka.T)
    # and vs float64 within the three-product kernel's own error plus tau
    sub = np.random.default_rng(1).choice(n, 512, replace=False)
    ref = _ref64(X[sub], X, g)
    e3 = np.abs(k3[torch.from_numpy(sub).cuda()].double().cpu().numpy() - ref).max()
    ea = np.abs(ka[torch.from_numpy(sub).cuda()].double().cpu().numpy() - ref).max()
    assert ea <= e3 + TAU, (ea, e3)


def test_adaptive_gram_slabs_equal_symmetric(K):
    """A rank's slab K(all rows, its columns) — the sharded Gram — holds the
    symmetric adaptive Gram's bits whatever the tiles that computed them."""
    n = 2600
    X = _data(n, seed=3)
    x = torch.from_numpy(X).cuda()
    ka = K.rbf_gram(x, None, 0.25, split=True, cold_tau=TAU)
    for c0, c1 in ((0, 650), (650, 1300), (1300, 2600), (777, 1111)):
        slab = K.rbf_gram(x, x[c0:c1].contiguous(), 0.25, split=True, cold_tau=TAU)
        assert torch.equal(slab, ka[:, c0:c1]), (c0, c1)


def test_adaptive_gram_all_cold_and_all_hot(K):
    """No near-duplicates: only tiles touching the diagonal are hot.  gamma
    tiny (every K near 1): every tile hot, the result is the three-product Gram."""
    n = 2048
    X, _ = synthetic("mnist", n=n, seed=5)
    x = torch.from_numpy(X).cuda()
    ka = K.rbf_gram(x, None, 0.25, split=True, cold_tau=TAU)
    tiles, hot = K.gram_adapt_last()
    k3 = K.rbf_gram(x, None, 0.25, split=True)
    assert (ka - k3).abs().max().item() <= TAU
    assert hot <= n // 128 + 1, (tiles, hot)  # one upper tile per 128-column block meets the diagonal
    ka = K.rbf_gram(x, None, 1e-4, split=True, cold_tau=TAU)
    tiles, hot = K.gram_adapt_last()
    assert hot == tiles
    assert torch.equal(ka, K.rbf_gram(x, None, 1e-4, split=True))


def test_adaptive_gram_in_ws_solve_matches_three_product():
    """ws-dense with the adaptive resident Gram (auto on MNIST-shape data) vs
    gram_adapt off: both converged (the Gram's last-bit changes move the
    trajectory, so b agrees to the stop tolerance, 2 eps), the same decisions."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dpsvm_amd import SVC

    X, y = synthetic("mnist", n=20000, seed=7)
    kw = dict(C=10.0, gamma=0.25, eps=1e-3, device="cuda", solver="ws")
    on = SVC(**kw).fit(X, y)
    off = SVC(gram_adapt="off", **kw).fit(X, y)
    assert on.setup_info_["gram"] == "split-f16-adaptive"
    assert off.setup_info_["gram"] == "split-f16"
    assert on.stats_["gram_hot_tiles"] >= 0 and on.stats_["gram_tiles"] > on.stats_["gram_hot_tiles"]
    assert on.stats_["converged"] and off.stats_["converged"]
    assert abs(on.b_ - off.b_) <= 2e-3
    Xt, _ = synthetic("mnist", n=2000, seed=8)
    assert (np.sign(on.decision_function(Xt)) == np.sign(off.decision_function(Xt))).mean() >= 0.999


def test_adaptive_gram_beyond_2_32_elements(K):
    """More than 2^32 Gram elements (66,000 rows: 17.4 GB): the adaptive
    kernels index tiles from 64-bit bases (rbf_gemm_store_split's idx_adapt).
    Rows past element 2^32 match the three-product Gram within tau."""
    free, _ = torch.cuda.mem_get_info()
    if free < 48 << 30:
        pytest.skip("needs ~40 GB of free device memory")
    n = 66000
    X, _ = synthetic("mnist", n=n, seed=9)
    x = torch.from_numpy(X).cuda()
    ka = K.rbf_gram(x, None, 0.25, split=True, cold_tau=TAU)
    tiles, hot = K.gram_adapt_last()
    assert tiles > 0 and 0 < hot < tiles
    rows = torch.arange(n - 2048, n, device="cuda")  # past row 2^32 / ld ~ 65,000
    top = ka[rows].clone()
    del ka
    torch.cuda.empty_cache()
    k3 = K.rbf_gram(x, None, 0.25, split=True)
    assert (top - k3[rows]).abs().max().item() <= TAU
    assert torch.isfinite(top).all()
