"""The fp16 split-operand RBF GEMM (kernels/rbf_gemm_split.hip) vs a float64
reference and vs the f32-MFMA GEMM (rbf_gemm.hip): same accuracy class, and
bit-identical values under operand swap (symmetric Gram == full Gram ==
indexed rows), which the sharded and cache-mode working-set engines rely on."""
import numpy as np
import pytest
import torch

from dpsvm_amd.utils.datasets import synthetic

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dpsvm_amd.ops import kernels

    return kernels


def _ref(a, b, gamma):
    a = a.astype(np.float64)
    b = b.astype(np.float64)
    d2 = (a * a).sum(1)[:, None] + (b * b).sum(1)[None, :] - 2 * a @ b.T
    return np.exp(-gamma * np.maximum(d2, 0))


@pytest.mark.parametrize("name,n,d,gamma", [("mnist", 1500, 784, 0.25), ("covtype", 1300, 54, 0.5),
                                            ("blobs", 700, 1100, 1.0 / 1100)])
def test_split_gram_matches_float64_like_f32_kernel(K, name, n, d, gamma):
    kw = dict(n=n, seed=3, d=d) if name == "blobs" else dict(n=n, seed=3)
    X, _ = synthetic(name, **kw)
    x = torch.from_numpy(X).cuda()
    ref = _ref(X, X, gamma)
    k32 = K.rbf_gram(x, None, gamma).cpu().numpy()
    k16 = K.rbf_gram(x, None, gamma, split=True).cpu().numpy()
    e32 = np.abs(k32 - ref).max()
    e16 = np.abs(k16 - ref).max()
    assert e16 <= max(3 * e32, 2e-6), (e16, e32)
    assert np.isfinite(k16).all()


def test_split_gram_operand_swap_bit_identical(K):
    X, _ = synthetic("mnist", n=1000, seed=4)
    Y, _ = synthetic("mnist", n=777, seed=5)
    x, yv = torch.from_numpy(X).cuda(), torch.from_numpy(Y).cuda()
    sym = K.rbf_gram(x, None, 0.25, split=True)
    full = K.rbf_gram(x, x.clone(), 0.25, split=True)
    assert torch.equal(sym, full)
    assert torch.equal(sym, sym.T)
    ab = K.rbf_gram(x, yv, 0.25, split=True)
    ba = K.rbf_gram(yv, x, 0.25, split=True)
    assert torch.equal(ab, ba.T)


@pytest.mark.parametrize("extra", [0, 340])
def test_split_rows_indexed_equals_split_gram_rows(K, extra):
    """The ws-cache row GEMM gives the Gram's rows bit for bit, for a partial
    192-row tile and (extra) several tile rows."""
    X, _ = synthetic("mnist", n=1200, seed=6)
    x = torch.from_numpy(X).cuda()
    full = K.rbf_gram(x, None, 0.25, split=True)
    rows = [5, 1199, 0, 640, 641, 77, 333, 1024] + list(range(100, 160)) + list(range(700, 700 + extra))
    lines = list(range(len(rows)))[::-1]
    got = K.rbf_rows_indexed(x, rows, 0.25, out_lines=lines, split=True)
    for r, ln in zip(rows, lines):
        assert torch.equal(got[ln], full[r]), r


def test_split_gram_extreme_row_scales(K):
    rng = np.random.default_rng(7)
    X = rng.standard_normal((300, 40)).astype(np.float32)
    X[0] = 0.0                      # zero row
    X[1] *= 1e-20                   # tiny row
    X[2] *= 1e15                    # huge row
    X[3, :5] = [1e6, 1e-6, -3.0, 0.0, 2.5e-30]  # wide range inside a row
    x = torch.from_numpy(X).cuda()
    g = 1e-3
    k16 = K.rbf_gram(x, None, g, split=True).cpu().numpy()
    k32 = K.rbf_gram(x, None, g).cpu().numpy()
    ref = _ref(X, X, g)
    assert np.isfinite(k16).all()
    assert np.abs(k16 - ref).max() <= max(3 * np.abs(k32 - ref).max(), 2e-6)
    assert k16[0, 0] == 1.0 and k16[1, 1] == 1.0


@pytest.mark.parametrize("n,m,d", [(1000, 777, 784), (4133, 2300, 300), (2600, 129, 1024)])
def test_split_gram_persistent_bit_identical_to_tile_kernel(K, n, m, d):
    """The LDS-DMA STORE GEMMs (tile per workgroup, persistent) run the
    register-staged tile kernel's MFMA sequence per tile: the same bits,
    symmetric (upper tiles + mirrored stores) and plain, with partial edge tiles."""
    from dpsvm_amd._native import load

    C = load()
    rng = np.random.default_rng(n)
    x = torch.from_numpy(rng.random((n, d), dtype=np.float32)).cuda()
    y = torch.from_numpy(rng.standard_normal((m, d), dtype=np.float32)).cuda()
    g = 1.0 / d
    try:
        C.k_set_split_gemm_variant(1)
        ref_sym, ref_xy = K.rbf_gram(x, None, g, split=True), K.rbf_gram(x, y, g, split=True)
        got = {}
        for v in (3, 4, 5):  # LDS-DMA (three k blocks in flight); persistent LDS-DMA; wide-wave 256 x 128
            C.k_set_split_gemm_variant(v)
            got[v] = K.rbf_gram(x, None, g, split=True), K.rbf_gram(x, y, g, split=True)
    finally:
        C.k_set_split_gemm_variant(0)
    for v, (got_sym, got_xy) in got.items():
        assert torch.equal(got_sym, ref_sym), v
        assert torch.equal(got_xy, ref_xy), v
        assert torch.isfinite(got_sym).all() and torch.isfinite(got_xy).all()


def _split_model(X, dp):
    """numpy model of split_rows_kernel: shift to [2^14, 2^15), fp16 hi / lo planes"""
    rows, d = X.shape
    nkb = (dp + 31) // 32
    Xp = np.zeros((rows, nkb * 32), np.float32)
    Xp[:, :d] = X
    m = np.abs(X).max(1)
    e = np.frexp(m)[1]
    s = np.where((m > 0) & np.isfinite(m), 15 - e, 0).astype(np.int32)
    v = np.ldexp(Xp, s[:, None]).astype(np.float32)
    h = v.astype(np.float16)
    lo = (v - h.astype(np.float32)).astype(np.float16)
    planes = np.stack([h.reshape(rows, nkb, 32), lo.reshape(rows, nkb, 32)], axis=2)
    return planes, s


@pytest.mark.parametrize("d,ldx,offset", [(2200, 2208, 0), (1100, 1105, 0), (784, 784, 1), (3000, 3009, 3)])
def test_split_rows_long_and_unaligned_rows(K, d, ldx, offset):
    """split_rows_kernel beyond 2,048 columns (the loop that reloads from memory
    past the register-held chunks) and with an odd row stride / a base pointer
    off 16-B alignment (the element-by-element path): bit-identical to the
    numpy model of the split."""
    rng = np.random.default_rng(d + ldx + offset)
    rows = 37
    X = (rng.standard_normal((rows, d)) * np.exp(rng.uniform(-8, 8, (rows, 1)))).astype(np.float32)
    buf = np.zeros(offset + rows * ldx, np.float32)
    for r in range(rows):
        buf[offset + r * ldx: offset + r * ldx + d] = X[r]
    xt = torch.from_numpy(buf).cuda()
    dp = (d + 15) // 16 * 16
    planes, shift = K.split_rows(xt[offset:], rows, dp, ldx)
    want_p, want_s = _split_model(X, dp)
    np.testing.assert_array_equal(shift.cpu().numpy(), want_s)
    np.testing.assert_array_equal(planes.cpu().numpy().view(np.uint16), want_p.view(np.uint16))
