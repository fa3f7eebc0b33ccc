"""HIP kernel numerics vs plain PyTorch fp32 references (GPU only)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dpsvm_amd.ops import kernels

    return kernels


def _rbf_ref(x, w, gamma):
    x64, w64 = x.double(), w.double()
    d2 = (x64 * x64).sum(1)[None, :] + (w64 * w64).sum(1)[:, None] - 2 * w64 @ x64.T
    return torch.exp(-gamma * d2.clamp_min(0))


def test_native_loaded_from_tree(K, C):
    import os

    from dpsvm_amd._native import is_loaded_from_tree

    assert is_loaded_from_tree()
    assert C.device_count() >= 1


@pytest.mark.parametrize("n,d", [(1, 3), (300, 17), (4097, 784), (1000, 1100)])
def test_row_sqnorm(K, n, d):
    x = torch.rand(n, d, device="cuda")
    got = K.row_sqnorm(x)
    ref = (x.double() ** 2).sum(1)
    assert torch.allclose(got.double(), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("nq", [1, 2, 5, 16])
@pytest.mark.parametrize("n,d,gamma", [(257, 13, 0.5), (3000, 784, 0.02), (1500, 2100, 0.001)])
def test_rbf_rows_mfma(K, nq, n, d, gamma):
    g = torch.Generator(device="cuda").manual_seed(nq * 7 + n)
    x = torch.rand(n, d, device="cuda", generator=g)
    w = torch.rand(nq, d, device="cuda", generator=g)
    w[0] = x[min(3, n - 1)]  # exact self-kernel: K = 1
    got = K.rbf_rows(x, w, gamma)
    ref = _rbf_ref(x, w, gamma)
    assert got.shape == (nq, n)
    assert torch.allclose(got.double(), ref, rtol=2e-4, atol=2e-5), (got.double() - ref).abs().max()
    assert abs(float(got[0, min(3, n - 1)]) - 1.0) < 1e-4


def test_rbf_rows_asymmetric_operands(K):
    # integer data: exact f32 arithmetic, catches swapped row/col maps
    n, d = 200, 32
    x = torch.randint(0, 3, (n, d), device="cuda").float()
    w = torch.randint(0, 3, (16, d), device="cuda").float()
    got = K.rbf_rows(x, w, 0.01)
    ref = _rbf_ref(x, w, 0.01)
    assert torch.allclose(got.double(), ref, rtol=1e-5, atol=1e-7)


def test_select_partials(K):
    from dpsvm_amd.ops.kernels import decode_key

    n, C_ = 5000, 2.0
    g = torch.Generator(device="cuda").manual_seed(0)
    f = torch.randn(n, device="cuda", generator=g)
    f[1234] = f[77] = -10.0  # tie across workgroups: lowest index must win
    y = torch.where(torch.rand(n, device="cuda", generator=g) > 0.5, 1.0, -1.0)
    a = torch.rand(n, device="cuda", generator=g) * C_
    a[torch.rand(n, device="cuda", generator=g) < 0.3] = 0.0
    a[torch.rand(n, device="cuda", generator=g) < 0.2] = C_
    y[77] = y[1234] = 1.0
    a[77] = a[1234] = 0.0
    part = K.select_partials(f, a, y, C_).cpu()
    kh = min(int(v) & (2**64 - 1) for v in part[:, 0].tolist())
    kl = min(int(v) & (2**64 - 1) for v in part[:, 1].tolist())
    up = ((a == 0) & (y == 1)) | ((a == C_) & (y != 1)) | ((a > 0) & (a < C_))
    lo = ((a == 0) & (y != 1)) | ((a == C_) & (y == 1)) | ((a > 0) & (a < C_))
    b_hi = float(torch.where(up, f, torch.inf).min())
    b_lo = float(torch.where(lo, f, -torch.inf).max())
    vh, ih = decode_key(kh)
    vl, il = decode_key(kl)
    assert vh == b_hi and ih == 77
    assert -vl == b_lo and float(f[il]) == b_lo and bool(lo[il])


@pytest.mark.parametrize("n,nsv,d", [(100, 1, 5), (2000, 3000, 784), (5000, 257, 54), (130, 129, 123)])
def test_rbf_decision_gemm(K, n, nsv, d):
    g = torch.Generator(device="cuda").manual_seed(n + nsv)
    x = torch.rand(n, d, device="cuda", generator=g)
    sv = torch.rand(nsv, d, device="cuda", generator=g)
    coef = torch.randn(nsv, device="cuda", generator=g)
    gamma = 1.0 / d
    got = K.rbf_decision(x, sv, coef, gamma, 0.25)
    ref = _rbf_ref(sv, x, gamma) @ coef.double() - 0.25
    assert torch.allclose(got.double(), ref, rtol=1e-4, atol=1e-4 * (1 + coef.abs().sum().item() / 100))


def test_compact(K):
    a = torch.rand(100003, device="cuda")
    a[a < 0.7] = 0
    got = K.compact_positive(a).long()
    ref = torch.nonzero(a > 0).flatten()
    assert torch.equal(got, ref)


@pytest.mark.parametrize("n,d", [(1000, 40), (777, 784), (256, 16)])
def test_rbf_gram_symmetric_mirror(K, n, d):
    """Dense-mode Gram GEMM: symmetric launch (upper tiles + mirrored
    transposes) == full launch bit for bit, and == fp32 reference."""
    g = torch.Generator().manual_seed(n + d)
    x = torch.rand(n, d, generator=g).cuda()
    gamma = 1.0 / d
    full = K.rbf_gram(x, x.clone(), gamma)
    sym = K.rbf_gram(x, None, gamma)
    torch.cuda.synchronize()
    assert torch.isfinite(sym).all()
    assert torch.equal(full, sym)
    assert torch.equal(sym, sym.T)
    ref = torch.exp(-gamma * torch.cdist(x.double(), x.double()) ** 2).float()
    assert torch.allclose(sym, ref, atol=2e-5, rtol=1e-4)


@pytest.mark.parametrize("n,d,rows,nq", [(1000, 54, 256, 16), (5000, 784, 512, 7), (2600, 1100, 1024, 3),
                                         (9000, 1024, 3072, 16)])
def test_xpass_rows_vs_torch_and_row_kernel(K, n, d, rows, nq):
    """The cache engines' X pass (xpass_fill: 16x16x4 f32 MFMA, double-buffered
    X loads, multi-chunk query staging for d > 1008) vs a float64 torch
    reference, and bit-identical to the chain's row kernel (the engines' shared
    trajectory depends on it)."""
    g = torch.Generator(device="cuda").manual_seed(n + d + nq)
    x = torch.rand(n, d, device="cuda", generator=g)
    keys = torch.randperm(n, generator=torch.Generator().manual_seed(n))[:nq].tolist()
    keys[0] = n - 1  # last row: the padded tail of the last workgroup
    gamma = 1.0 / d
    got = K.xpass_rows(x, keys, gamma, rows_per_group=rows)
    ref = _rbf_ref(x, x[keys], gamma)
    assert got.shape == (nq, n) and torch.isfinite(got).all()
    assert (got.double() - ref).abs().max().item() < 2e-5
    # K(x, x) = exp(-0) up to the fp32 expansion |x|^2 + |x|^2 - 2 x.x (no clamp
    # at 0: svmTrain.cu:128-130), i.e. within a few ulp of 1
    assert abs(float(got[0, n - 1]) - 1.0) < 1e-6
    rows_k = K.rbf_rows(x, x[keys], gamma)
    assert torch.equal(got, rows_k)


def test_fused_select_vs_torch(K):
    """Per-workgroup selection of the fused / persistent engines (I-set
    classification, DPP wave-64 minimum with payload, LDS across waves): each
    workgroup's keys equal a torch argmin / argmax over its rows, ties to the
    lowest index."""
    from dpsvm_amd.ops.kernels import decode_key

    n, C_, rows = 9000, 2.0, 512
    g = torch.Generator(device="cuda").manual_seed(5)
    f = torch.randn(n, device="cuda", generator=g)
    y = torch.where(torch.rand(n, device="cuda", generator=g) > 0.5, 1.0, -1.0)
    a = torch.rand(n, device="cuda", generator=g) * C_
    a[torch.rand(n, device="cuda", generator=g) < 0.3] = 0.0
    a[torch.rand(n, device="cuda", generator=g) < 0.2] = C_
    f[600:612] = -5.0  # ties inside one workgroup: lowest index wins
    y[600:612] = 1.0
    a[600:612] = 0.0
    keys = K.fused_select(f, a, y, C_, rows_per_group=rows).cpu()
    up = ((a == 0) & (y == 1)) | ((a == C_) & (y != 1)) | ((a > 0) & (a < C_))
    lo = ((a == 0) & (y != 1)) | ((a == C_) & (y == 1)) | ((a > 0) & (a < C_))
    fu = torch.where(up, f, torch.inf).cpu()
    fl = torch.where(lo, -f, torch.inf).cpu()
    for b in range((n + rows - 1) // rows):
        s = slice(b * rows, min(n, (b + 1) * rows))
        ih = b * rows + int(torch.argmin(fu[s]))  # torch.argmin: first occurrence
        il = b * rows + int(torch.argmin(fl[s]))
        vh, gh = decode_key(int(keys[b, 0]) & (2**64 - 1))
        vl, gl = decode_key(int(keys[b, 1]) & (2**64 - 1))
        assert (gh, vh) == (ih, float(f[ih])), b
        assert (gl, -vl) == (il, float(f[il])), b
    assert decode_key(int(keys[1, 0]) & (2**64 - 1))[1] == 600


@pytest.mark.parametrize("n,d,m", [(5000, 54, 35), (3000, 784, 130), (2000, 1024, 7), (777, 16, 1)])
def test_rbf_rows_indexed_vs_torch_and_gram(K, n, d, m):
    """The working-set cache engine's row GEMM (rbf_gemm EPI_ROWS: A rows by
    index, output rows scattered to lines, M read on the device) vs a float64
    torch reference, and bit-identical to the resident-Gram GEMM's rows (the
    ws-cache / ws-dense engines share their trajectory through it)."""
    g = torch.Generator(device="cuda").manual_seed(n + d + m)
    x = torch.rand(n, d, device="cuda", generator=g)
    rows = torch.randperm(n, generator=torch.Generator().manual_seed(m))[:m].tolist()
    lines = torch.randperm(m + 5, generator=torch.Generator().manual_seed(n))[:m].tolist()
    gamma = 1.0 / d
    out = K.rbf_rows_indexed(x, rows, gamma, out_lines=lines, n_lines=m + 5)
    got = out[lines]
    ref = _rbf_ref(x, x[rows], gamma)
    assert torch.isfinite(got).all()
    assert (got.double() - ref).abs().max().item() < 2e-5
    untouched = sorted(set(range(m + 5)) - set(lines))
    assert torch.isnan(out[untouched]).all()  # only the assigned lines are written
    gram = K.rbf_gram(x, x.clone(), gamma)
    assert torch.equal(got, gram[rows])
