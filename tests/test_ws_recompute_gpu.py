"""ws-cache rounds without the kernel-row cache (ws_recompute.hip) on MI355X.

With short rows (d <= 64 padded) the round's kernel rows are recomputed inside
the f update and the sub-Gram comes straight from the split X rows.  The K
values are the split GEMMs' bits, the f update sums them per column instead of
per changed row, so the run must stop at the resident-Gram engine's optimum
(same stop test, intercept, support set and decisions to rounding), and the
sub-Gram kernel must reproduce the Gram's entries bit for bit."""
import numpy as np
import pytest
import torch

from dpsvm_amd import SVC
from dpsvm_amd.utils.datasets import synthetic

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("case", [("covtype", 6000, 54, 4.0, 0.5, "independent"),
                                  ("covtype", 8000, 54, 64.0, 0.5, "box"),
                                  ("blobs", 5000, 20, 2.0, 0.15, "box"),
                                  ("covtype", 4000, 30, 1.0, 0.1, "independent")],
                         ids=["cov6000-indep", "cov8000-box", "blobs20-box", "cov30-indep"])
def test_recompute_rounds_reach_the_resident_gram_optimum(case):
    name, n, d, C_, g, clip = case
    kw = dict(n=n, d=d, seed=5)
    if name == "blobs":
        kw["sep"] = 1.2
    X, y = synthetic(name, **kw)
    base = dict(C=C_, gamma=g, eps=1e-3, clip=clip, device="cuda", solver="ws", ws_blocks=1)
    dense = SVC(**base).fit(X, y)
    rec = SVC(force_cache=True, cache_lines=2048, **base).fit(X, y)
    assert dense.setup_info_["ws_rows"] == "gram"
    assert rec.setup_info_["iteration"] == "ws-cache" and rec.setup_info_["ws_rows"] == "recompute"
    assert rec.converged_ and dense.converged_
    dd, dr = dense.decision_function(X), rec.decision_function(X)
    agree = float(np.mean(np.sign(dd) == np.sign(dr)))
    print(f"{name}{n}x{d}/{clip}: rounds {rec.n_rounds_} vs {dense.n_rounds_}, steps {rec.n_iter_} vs "
          f"{dense.n_iter_}, b {rec.b_:.6f} vs {dense.b_:.6f}, agree {agree:.5f}, sv {rec.n_support_} vs "
          f"{dense.n_support_}")
    assert agree > 0.995
    assert abs(rec.b_ - dense.b_) < 1e-2 * max(1.0, abs(dense.b_))
    assert abs(rec.n_support_ - dense.n_support_) <= max(3, dense.n_support_ // 100)
    if clip == "box":  # unique optimum
        assert np.abs(rec.alpha_ - dense.alpha_).max() < 0.05 * C_


def test_recompute_modes_and_fallbacks():
    """auto: recompute for d <= 64; "off" keeps the row cache (bit-identical to
    ws-dense, test_ws_gpu.py); rows longer than 64 keep the cache; a max_iter
    cap stops at exactly max_iter"""
    X, y = synthetic("covtype", n=5000, d=54, seed=2)
    kw = dict(C=8.0, gamma=0.5, eps=1e-3, device="cuda", solver="ws", force_cache=True, cache_lines=2048)
    assert SVC(ws_recompute="off", **kw).fit(X, y).setup_info_["ws_rows"] == "cache"
    capped = SVC(max_iter=777, **kw).fit(X, y)
    assert capped.setup_info_["ws_rows"] == "recompute" and capped.n_iter_ == 777 and not capped.converged_
    Xa, ya = synthetic("adult", n=3000, seed=2)  # 123 features: 128 padded
    wide = SVC(C=1.0, gamma=0.05, eps=1e-3, device="cuda", solver="ws", force_cache=True, cache_lines=2048).fit(Xa, ya)
    assert wide.setup_info_["ws_rows"] == "cache" and wide.converged_


def test_recompute_checkpoint_resume(tmp_path):
    X, y = synthetic("covtype", n=6000, d=54, seed=9)
    kw = dict(C=16.0, gamma=0.5, eps=1e-3, clip="box", device="cuda", solver="ws", force_cache=True,
              cache_lines=2048)
    full = SVC(**kw).fit(X, y)
    ck = str(tmp_path / "rc.ck")
    part = SVC(max_iter=full.n_iter_ // 2, checkpoint_path=ck, checkpoint_every=10**9, **kw).fit(X, y)
    assert not part.converged_
    res = SVC(**kw).fit(X, y, resume=ck)
    assert res.converged_ and abs(res.b_ - full.b_) < 1e-2 * max(1.0, abs(full.b_))


def test_recompute_after_the_multi_block_switch():
    """A multi-block ws-cache engine runs its multi-block rounds on the row
    cache and, once the adaptive block count reached 1 (coupled covtype rows),
    its one-block rounds without it — and still stops at the resident-Gram
    optimum"""
    X, y = synthetic("covtype", n=14000, d=54, seed=4)
    base = dict(C=64.0, gamma=0.5, eps=1e-3, clip="box", device="cuda", solver="ws", ws_blocks=4, ws_size=96)
    dense = SVC(**base).fit(X, y)
    rec = SVC(force_cache=True, cache_lines=10000, **base).fit(X, y)  # >= 2 P q + 8192: multi-block ws-cache
    assert rec.setup_info_["iteration"] == "ws-cache" and rec.setup_info_["ws_rows"] == "recompute"
    print(f"blocks {rec.stats_.get('ws_blocks')} -> {rec.stats_.get('ws_blocks_end')}, rounds {rec.n_rounds_} vs "
          f"{dense.n_rounds_}, b {rec.b_:.6f} vs {dense.b_:.6f}")
    assert rec.stats_.get("ws_blocks") == 4 and rec.stats_.get("ws_blocks_end") == 1
    assert rec.converged_
    agree = float(np.mean(np.sign(rec.decision_function(X)) == np.sign(dense.decision_function(X))))
    assert agree > 0.995 and abs(rec.b_ - dense.b_) < 1e-2 * max(1.0, abs(dense.b_))
