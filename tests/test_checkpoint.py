"""Checkpoint / resume (absent from the reference)."""
import numpy as np

from dpsvm_amd import SVC
from dpsvm_amd._native import load
from dpsvm_amd.utils.datasets import synthetic


def test_resume_bit_exact(tmp_path):
    X, y = synthetic("blobs", n=500, d=4, seed=12, sep=1.0)
    full = SVC(C=1.0, gamma=0.5, device="cpu").fit(X, y)
    ck = str(tmp_path / "ck.bin")
    part = SVC(C=1.0, gamma=0.5, device="cpu", max_iter=full.n_iter_ // 2, checkpoint_path=ck,
               checkpoint_every=full.n_iter_ // 5).fit(X, y)
    assert not part.converged_
    c = load().read_checkpoint(ck)
    assert 0 < c.iter <= full.n_iter_ // 2 and c.n == 500 and len(c.f) == 500
    res = SVC(C=1.0, gamma=0.5, device="cpu").fit(X, y, resume=ck)
    assert res.n_iter_ == full.n_iter_
    assert np.array_equal(res.alpha_, full.alpha_)


def test_resume_recomputes_f(tmp_path):
    X, y = synthetic("blobs", n=400, d=4, seed=13, sep=1.0)
    full = SVC(C=1.0, gamma=0.5, device="cpu").fit(X, y)
    C = load()
    ck = str(tmp_path / "ck.bin")
    SVC(C=1.0, gamma=0.5, device="cpu", max_iter=full.n_iter_ // 2, checkpoint_path=ck,
        checkpoint_every=full.n_iter_ // 2).fit(X, y)
    c = C.read_checkpoint(ck)
    c.f = np.zeros(0, dtype=np.float32)  # drop f: solver rebuilds it from alpha
    res = SVC(C=1.0, gamma=0.5, device="cpu").fit(X, y, resume=c)
    assert res.converged_ and abs(res.b_ - full.b_) < 1e-2
    assert abs(res.n_support_ - full.n_support_) <= 3


def test_resume_rejects_mismatched_problem(tmp_path):
    """A checkpoint of another problem (gamma, C, clip, n, d) must be refused:
    its f is inconsistent with this kernel and its alphas may violate this box."""
    import pytest

    X, y = synthetic("blobs", n=300, d=4, seed=12, sep=1.0)
    ck = str(tmp_path / "ck.bin")
    SVC(C=1.0, gamma=0.5, device="cpu", max_iter=50, checkpoint_path=ck, checkpoint_every=25).fit(X, y)
    for kw, what in ((dict(C=1.0, gamma=0.25), "gamma"), (dict(C=2.0, gamma=0.5), "C ="),
                     (dict(C=1.0, gamma=0.5, clip="box"), "clip")):
        with pytest.raises(Exception, match=what):
            SVC(device="cpu", **kw).fit(X, y, resume=ck)
    with pytest.raises(Exception, match="n ="):
        SVC(C=1.0, gamma=0.5, device="cpu").fit(X[:200], y[:200], resume=ck)
    with pytest.raises(Exception, match="d ="):
        SVC(C=1.0, gamma=0.5, device="cpu").fit(np.hstack([X, X]), y, resume=ck)
    assert SVC(C=1.0, gamma=0.5, eps=1e-2, device="cpu").fit(X, y, resume=ck).converged_  # eps may differ


def _run_ranks(native, world, X, y, **kw):
    import threading

    resume = kw.pop("resume", None)
    if world == 1:
        return [SVC(device="cpu", **kw).fit(X, y, resume=resume)]
    g = native.ThreadCommGroup(world)
    comms = [g.comm(r) for r in range(world)]
    out, errs = [None] * world, []

    def work(r):
        try:
            out[r] = SVC(device="cpu", **kw).fit(X, y, comm=comms[r], resume=resume)
        except Exception as e:  # pragma: no cover
            errs.append(e)

    ts = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errs, errs
    return out


def test_resume_at_other_rank_count(tmp_path):
    """A checkpoint written by P ranks (global alpha + gathered f) resumes at
    P' ranks on the uninterrupted trajectory (P -> P')."""
    nat = load()
    X, y = synthetic("blobs", n=600, d=5, seed=14, sep=1.0)
    kw = dict(C=1.0, gamma=0.5)
    full = SVC(device="cpu", **kw).fit(X, y)
    for p_from, p_to in ((2, 1), (2, 3), (3, 2)):
        ck = str(tmp_path / f"ck{p_from}{p_to}.bin")
        part = _run_ranks(nat, p_from, X, y, max_iter=full.n_iter_ // 2, checkpoint_path=ck,
                          checkpoint_every=full.n_iter_ // 4, **kw)
        assert not part[0].converged_
        assert nat.read_checkpoint(ck).iter == full.n_iter_ // 2
        res = _run_ranks(nat, p_to, X, y, resume=ck, **kw)
        for r in res:
            assert r.n_iter_ == full.n_iter_ and np.array_equal(r.alpha_, full.alpha_)
