"""CPU solver (reference seq.cpp path / test oracle) vs an independent numpy
model of the reference algorithm and vs scikit-learn's libsvm."""
import numpy as np
import pytest

from dpsvm_amd import SVC
from dpsvm_amd.utils.datasets import synthetic
from ref_smo import decision, smo_reference


@pytest.mark.parametrize("clip", ["independent", "box"])
def test_matches_numpy_reference(clip):
    X, y = synthetic("blobs", n=300, d=5, seed=3, sep=1.5)
    a_ref, b_ref, it_ref = smo_reference(X, y, C=2.0, gamma=0.4, eps=1e-3, clip=clip)
    clf = SVC(C=2.0, gamma=0.4, eps=1e-3, clip=clip, device="cpu").fit(X, y)
    assert clf.converged_
    # same algorithm, f32 vs f64 arithmetic: iterate counts and alphas agree closely
    assert abs(clf.n_iter_ - it_ref) <= max(5, it_ref // 20)
    assert np.abs(clf.alpha_ - a_ref).max() < 5e-2
    assert abs(clf.b_ - b_ref) < 5e-3
    sv_ours, sv_ref = set(np.nonzero(clf.alpha_ > 0)[0]), set(np.nonzero(a_ref > 0)[0])
    assert len(sv_ours ^ sv_ref) <= max(2, len(sv_ref) // 20)


def test_box_clip_keeps_equality_constraint():
    X, y = synthetic("blobs", n=400, d=4, seed=5, sep=1.0)
    clf = SVC(C=1.0, gamma=0.5, clip="box", device="cpu").fit(X, y)
    assert abs(float((clf.alpha_ * np.where(y > 0, 1, -1)).sum())) < 1e-3
    assert clf.alpha_.min() >= 0 and clf.alpha_.max() <= 1.0


def test_independent_clip_reproduces_reference_drift():
    # the reference clips both alphas independently; sum(alpha*y) drifts
    X, y = synthetic("blobs", n=600, d=4, seed=11, sep=1.5)
    clf = SVC(C=2.0, gamma=0.5, device="cpu").fit(X, y)
    assert clf.converged_
    assert abs(float((clf.alpha_ * y).sum())) > 1e-3


def test_against_sklearn_libsvm():
    sk = pytest.importorskip("sklearn.svm")
    X, y = synthetic("adult", n=2000, seed=2)
    X = X[:, :]
    C_, g = 1.0, 0.05
    ref = sk.SVC(C=C_, gamma=g, kernel="rbf", tol=1e-3).fit(X, y)
    clf = SVC(C=C_, gamma=g, eps=1e-3, clip="box", device="cpu").fit(X, y)
    # same optimum (libsvm uses 2nd-order WSS; both reach the same KKT point)
    n_ref = int(ref.n_support_.sum())
    assert abs(clf.n_support_ - n_ref) <= max(5, n_ref // 50)
    assert abs(clf.score(X, y) - ref.score(X, y)) < 0.01
    # intercept: ours b with decision = sum - b; sklearn decision = sum + intercept
    assert abs(-clf.b_ - ref.intercept_[0]) < 0.05
    agree = np.mean(np.sign(clf.decision_function(X)) == np.sign(ref.decision_function(X)))
    assert agree > 0.99


def test_decision_matches_numpy():
    X, y = synthetic("mnist-parity", n=500, seed=1)
    clf = SVC(C=10, gamma=0.02, device="cpu").fit(X, y)
    dec = clf.decision_function(X[:100])
    ref = decision(X, y, clf.alpha_, clf.b_, clf.gamma_, X[:100])
    assert np.allclose(dec, ref, atol=1e-3, rtol=1e-4)
    assert clf.score(X, y) > 0.95


def test_default_gamma_is_one_over_d():
    X, y = synthetic("blobs", n=200, d=8, seed=0)
    clf = SVC(C=1.0, device="cpu").fit(X, y)
    assert abs(clf.gamma_ - 1.0 / 8) < 1e-7


def test_max_iter_stops():
    X, y = synthetic("blobs", n=500, d=4, seed=0, sep=0.5)
    clf = SVC(C=10.0, gamma=1.0, max_iter=37, device="cpu").fit(X, y)
    assert clf.n_iter_ == 37 and clf.status_ == 2 and not clf.converged_


def test_arbitrary_labels_mapped():
    X, y = synthetic("blobs", n=300, d=3, seed=4)
    lab = np.where(y > 0, 7, 3)
    clf = SVC(C=1.0, gamma=0.5, device="cpu").fit(X, lab)
    pred = clf.predict(X)
    assert set(np.unique(pred)) <= {3, 7}
    assert clf.score(X, lab) > 0.8


def test_cache_lines_small_same_result():
    X, y = synthetic("blobs", n=400, d=4, seed=8, sep=1.0)
    full = SVC(C=1.0, gamma=0.5, device="cpu").fit(X, y)
    tiny = SVC(C=1.0, gamma=0.5, cache_lines=2, device="cpu").fit(X, y)
    assert tiny.n_iter_ == full.n_iter_
    assert np.array_equal(tiny.alpha_, full.alpha_)
    assert tiny.stats_["cache_misses"] > full.stats_["cache_misses"]


def test_fault_injection_nonfinite_abort(monkeypatch):
    """DPSVM_FAULT=nan@K poisons f; the solver must stop with status 4."""
    X, y = synthetic("blobs", n=400, d=4, seed=3, sep=1.0)
    monkeypatch.setenv("DPSVM_FAULT", "nan@25")
    clf = SVC(C=1.0, gamma=0.5, device="cpu").fit(X, y)
    assert clf.status_ == 4 and not clf.converged_ and clf.n_iter_ == 25


def test_verify_ranks_consistent(monkeypatch, C):
    import threading

    monkeypatch.setenv("DPSVM_VERIFY", "1")
    X, y = synthetic("blobs", n=300, d=4, seed=3, sep=1.0)
    g = C.ThreadCommGroup(2)
    comms = [g.comm(r) for r in range(2)]
    out, errs = [None, None], []

    def work(r):
        try:
            out[r] = SVC(C=1.0, gamma=0.5, device="cpu").fit(X, y, comm=comms[r])
        except Exception as e:  # pragma: no cover
            errs.append(e)

    ts = [threading.Thread(target=work, args=(r,)) for r in range(2)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errs and out[0].converged_
    # invariant check ran on both ranks: f consistent with alpha
    assert all(0.0 <= o.stats_["verify_f_err"] < 1e-4 for o in out)
