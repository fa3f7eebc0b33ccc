"""Persistent small-problem rounds (ws_persist.hip) on MI355X.

One launch runs ws_block one-block rounds on a co-resident grid (workgroup 0
merges, gathers the sub-Gram into LDS and solves; every workgroup then applies
the changes to its columns of f and publishes candidates).  It keeps the
ws_select / ws_merge / ws_solve arithmetic, so the trajectory must be the graph
path's bit for bit: same alphas, b, pair steps and rounds — with box and
independent clipping, first- and second-order pair choice, 1 / 2 / 3 slots per
lane, a max_iter cap inside a launch and rows not a multiple of 256."""
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


CASES = [
    # name, n, C, gamma, clip, extra SVC knobs
    ("covtype", 7488, 2048.0, 0.03125, "box", {}),
    ("covtype", 5003, 64.0, 0.5, "independent", {"ws_wss": 1}),
    ("adult", 3000, 1.0, 0.05, "box", {"ws_size": 96}),
    ("mnist", 4100, 10.0, 0.25, "independent", {"ws_size": 48, "ws_block": 3}),
    ("blobs", 2500, 2.0, 0.15, "box", {"ws_size": 130, "max_iter": 1234}),
]


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}{c[1]}-{c[4]}" for c in CASES])
def test_persistent_rounds_bit_identical_to_graph_rounds(case):
    name, n, C_, g, clip, extra = case
    kw = dict(n=n, seed=3)
    if name == "blobs":
        kw.update(d=12, sep=1.2)
    X, y = synthetic(name, **kw)
    extra = dict(extra)
    base = dict(C=C_, gamma=g, eps=1e-3, clip=clip, device="cuda", solver="ws", max_iter=extra.pop("max_iter", 2_000_000))
    base.update(extra)
    per = SVC(ws_persist="on", **base).fit(X, y)
    gra = SVC(ws_persist="off", **base).fit(X, y)
    assert per.setup_info_["iteration"] == "ws-dense" and gra.setup_info_["iteration"] == "ws-dense"
    assert per.setup_info_["ws_rounds"] == "persistent", per.setup_info_["engine_note"]
    assert gra.setup_info_["ws_rounds"] == "graph"
    print(f"{name}{n}/{clip}: rounds {per.n_rounds_} steps {per.n_iter_} persistent {per.fit_time_:.4f} s "
          f"graph {gra.fit_time_:.4f} s")
    assert per.n_iter_ == gra.n_iter_ and per.n_rounds_ == gra.n_rounds_
    assert per.converged_ == gra.converged_
    assert np.array_equal(per.alpha_, gra.alpha_) and per.b_ == gra.b_
    if base["max_iter"] == 1234:
        assert per.n_iter_ == 1234 and not per.converged_


def test_persistent_rounds_opt_in_and_multi_block_refusal():
    """auto keeps the graph of launches (measured faster on MI355X,
    profiles/r5_ws_persist_ab.txt); "on" takes the persistent rounds where
    supported — one block per round: a multi-block engine keeps its graph"""
    X, y = synthetic("adult", n=2000, seed=9)
    kw = dict(C=1.0, gamma=0.05, eps=1e-3, device="cuda", solver="ws")
    assert SVC(**kw).fit(X, y).setup_info_["ws_rounds"] == "graph"
    assert SVC(ws_persist="on", **kw).fit(X, y).setup_info_["ws_rounds"] == "persistent"
    mb = SVC(ws_persist="on", ws_blocks=4, ws_size=96, **kw).fit(X, y)
    assert mb.setup_info_["ws_rounds"] == "graph" and mb.converged_


def test_persistent_rounds_repeated_solves_and_resume(tmp_path):
    """the grid's round counters persist on the device across launches and
    solves (reset per seed): a second fit on the same model object and a resumed
    solve follow the graph path's results"""
    X, y = synthetic("covtype", n=6000, seed=8)
    kw = dict(C=64.0, gamma=0.5, eps=1e-3, clip="box", device="cuda", solver="ws")
    ref = SVC(ws_persist="off", **kw).fit(X, y)
    clf = SVC(ws_persist="on", **kw)
    for _ in range(2):
        clf.fit(X, y)
        assert np.array_equal(clf.alpha_, ref.alpha_) and clf.b_ == ref.b_
    ck = str(tmp_path / "wp.ck")
    part = SVC(ws_persist="on", max_iter=ref.n_iter_ // 2, checkpoint_path=ck, checkpoint_every=10**9, **kw).fit(X, y)
    assert not part.converged_
    res = SVC(ws_persist="on", **kw).fit(X, y, resume=ck)
    assert res.converged_ and abs(res.b_ - ref.b_) < 1e-2
