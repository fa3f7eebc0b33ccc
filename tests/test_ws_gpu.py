"""Working-set engine (solver="ws", ws_*.hip) on MI355X.

The ws engine applies the reference's pair rule (svmTrainMain.cpp:255-299) to a
q-row sub-problem per round, so its trajectory differs from the pair-at-a-time
engines; what must agree is the optimum it stops at: the reference's stop test
!(b_lo > b_hi + 2 eps) (svmTrainMain.cpp:310) on the exact gradient, the
intercept, the support set and the decision function — checked here against
the float64 numpy model of the reference (tests/ref_smo.py) and against the
persistent SMO engine."""
import os

import numpy as np
import pytest
import torch

from dpsvm_amd import SVC
from dpsvm_amd.utils.datasets import synthetic

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _kkt_gap(X, y, alpha, C, gamma):
    """b_lo - b_hi of the exact float64 gradient f = K (alpha y) - y."""
    from ref_smo import rbf_gram

    yy = np.where(y > 0, 1.0, -1.0)
    a = alpha.astype(np.float64)
    f = rbf_gram(X, gamma) @ (a * yy) - yy
    up = ((a == 0) & (yy == 1)) | ((a == C) & (yy != 1)) | ((a > 0) & (a < C))
    lo = ((a == 0) & (yy != 1)) | ((a == C) & (yy == 1)) | ((a > 0) & (a < C))
    return f[lo].max() - f[up].min()


@pytest.mark.parametrize("clip", ["independent", "box"])
@pytest.mark.parametrize("case", ["blobs", "mnist", "adult"])
def test_ws_engine_reaches_the_reference_optimum(case, clip):
    """box: the dual optimum is unique, so alphas, b, support set and decisions
    match the float64 model.  independent (the reference's default clipping,
    svmTrainMain.cpp:294-295) does not keep sum(alpha y) = 0, so the point it
    stops at depends on the trajectory: there the ws engine must satisfy the
    same stop test on the exact gradient and classify as well."""
    from ref_smo import smo_reference, decision

    X, y, C_, g = {
        "blobs": synthetic("blobs", n=2500, d=12, seed=41, sep=1.2) + (2.0, 0.15),
        "mnist": synthetic("mnist", n=3000, seed=4) + (10.0, 0.25),
        "adult": synthetic("adult", n=3000, seed=2) + (1.0, 0.05),
    }[case]
    a_ref, b_ref, it_ref = smo_reference(X, y, C=C_, gamma=g, eps=1e-3, clip=clip)
    ws = SVC(C=C_, gamma=g, eps=1e-3, clip=clip, device="cuda", solver="ws").fit(X, y)
    assert ws.setup_info_["iteration"] == "ws-dense"
    assert ws.converged_ and ws.n_rounds_ > 0
    gap = _kkt_gap(X, y, ws.alpha_, C_, g)
    yy = np.where(y > 0, 1.0, -1.0)
    d_ref = decision(X, y, a_ref, b_ref, g, X)
    d_ws = ws.decision_function(X)
    acc_ref, acc_ws = np.mean(np.sign(d_ref) == yy), np.mean(np.sign(d_ws) == yy)
    agree = np.mean(np.sign(d_ref) == np.sign(d_ws))
    print(f"{case}/{clip}: gap {gap:.2e} b {ws.b_:.5f} vs {b_ref:.5f} iters {ws.n_iter_} vs {it_ref} "
          f"acc {acc_ws:.4f} vs {acc_ref:.4f} agree {agree:.4f} max|da| {np.abs(ws.alpha_ - a_ref).max():.3g}")
    # the stop test holds on the exact gradient (fp32 drift allowance)
    assert gap < 2e-3 + 2e-4
    assert abs(acc_ws - acc_ref) < 0.02
    assert ws.n_iter_ < 3 * it_ref
    if clip == "box":
        assert abs(ws.b_ - b_ref) < 1e-2
        assert np.abs(ws.alpha_ - a_ref).max() < 0.1 * C_
        sv_ws, sv_ref = set(np.nonzero(ws.alpha_ > 0)[0]), set(np.nonzero(a_ref > 0)[0])
        assert len(sv_ws ^ sv_ref) <= max(3, len(sv_ref) // 50)
        assert agree > 0.99


def test_ws_engine_deterministic_and_matches_persistent_engine():
    X, y = synthetic("mnist", n=6000, seed=7)
    kw = dict(C=10.0, gamma=0.25, eps=1e-3, device="cuda")
    a = SVC(solver="ws", **kw).fit(X, y)
    b = SVC(solver="ws", **kw).fit(X, y)
    assert a.n_iter_ == b.n_iter_ and np.array_equal(a.alpha_, b.alpha_)
    p = SVC(solver="smo", **kw).fit(X, y)
    assert p.setup_info_["iteration"] == "persistent-dense"
    assert abs(a.b_ - p.b_) < 1e-2 and abs(a.n_support_ - p.n_support_) <= max(3, p.n_support_ // 100)
    assert abs(a.train_accuracy() - p.train_accuracy()) < 0.01


@pytest.mark.parametrize("q", [2, 16, 64, 130])
def test_ws_engine_small_working_sets_and_max_iter(q):
    X, y = synthetic("adult", n=2000, seed=9)
    kw = dict(C=1.0, gamma=0.05, eps=1e-3, device="cuda", solver="ws", ws_size=q)
    w = SVC(**kw).fit(X, y)
    assert w.converged_ and _kkt_gap(X, y, w.alpha_, 1.0, 0.05) < 2.2e-3
    capped = SVC(max_iter=500, **kw).fit(X, y)
    assert not capped.converged_ and capped.n_iter_ == 500


def test_ws_engine_checkpoint_resume(tmp_path):
    X, y = synthetic("mnist", n=4000, seed=11)
    kw = dict(C=10.0, gamma=0.25, eps=1e-3, device="cuda", solver="ws")
    full = SVC(**kw).fit(X, y)
    ck = str(tmp_path / "ws.ck")
    part = SVC(max_iter=full.n_iter_ // 2, checkpoint_path=ck, checkpoint_every=10**9, **kw).fit(X, y)
    assert not part.converged_
    res = SVC(**kw).fit(X, y, resume=ck)
    assert res.converged_ and abs(res.b_ - full.b_) < 1e-2
    assert _kkt_gap(X, y, res.alpha_, 10.0, 0.25) < 2.2e-3


@pytest.mark.parametrize("case", [("mnist", 4000, 10.0, 0.25, 1500), ("adult", 5000, 1.0, 0.05, 900),
                                  ("covtype", 6000, 4.0, 0.5, 2000)])
def test_ws_cache_engine_bit_identical_to_resident_gram(case):
    """ws-cache (kernel-row cache, the set's missing rows by one indexed MFMA
    GEMM per round, CLOCK-window victims) follows the ws-dense trajectory bit
    for bit: the same K values (same GEMM arithmetic), the same merge, the same
    f-update order.  A cache of ~900-2000 lines forces evictions.  (The
    resident Gram three-product, gram_adapt off: the rows GEMM has no
    one-product pass, docs/DESIGN.md §13.)"""
    name, n, C_, g, lines = case
    X, y = synthetic(name, n=n, seed=5)
    kw = dict(C=C_, gamma=g, eps=1e-3, device="cuda", solver="ws")
    dense = SVC(gram_adapt="off", **kw).fit(X, y)
    cache = SVC(force_cache=True, cache_lines=lines, ws_recompute="off", **kw).fit(X, y)
    assert dense.setup_info_["iteration"] == "ws-dense"
    assert cache.setup_info_["iteration"] == "ws-cache" and cache.setup_info_["cache_lines"] == lines
    assert cache.setup_info_["ws_rows"] == "cache"
    assert cache.converged_ and cache.n_iter_ == dense.n_iter_ and cache.n_rounds_ == dense.n_rounds_
    assert np.array_equal(cache.alpha_, dense.alpha_) and cache.b_ == dense.b_
    assert cache.stats_["rows_computed"] > lines  # more rows than lines: evictions happened


def test_ws_cache_engine_small_cache_raised_to_its_minimum():
    """A cache below ws-cache's 2 q + 512 lines (the reference's -s N takes any
    count, svmTrainMain.cpp:71): the production engines raise it to that
    minimum with a note and run; engines=all keeps the count for the
    (quarantined) pair cache engines."""
    X, y = synthetic("adult", n=3000, seed=1)
    # box clipping: one optimum for both engine families (independent clipping's depends on the trajectory)
    kw = dict(C=1.0, gamma=0.05, device="cuda", solver="ws", force_cache=True, cache_lines=300, clip="box")
    s = SVC(**kw).fit(X, y)
    assert s.setup_info_["iteration"] == "ws-cache" and s.converged_
    assert s.setup_info_["cache_lines"] == 2 * 192 + 512
    assert "raised to 896" in s.setup_info_["cache_note"]
    p = SVC(engines="all", **kw).fit(X, y)
    assert p.setup_info_["iteration"] in ("persistent-cache", "fused-cache")
    assert p.setup_info_["cache_lines"] == 300 and p.setup_info_["cache_note"] == ""
    assert "ws-cache needs" in p.setup_info_["engine_note"]
    assert abs(p.b_ - s.b_) < 2e-2


def test_cli_reference_cache_size_10_lines_production_engines():
    """svmTrain -s 10 (the reference's default cache: 10 kernel-row lines) on a
    50k-row problem whose Gram is therefore not resident: the production
    engines run it (ws-cache at its minimum line count, with a note on stderr)
    to convergence."""
    import subprocess
    import tempfile

    exe = os.path.join(ROOT, "bin", "svmTrain")
    if not os.path.exists(exe):
        pytest.skip("bin/svmTrain not built")
    with tempfile.TemporaryDirectory() as td:
        model = os.path.join(td, "m.txt")
        cmd = [exe, "-a", "32", "-x", "50000", "--synthetic", "blobs", "--seed", "5", "-c", "1", "-g", "0.05",
               "-e", "0.001", "-s", "10", "-m", model, "--metrics-json", os.path.join(td, "m.json")]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        assert "cache_lines 10 raised to 896" in r.stderr
        assert "Converged at iteration number" in r.stdout, r.stdout[-2000:]
        import json
        mj = json.load(open(os.path.join(td, "m.json")))
        assert mj["engine"] == "ws-cache" and mj["cache_lines"] == 896 and "raised to 896" in mj["cache_note"], mj


def test_production_engines_route_small_cache_problems_to_ws():
    """Production engines, solver auto below 50k rows: the pair-at-a-time
    engines only with the resident Gram; a Gram that is not resident (here a
    capped cache) runs ws-cache, and solver=smo there is refused with the
    reason (the pair cache engines are quarantined behind engines=all)."""
    X, y = synthetic("covtype", n=6000, seed=2)
    kw = dict(C=4.0, gamma=0.5, eps=1e-3, device="cuda", clip="box")  # box: one optimum for both engines
    dense = SVC(**kw).fit(X, y)
    assert dense.setup_info_["iteration"] == "persistent-dense"
    cap = SVC(force_cache=True, cache_lines=2000, **kw).fit(X, y)
    assert cap.setup_info_["iteration"] == "ws-cache" and cap.converged_
    assert abs(cap.b_ - dense.b_) < 1e-2
    with pytest.raises(Exception, match="solver=smo .*engines=all"):
        SVC(solver="smo", force_cache=True, cache_lines=2000, **kw).fit(X, y)
    pair = SVC(solver="smo", force_cache=True, cache_lines=2000, engines="all", **kw).fit(X, y)
    assert pair.setup_info_["iteration"] == "persistent-cache"
    assert pair.converged_ and abs(pair.b_ - dense.b_) < 1e-2


def _fit_threads(native, world, X, y, **kw):
    import threading

    g = native.ThreadCommGroup(world)
    comms = [g.comm(r) for r in range(world)]
    out, errs = [None] * world, []

    def work(r):
        try:
            out[r] = SVC(**kw).fit(X, y, comm=comms[r])
        except Exception as e:  # pragma: no cover
            errs.append(e)

    ts = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errs, errs
    return out


@pytest.mark.parametrize("world,extra", [(2, {}), (3, {}), (4, {"force_cache": True, "cache_lines": 1200})])
def test_ws_engine_sharded_ranks(world, extra):
    """Rows sharded over ranks (threads sharing the GPU, host-staged
    collectives): per round the candidate lists are all-gathered and the
    sub-Gram is summed from the columns each rank owns; every rank runs the
    merge and the sub-problem on identical inputs, so every rank ends with the
    same alphas (cross-rank digest), and the run reaches the one-rank optimum
    (box clipping: unique dual optimum)."""
    from dpsvm_amd._native import load

    X, y = synthetic("adult", n=4000, seed=13)
    kw = dict(C=1.0, gamma=0.05, eps=1e-3, clip="box", device="cuda", solver="ws", dp="shard", **extra)
    ref = SVC(**kw).fit(X, y)
    out = _fit_threads(load(), world, X, y, **kw)
    want = "ws-cache" if extra else "ws-dense"
    for r in range(world):
        assert out[r].setup_info_["iteration"] == want and out[r].setup_info_["n_local"] < 4000
        assert out[r].converged_
        assert np.array_equal(out[r].alpha_, out[0].alpha_)
    assert _kkt_gap(X, y, out[0].alpha_, 1.0, 0.05) < 2.2e-3
    assert abs(out[0].b_ - ref.b_) < 1e-2
    assert abs(out[0].n_support_ - ref.n_support_) <= max(3, ref.n_support_ // 50)


@pytest.mark.parametrize("extra", [{}, {"force_cache": True, "cache_lines": 1500}])
def test_ws_engine_rccl_one_rank_collective_path(extra):
    """The ws engines' RCCL collectives (in-place candidate all-gather, sub-Gram
    sum all-reduce) captured in the round hipGraph, on one GPU with a one-rank
    communicator (force_collectives): bit-identical to the local path."""
    from dpsvm_amd._native import load

    C = load()
    X, y = synthetic("mnist", n=4000, seed=3)
    kw = dict(C=10.0, gamma=0.25, eps=1e-3, device="cuda", solver="ws", **extra)
    ref = SVC(**kw).fit(X, y)
    comm = C.rccl_comm(C.rccl_unique_id(), 0, 1, 0)
    got = SVC(force_collectives=True, **kw).fit(X, y, comm=comm)
    assert got.setup_info_["iteration"] == ref.setup_info_["iteration"]
    assert got.n_iter_ == ref.n_iter_ and got.n_rounds_ == ref.n_rounds_
    assert np.array_equal(got.alpha_, ref.alpha_) and got.b_ == ref.b_


@pytest.mark.parametrize("world,extra", [(1, {}), (1, {"force_cache": True, "cache_lines": 1500}),
                                         (2, {}), (4, {"force_cache": True, "cache_lines": 1500})])
def test_ws_engine_partitioned_x_bit_identical(world, extra):
    """x_mode=partitioned (each rank holds only its X shard): ws-dense builds
    the Gram block from broadcast shard panels, ws-cache sums the misses' packed
    X rows over ranks each round.  Same K values, same collectives: the
    trajectory is bit-identical to replicated X at the same rank count."""
    from dpsvm_amd._native import load

    X, y = synthetic("mnist", n=4000, seed=21)
    kw = dict(C=10.0, gamma=0.25, eps=1e-3, device="cuda", solver="ws", dp="shard", **extra)
    if world == 1:
        rep = [SVC(**kw).fit(X, y)]
        part = [SVC(x_mode="partitioned", **kw).fit(X, y)]
    else:
        rep = _fit_threads(load(), world, X, y, **kw)
        part = _fit_threads(load(), world, X, y, x_mode="partitioned", **kw)
    want = "ws-cache" if extra else "ws-dense"
    for r in range(world):
        assert part[r].setup_info_["iteration"] == want and not part[r].setup_info_["x_replicated"]
        assert rep[r].setup_info_["x_replicated"]
        assert part[r].n_iter_ == rep[r].n_iter_ and part[r].n_rounds_ == rep[r].n_rounds_
        assert np.array_equal(part[r].alpha_, rep[r].alpha_) and part[r].b_ == rep[r].b_
    assert part[0].converged_


@pytest.mark.parametrize("n", [150_000, 1_100_000])
def test_ws_engine_large_n_rows_per_thread(n):
    """Selection geometries whose rows per thread (a.rpt) is below the kernel's
    register size RPT: 150k rows = 3 per thread on the RPT=4 kernel (ws-dense);
    1.1M rows = 17 per thread on the RPT=32 kernel (ws-cache; 256 x 256 x 32 =
    2.1M rows per rank, the synthetic-2m preset's geometry).  The stop test
    must hold on the exact gradient (K(X, SVs) coef - y on the GPU in fp64) —
    a workgroup indexing its rows by RPT instead of a.rpt once left rows
    without f updates (a 'converged' run with an exact gap of 1.4)."""
    d = 8
    X, y = synthetic("blobs", n=n, d=d, seed=3, sep=10.0)  # well separated: few SVs
    C_, g = 1.0, 0.125
    # solver auto picks the working-set engines from 50k rows on
    s = SVC(C=C_, gamma=g, eps=1e-3, device="cuda", max_iter=200000, shrink="off").fit(X, y)
    rpt = s.setup_info_["rows_per_group"] // 256
    if n > 1_000_000:
        assert s.setup_info_["iteration"] == "ws-cache" and rpt == 17  # RPT=32 kernel
    else:
        assert s.setup_info_["iteration"] == "ws-dense" and rpt == 3  # RPT=4 kernel
    assert s.converged_
    yy = torch.tensor(np.where(y > 0, 1.0, -1.0), device="cuda", dtype=torch.float64)
    a = torch.tensor(s.alpha_, device="cuda", dtype=torch.float64)
    Xd = torch.tensor(X, device="cuda", dtype=torch.float64)
    sv = torch.nonzero(a > 0).flatten()
    coef = a[sv] * yy[sv]
    f = torch.empty(n, device="cuda", dtype=torch.float64)
    for i in range(0, n, 1 << 16):
        xb = Xd[i:i + (1 << 16)]
        k = torch.exp(-g * torch.cdist(xb, Xd[sv]) ** 2)
        f[i:i + (1 << 16)] = k @ coef - yy[i:i + (1 << 16)]
    up = ((a == 0) & (yy == 1)) | ((a == C_) & (yy != 1)) | ((a > 0) & (a < C_))
    lo = ((a == 0) & (yy != 1)) | ((a == C_) & (yy == 1)) | ((a > 0) & (a < C_))
    gap = float(f[lo].max() - f[up].min())
    print(f"{n} rows: {s.n_iter_} pair steps, {s.n_rounds_} rounds, {s.n_support_} SVs, gap {gap:.2e}")
    assert gap < 2e-3 + 2e-4


def test_svmtrain_cli_ws_simulated_ranks_partitioned(tmp_path, bin_dir):
    """svmTrain --solver ws with 3 simulated ranks on one device (in-process
    communicator) and partitioned X: converges to the one-rank optimum (box
    clipping), reports the ws engine in --metrics-json, and writes a model
    whose b matches."""
    import json
    import os
    import subprocess

    outs = {}
    for ranks, extra in ((1, []), (3, ["--ranks", "3", "--x-mode", "partitioned", "--dp", "shard"])):
        mj = str(tmp_path / f"m{ranks}.json")
        cmd = [os.path.join(bin_dir, "svmTrain"), "-a", "123", "-x", "4000", "--synthetic", "adult", "-c", "1",
               "-g", "0.05", "-m", str(tmp_path / f"model{ranks}.txt"), "--solver", "ws", "--clip", "box",
               "--metrics-json", mj] + extra
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        outs[ranks] = json.load(open(mj))
    one, three = outs[1], outs[3]
    assert one["engine"] == "ws-dense" and three["engine"] == "ws-dense" and three["world"] == 3
    assert abs(one["b"] - three["b"]) < 1e-2 and abs(one["n_sv"] - three["n_sv"]) <= 40


@pytest.mark.parametrize("extra", [{}, {"force_cache": True, "cache_lines": 1500}])
def test_ws_peer_exchange_loopback_bit_identical(extra):
    """exchange="peer" at world 1: the rounds' candidate lists and sub-Gram rows
    go through the in-kernel exchange (pushed to the own receive buffer, polled
    back) — the same values as the direct path, so the same trajectory bit for bit."""
    X, y = synthetic("mnist", n=4000, seed=3)
    kw = dict(C=10.0, gamma=0.25, eps=1e-3, device="cuda", solver="ws", xch_timeout_s=30.0, **extra)
    ref = SVC(**kw).fit(X, y)
    got = SVC(exchange="peer", **kw).fit(X, y)
    assert got.setup_info_["exchange"] == "loopback" and ref.setup_info_["exchange"] == "none"
    assert got.setup_info_["iteration"] == ref.setup_info_["iteration"]
    assert got.n_iter_ == ref.n_iter_ and got.n_rounds_ == ref.n_rounds_
    assert np.array_equal(got.alpha_, ref.alpha_) and got.b_ == ref.b_


@pytest.mark.parametrize("world,engine,n", [(2, "ws", 6000), (4, "ws", 6000), (2, "ws-cache", 6000),
                                           (2, "ws", 70000)])
def test_ws_peer_exchange_processes_one_gpu(tmp_path, world, engine, n):
    """Sharded working-set rounds with ranks as processes sharing the GPU (gloo
    bootstrap, IPC-mapped uncached receive buffers): no collective per round —
    each selection workgroup pushes its candidate lists to every rank, each
    gather workgroup the sub-Gram entries its rank owns.  Every rank ends with
    the same alphas (cross-rank digest, on by default), bit-identical to the
    same rank count over host-staged collectives (thread ranks).  Four ranks
    sharing one GPU run q = 64: gather workgroups of three ranks spinning on one
    device must leave CUs (LDS) free for the fourth rank's solve workgroup —
    on distinct GPUs each device runs only its own rank's kernels."""
    import hashlib
    import json
    import os
    import subprocess
    import sys

    from dpsvm_amd._native import load

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DPSVM_FORCE_DEVICE="0")
    out = tmp_path / f"ws{world}"
    port = 29680 + world + (10 if engine == "ws-cache" else 0) + (20 if n > 6000 else 0)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(root, "tests", "mp_exchange_worker.py"), str(out), engine, str(n),
           json.dumps({"ws_size": 64} if world > 2 else {})]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=root)
    errs = "".join(open(f"{out}.rank{k}.err").read()[-1500:] for k in range(world)
                   if os.path.exists(f"{out}.rank{k}.err"))
    assert r.returncode == 0, errs + r.stderr[-2000:]
    res = [json.load(open(f"{out}.rank{k}.json")) for k in range(world)]
    X, y = synthetic("covtype", n=n, seed=2)
    kw = dict(C=4.0, gamma=0.5, eps=1e-3, device="cuda", solver="ws", dp="shard")
    if engine == "ws-cache":
        kw.update(force_cache=True, cache_lines=1500)
    if world > 2:
        kw.update(ws_size=64)
    # host-staged collectives on the thread ranks (70k rows: multi-block rounds on both sides)
    ref = _fit_threads(load(), world, X, y, exchange="allreduce", **kw)
    sha = hashlib.sha256(ref[0].alpha_.tobytes()).hexdigest()
    for k in range(world):
        assert res[k]["exchange"] == "peer" and res[k]["exchange_mem"] == "uncached"
        assert res[k]["iteration"] == ("ws-cache" if engine == "ws-cache" else "ws-dense")
        assert ref[k].setup_info_["exchange"] == "allreduce"
        assert res[k]["iters"] == ref[0].n_iter_ and res[k]["rounds"] == ref[0].n_rounds_
        assert res[k]["alpha_sha"] == sha
    if n > 6000:  # 2 x 137 selection workgroups: the merge folds two candidate lists per thread
        assert ref[0].setup_info_["groups"] * world > 256


@pytest.mark.parametrize("clip", ["independent", "box"])
@pytest.mark.parametrize("extra", [{}, {"force_cache": True, "cache_lines": 11000}])
def test_ws_multi_block_peer_exchange_loopback_bit_identical(clip, extra):
    """Multi-block rounds over the in-kernel peer exchange at world 1
    (exchange="peer": loopback into the own receive buffer): the candidate
    lists (ws_rank polls them), the P sub-Grams' entries and f (pushed by
    ws_gather_multi, polled by ws_solve) and the line-search partials (pushed
    by pass 1, polled by pass 2) — the same values as the direct path, so the
    same trajectory bit for bit (coupled data: the adaptive count falls to one
    block mid-run, so the one-block rounds of a multi-block engine's exchange
    layout are covered too)."""
    # (ws-cache multi-block rounds need L >= 2 P q + 8192 lines: 12,000 rows, 11,000 lines)
    n = 12000 if extra else 8000
    for case in ("mnist", "blobs"):
        X, y = (synthetic("mnist", n=n, seed=3) if case == "mnist"
                else synthetic("blobs", n=n, d=12, seed=41, sep=1.2))
        kw = dict(C=10.0 if case == "mnist" else 2.0, gamma=0.25 if case == "mnist" else 0.15, eps=1e-3,
                  clip=clip, device="cuda", solver="ws", ws_blocks=4, xch_timeout_s=30.0, **extra)
        if extra:  # the row cache on both sides (recompute rounds are a world-1, no-exchange mode)
            kw["ws_recompute"] = "off"
        ref = SVC(**kw).fit(X, y)
        got = SVC(exchange="peer", **kw).fit(X, y)
        assert got.setup_info_["exchange"] == "loopback" and ref.setup_info_["exchange"] == "none"
        assert got.stats_["ws_blocks"] == 4 and ref.stats_["ws_blocks"] == 4, got.setup_info_.get("engine_note")
        assert got.setup_info_["iteration"] == ref.setup_info_["iteration"]
        assert got.n_iter_ == ref.n_iter_ and got.n_rounds_ == ref.n_rounds_
        assert np.array_equal(got.alpha_, ref.alpha_) and got.b_ == ref.b_
        assert got.converged_


@pytest.mark.parametrize("world,clip", [(2, "independent"), (2, "box"), (4, "box")])
def test_ws_multi_block_peer_exchange_processes_one_gpu(tmp_path, world, clip):
    """Sharded MULTI-BLOCK rounds with ranks as processes sharing the GPU (gloo
    bootstrap, IPC-mapped uncached receive buffers): zero collectives per round
    (candidates, sub-Gram entries and line-search partials pushed in-kernel),
    bit-identical to the same rank count over host-staged collectives (thread
    ranks, exchange=allreduce)."""
    import hashlib
    import json
    import os
    import subprocess
    import sys

    from dpsvm_amd._native import load

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DPSVM_FORCE_DEVICE="0")
    out = tmp_path / f"wsm{world}"
    port = 29720 + world + (5 if clip == "box" else 0)
    knobs = {"ws_blocks": 4, "clip": clip}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(root, "tests", "mp_exchange_worker.py"), str(out), "ws", "6000", json.dumps(knobs)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=root)
    errs = "".join(open(f"{out}.rank{k}.err").read()[-1500:] for k in range(world)
                   if os.path.exists(f"{out}.rank{k}.err"))
    assert r.returncode == 0, errs + r.stderr[-2000:]
    res = [json.load(open(f"{out}.rank{k}.json")) for k in range(world)]
    X, y = synthetic("covtype", n=6000, seed=2)
    kw = dict(C=4.0, gamma=0.5, eps=1e-3, device="cuda", solver="ws", dp="shard", ws_blocks=4, clip=clip)
    ref = _fit_threads(load(), world, X, y, exchange="allreduce", **kw)
    sha = hashlib.sha256(ref[0].alpha_.tobytes()).hexdigest()
    assert ref[0].stats_["ws_blocks"] == 4
    for k in range(world):
        assert res[k]["exchange"] == "peer" and res[k]["ws_blocks"] == 4, res[k]
        assert ref[k].setup_info_["exchange"] == "allreduce"
        assert res[k]["iters"] == ref[0].n_iter_ and res[k]["rounds"] == ref[0].n_rounds_
        assert res[k]["alpha_sha"] == sha


def test_ws_wide_union_peer_exchange_two_processes_one_gpu(tmp_path):
    """Sharded rounds of 128 blocks of 48 rows (the 6,144-row union the
    uncoupled headline takes) over the in-kernel peer exchange, two ranks as
    processes sharing the GPU: 16 candidate keys a side per list pushed and
    collected, 128 sub-problems' entries polled by the solve — bit-identical to
    the same two ranks over host-staged collectives (thread ranks)."""
    import hashlib
    import json
    import os
    import subprocess
    import sys

    from dpsvm_amd._native import load

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DPSVM_FORCE_DEVICE="0")
    out = tmp_path / "wide2"
    knobs = {"ws_blocks": 128, "ws_size": 48, "_data": "mnist"}
    n = 14000
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29761",
           os.path.join(root, "tests", "mp_exchange_worker.py"), str(out), "ws", str(n), json.dumps(knobs)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=root)
    errs = "".join(open(f"{out}.rank{k}.err").read()[-1500:] for k in range(2) if os.path.exists(f"{out}.rank{k}.err"))
    assert r.returncode == 0, errs + r.stderr[-2000:]
    res = [json.load(open(f"{out}.rank{k}.json")) for k in range(2)]
    X, y = synthetic("mnist", n=n, seed=2)
    kw = dict(C=10.0, gamma=0.25, eps=1e-3, device="cuda", solver="ws", dp="shard", ws_blocks=128, ws_size=48)
    ref = _fit_threads(load(), 2, X, y, exchange="allreduce", **kw)
    sha = hashlib.sha256(ref[0].alpha_.tobytes()).hexdigest()
    assert ref[0].stats_["ws_blocks"] == 128 and ref[0].converged_
    for k in range(2):
        assert res[k]["exchange"] == "peer" and res[k]["ws_blocks"] == 128, res[k]
        assert res[k]["iters"] == ref[0].n_iter_ and res[k]["rounds"] == ref[0].n_rounds_
        assert res[k]["alpha_sha"] == sha


@pytest.mark.parametrize("clip", ["independent", "box"])
@pytest.mark.parametrize("knobs", [{"ws_blocks": 4}, {"ws_blocks": 1}])
def test_ws_peer_exchange_eight_processes_one_gpu(tmp_path, clip, knobs):
    """EIGHT ranks as processes sharing the GPU (the rank count of the 8-GPU
    node) at the default working-set size: every producer pushes and returns,
    only the collect kernels and the solve poll, so eight ranks' spinning
    consumers leave the device room for every rank's producers.  Multi-block
    rounds on covtype-shape data fall to one block mid-run (damped rounds), so
    the one-block rounds of a multi-block engine run over the exchange too.
    Bit-identical to the same 8 ranks over host-staged collectives, in both
    clipping modes."""
    import hashlib
    import json
    import os
    import subprocess
    import sys

    from dpsvm_amd._native import load

    world = 8
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DPSVM_FORCE_DEVICE="0")
    out = tmp_path / "ws8"
    port = 29760 + (1 if clip == "box" else 0) + (2 if knobs["ws_blocks"] > 1 else 0)
    kn = dict(knobs, clip=clip)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(root, "tests", "mp_exchange_worker.py"), str(out), "ws", "6000", json.dumps(kn)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=root)
    errs = "".join(open(f"{out}.rank{k}.err").read()[-1500:] for k in range(world)
                   if os.path.exists(f"{out}.rank{k}.err"))
    assert r.returncode == 0, errs + r.stderr[-2000:]
    res = [json.load(open(f"{out}.rank{k}.json")) for k in range(world)]
    X, y = synthetic("covtype", n=6000, seed=2)
    kw = dict(C=4.0, gamma=0.5, eps=1e-3, device="cuda", solver="ws", dp="shard", **kn)
    ref = _fit_threads(load(), world, X, y, exchange="allreduce", **kw)
    sha = hashlib.sha256(ref[0].alpha_.tobytes()).hexdigest()
    for k in range(world):
        assert res[k]["ws_exchange"] == "peer" and res[k]["engine_note"] == "", res[k]
        assert ref[k].setup_info_["ws_exchange"] == "collectives"
        assert res[k]["iters"] == ref[0].n_iter_ and res[k]["rounds"] == ref[0].n_rounds_
        assert res[k]["alpha_sha"] == sha
    if knobs["ws_blocks"] > 1:  # the one-block switch ran under the peer exchange
        assert res[0]["ws_blocks"] == 4 and res[0]["ws_p1_round"] > 0, res[0]


@pytest.mark.parametrize("blocks", [2, 8])
@pytest.mark.parametrize("clip", ["independent", "box"])
@pytest.mark.parametrize("case", ["blobs", "mnist", "adult"])
def test_ws_multi_block_rounds_reach_the_reference_optimum(case, clip, blocks):
    """ws_blocks = P: P disjoint sub-problems per round, the combined step scaled
    by the exact line search (ws_*.hip, multi-block rounds).  Coupled problems
    (blobs, adult: K far from I) exercise t < 1; the stop test must hold on the
    exact float64 gradient and, with box clipping, the unique dual optimum must
    be reached."""
    from ref_smo import smo_reference, decision

    X, y, C_, g = {
        "blobs": synthetic("blobs", n=2500, d=12, seed=41, sep=1.2) + (2.0, 0.15),
        "mnist": synthetic("mnist", n=3000, seed=4) + (10.0, 0.25),
        "adult": synthetic("adult", n=3000, seed=2) + (1.0, 0.05),
    }[case]
    a_ref, b_ref, it_ref = smo_reference(X, y, C=C_, gamma=g, eps=1e-3, clip=clip)
    ws = SVC(C=C_, gamma=g, eps=1e-3, clip=clip, device="cuda", solver="ws", ws_blocks=blocks).fit(X, y)
    assert ws.setup_info_["iteration"] == "ws-dense" and "ws_blocks" not in ws.setup_info_.get("engine_note", "")
    assert ws.converged_
    gap = _kkt_gap(X, y, ws.alpha_, C_, g)
    yy = np.where(y > 0, 1.0, -1.0)
    d_ref = decision(X, y, a_ref, b_ref, g, X)
    d_ws = ws.decision_function(X)
    acc_ref, acc_ws = np.mean(np.sign(d_ref) == yy), np.mean(np.sign(d_ws) == yy)
    agree = np.mean(np.sign(d_ref) == np.sign(d_ws))
    print(f"P={blocks} {case}/{clip}: gap {gap:.2e} b {ws.b_:.5f} vs {b_ref:.5f} steps {ws.n_iter_} vs {it_ref} "
          f"rounds {ws.n_rounds_} acc {acc_ws:.4f} vs {acc_ref:.4f} agree {agree:.4f}")
    assert gap < 2e-3 + 2e-4
    assert np.all((ws.alpha_ >= 0) & (ws.alpha_ <= C_))
    assert abs(acc_ws - acc_ref) < 0.02
    if clip == "box":
        assert abs(float(np.sum(ws.alpha_ * yy))) < 1e-2 * C_  # the line search keeps sum(alpha y)
        assert abs(ws.b_ - b_ref) < 1e-2
        assert np.abs(ws.alpha_ - a_ref).max() < 0.1 * C_
        assert agree > 0.99


def test_ws_multi_block_deterministic_max_iter_and_fallback():
    X, y = synthetic("adult", n=4000, seed=9)
    kw = dict(C=1.0, gamma=0.05, eps=1e-3, device="cuda", solver="ws", ws_blocks=4)
    a = SVC(**kw).fit(X, y)
    b = SVC(**kw).fit(X, y)
    assert a.converged_ and a.n_iter_ == b.n_iter_ and np.array_equal(a.alpha_, b.alpha_)
    # fewer rounds where the blocks decouple (K ~ I, no clipping: the headline's regime)
    Xm, ym = synthetic("mnist", n=20000, seed=5)
    km = dict(C=10.0, gamma=0.25, eps=1e-3, device="cuda", solver="ws")
    m4, m1 = SVC(ws_blocks=4, **km).fit(Xm, ym), SVC(ws_blocks=1, **km).fit(Xm, ym)
    assert m4.converged_ and m1.converged_ and m4.n_rounds_ < 0.5 * m1.n_rounds_
    assert abs(m4.b_ - m1.b_) < 2e-3 and abs(m4.train_accuracy() - m1.train_accuracy()) < 0.005
    capped = SVC(max_iter=700, **kw).fit(X, y)  # the blocks share the pair-step budget exactly
    assert not capped.converged_ and capped.n_iter_ == 700
    # ineligible engine (kernel-row cache): one block per round, said so
    c = SVC(cache_lines=900, force_cache=True, **kw).fit(X, y)
    assert c.setup_info_["iteration"] == "ws-cache" and "ws_blocks" in c.setup_info_["engine_note"]
    assert c.converged_


@pytest.mark.parametrize("world", [2, 3])
def test_ws_multi_block_sharded_ranks(world):
    """Multi-block rounds with rows sharded over ranks (threads sharing the GPU,
    host-staged collectives): candidate lists all-gathered, the P sub-Grams and
    the members' f summed from the owners' columns, the line-search partials
    all-gathered between the two f-update passes.  Every rank ends with the same
    alphas and the run reaches the one-rank optimum (box clipping)."""
    from dpsvm_amd._native import load

    X, y = synthetic("adult", n=4000, seed=13)
    kw = dict(C=1.0, gamma=0.05, eps=1e-3, clip="box", device="cuda", solver="ws", dp="shard", ws_blocks=4)
    ref = SVC(**kw).fit(X, y)
    # host communicators take multi-block rounds only with exchange=allreduce
    # (else the one-block rounds over the peer exchange)
    out = _fit_threads(load(), world, X, y, exchange="allreduce", **kw)
    for r in range(world):
        assert out[r].setup_info_["iteration"] == "ws-dense" and out[r].setup_info_["n_local"] < 4000
        assert "ws_blocks" not in out[r].setup_info_.get("engine_note", "")
        assert out[r].converged_
        assert np.array_equal(out[r].alpha_, out[0].alpha_)
    assert _kkt_gap(X, y, out[0].alpha_, 1.0, 0.05) < 2.2e-3
    assert abs(out[0].b_ - ref.b_) < 1e-2
    assert abs(out[0].n_support_ - ref.n_support_) <= max(3, ref.n_support_ // 50)


@pytest.mark.parametrize("world", [4, 8])
def test_ws_wide_union_sharded_thread_ranks_host_collectives(world):
    """The default 8-GPU path's round shape, rehearsed with thread ranks over
    host collectives: mnist-shape rows sharded over
    4 / 8 ranks in rounds of 128 blocks of 48 rows (a 6,144-row union: what
    ws_blocks auto picks from 50k rows on numerically diagonal data at every
    rank count), candidate lists / sub-Grams / line-search partials through the
    communicator each round.  Every rank converges with the same alphas.  The
    trajectory is not the one-rank one bit for bit: the line search's double
    partial sums are reduced per 1,024-column group of each rank's shard, so
    their rounding depends on the partition (4 and 8 ranks land within 1e-8 of
    each other in b, 2.4e-4 from one rank) — both stop inside the same
    2 eps band, with the same support set and decision signs."""
    from dpsvm_amd._native import load

    X, y = synthetic("mnist", n=16000, seed=21)
    kw = dict(C=10.0, gamma=0.25, eps=1e-3, device="cuda", solver="ws", ws_blocks=128, ws_size=48)
    ref = SVC(**kw).fit(X, y)
    assert ref.setup_info_["iteration"] == "ws-dense" and ref.converged_
    assert ref.stats_["ws_blocks"] == 128, ref.stats_
    out = _fit_threads(load(), world, X, y, exchange="allreduce", dp="shard", **kw)
    for r in range(world):
        assert out[r].setup_info_["iteration"] == "ws-dense" and out[r].setup_info_["n_local"] <= 16000 // world + 1
        assert out[r].setup_info_["exchange"] == "allreduce"
        assert out[r].stats_["ws_blocks"] == 128, out[r].stats_  # the 6,144-row union at every rank count
        assert out[r].converged_
        assert np.array_equal(out[r].alpha_, out[0].alpha_)
    assert abs(out[0].b_ - ref.b_) < 1e-3, (out[0].b_, ref.b_)  # eps: inside the stop band
    assert out[0].n_support_ == ref.n_support_
    d_ref = ref.decision_function(X[:4000])
    d_out = out[0].decision_function(X[:4000])
    assert np.mean(np.sign(d_ref) == np.sign(d_out)) > 0.999


def test_ws_multi_block_rccl_one_rank_collective_path():
    """Multi-block rounds over a one-rank RCCL communicator (force_collectives:
    sub-Gram sum, partials and candidate all-gathers captured in the round
    graph): bit-identical to the local path."""
    from dpsvm_amd._native import load

    C = load()
    X, y = synthetic("mnist", n=8000, seed=3)
    kw = dict(C=10.0, gamma=0.25, eps=1e-3, device="cuda", solver="ws", ws_blocks=4)
    ref = SVC(**kw).fit(X, y)
    comm = C.rccl_comm(C.rccl_unique_id(), 0, 1, 0)
    got = SVC(force_collectives=True, **kw).fit(X, y, comm=comm)
    assert "ws_blocks" not in got.setup_info_.get("engine_note", "")
    assert got.n_iter_ == ref.n_iter_ and got.n_rounds_ == ref.n_rounds_
    assert np.array_equal(got.alpha_, ref.alpha_) and got.b_ == ref.b_


def test_ws_multi_block_checkpoint_resume(tmp_path):
    """Multi-block rounds (4 blocks, box clipping) stopped at half the pair
    steps with a checkpoint, resumed: the resumed run reaches the uninterrupted
    run's optimum (unique with box clipping)."""
    X, y = synthetic("mnist", n=6000, seed=11)
    kw = dict(C=10.0, gamma=0.25, eps=1e-3, clip="box", device="cuda", solver="ws", ws_blocks=4)
    full = SVC(**kw).fit(X, y)
    assert full.stats_["ws_blocks"] == 4
    ck = str(tmp_path / "wsm.ck")
    part = SVC(max_iter=full.n_iter_ // 2, checkpoint_path=ck, checkpoint_every=10**9, **kw).fit(X, y)
    assert not part.converged_
    res = SVC(**kw).fit(X, y, resume=ck)
    assert res.converged_ and abs(res.b_ - full.b_) < 1e-2
    assert _kkt_gap(X, y, res.alpha_, 10.0, 0.25) < 2.2e-3
    assert np.abs(res.alpha_ - full.alpha_).max() < 0.05 * 10.0


@pytest.mark.parametrize("clip", ["independent", "box"])
def test_ws_adaptive_blocks_fall_back_to_one_block_rounds(clip):
    """Coupled data (adult-shape, C = 100): the adaptive block count falls from
    8 on damped rounds (or to 1 on a clip event with independent clipping), and
    at 1 the engine runs the one-block round kernels; the run converges to the
    reference stop test on the exact gradient in no more rounds than one block
    per round, and never collapses into the ~3.5-pair-step rounds of round 2."""
    X, y = synthetic("adult", n=6000, seed=4)
    kw = dict(C=100.0, gamma=0.5, eps=1e-3, clip=clip, device="cuda", solver="ws")
    m8 = SVC(ws_blocks=8, **kw).fit(X, y)
    m1 = SVC(ws_blocks=1, **kw).fit(X, y)
    assert m8.converged_ and m1.converged_
    st = m8.stats_
    print(f"{clip}: P=8 rounds {m8.n_rounds_} steps {m8.n_iter_} end {st['ws_blocks_end']} one-block from round "
          f"{st['ws_p1_round']} damped {st['ws_damped']} | P=1 rounds {m1.n_rounds_} steps {m1.n_iter_}")
    assert st["ws_blocks"] == 8
    if st["ws_blocks_end"] == 1:  # fell back: from a round the status reported
        assert st["ws_p1_round"] > 0
    else:
        assert st["ws_p1_round"] == 0
    # no short-round collapse after a fallback (round 2: ~3.5 pair steps per round)
    assert m8.n_rounds_ <= 1.5 * m1.n_rounds_ + 64
    assert m8.n_iter_ / m8.n_rounds_ > 0.5 * m1.n_iter_ / m1.n_rounds_
    assert _kkt_gap(X, y, m8.alpha_, 100.0, 0.5) < 2e-3 + 2e-4


@pytest.mark.parametrize("clip", ["independent", "box"])
def test_ws_cache_multi_block_bit_identical_to_resident_gram(clip):
    """Multi-block rounds on the kernel-row cache: the union's lines come from
    an 8192-line CLOCK window (misses computed by one row GEMM per round).  The
    K values and the round arithmetic are the dense engine's, so the trajectory
    — including the adaptive block count — is bit-identical to ws-dense with the
    same blocks (its Gram three-product: gram_adapt off), with a cache small
    enough to evict."""
    X, y = synthetic("mnist", n=14000, seed=12)
    kw = dict(C=10.0, gamma=0.25, eps=1e-3, clip=clip, device="cuda", solver="ws", ws_blocks=4, ws_size=64)
    dense = SVC(gram_adapt="off", **kw).fit(X, y)
    cache = SVC(force_cache=True, cache_lines=9000, **kw).fit(X, y)
    assert dense.setup_info_["iteration"] == "ws-dense" and cache.setup_info_["iteration"] == "ws-cache"
    assert "ws_blocks" not in cache.setup_info_.get("engine_note", "")
    assert cache.stats_["ws_blocks"] == 4
    assert cache.converged_ and cache.n_iter_ == dense.n_iter_ and cache.n_rounds_ == dense.n_rounds_
    assert np.array_equal(cache.alpha_, dense.alpha_) and cache.b_ == dense.b_
    assert cache.stats_["ws_blocks_end"] == dense.stats_["ws_blocks_end"]
    assert cache.stats_["rows_computed"] > 9000  # more rows than lines: evictions happened


@pytest.mark.parametrize("clip", ["box", "independent"])
def test_shrinking_reaches_the_stop_test_on_the_whole_problem(clip):
    """solve_shrinking: phases on the active rows (free alphas and bounded ones
    that can still violate), the inactive rows' gradient updated by a predict
    GEMM over each phase's changes; the result satisfies the reference's stop
    test on the exact float64 gradient of the WHOLE problem, and (box clipping:
    unique optimum) matches the unshrunk solve."""
    X, y = synthetic("covtype", n=30000, seed=8)
    C_, g = 64.0, 0.25
    kw = dict(C=C_, gamma=g, eps=1e-3, clip=clip, device="cuda", solver="ws", max_iter=5_000_000)
    full = SVC(shrink="off", **kw).fit(X, y)
    shr = SVC(shrink="on", **kw).fit(X, y)
    assert shr.setup_info_["iteration"] == "ws+shrinking" and shr.stats_["shrink_phases"] >= 2
    assert full.converged_, (full.status_, full.n_iter_, full.stats_)
    assert shr.converged_, (shr.status_, shr.n_iter_, shr.stats_)
    gap = _kkt_gap(X, y, shr.alpha_, C_, g)
    print(f"{clip}: phases {shr.stats_['shrink_phases']} gap {gap:.2e} b {shr.b_:.5f} vs {full.b_:.5f} "
          f"nsv {shr.n_support_} vs {full.n_support_} steps {shr.n_iter_} vs {full.n_iter_}")
    assert gap < 2e-3 + 5e-4
    assert np.all((shr.alpha_ >= 0) & (shr.alpha_ <= C_))
    if clip == "box":
        assert abs(shr.b_ - full.b_) < 2e-2
        assert abs(shr.n_support_ - full.n_support_) <= max(5, full.n_support_ // 50)


@pytest.mark.parametrize("world", [2, 3])
def test_shrinking_multi_rank(world):
    """Shrinking phases over a communicator (ranks as threads sharing the GPU):
    each phase is a rows-sharded multi-rank solve, the inactive rows' update is
    split over the ranks and all-gathered — every rank ends on the same alpha
    bits, at the one-rank optimum (box clipping: unique), through the same
    number of phases' stop tests on the whole problem."""
    from dpsvm_amd._native import load

    X, y = synthetic("covtype", n=20000, seed=8)
    C_, g = 64.0, 0.25
    kw = dict(C=C_, gamma=g, eps=1e-3, clip="box", device="cuda", solver="ws", shrink="on", dp="shard",
              max_iter=5_000_000)
    one = SVC(**kw).fit(X, y)
    outs = _fit_threads(load(), world, X, y, **kw)
    for o in outs:
        assert o.setup_info_["iteration"] == "ws+shrinking" and o.converged_
        assert np.array_equal(o.alpha_, outs[0].alpha_) and o.b_ == outs[0].b_
        assert o.stats_["shrink_phases"] >= 2 and o.stats_["world"] == world
    assert one.converged_
    assert abs(outs[0].b_ - one.b_) < 2e-2
    assert abs(outs[0].n_support_ - one.n_support_) <= max(5, one.n_support_ // 50)
    assert _kkt_gap(X, y, outs[0].alpha_, C_, g) < 2e-3 + 5e-4


def test_shrink_auto_judges_the_rank_shard_not_the_whole_gram():
    """shrink="auto" at world > 1 compares the per-rank Gram footprint of the
    sharded solve (n x n / P columns) with the device budget, not the whole n x n
    Gram: a cap that holds half of the headline's Gram but not
    all of it shrinks at one rank and not at two (dp auto / shard), and still
    shrinks at two with dp replicate."""
    import threading

    from dpsvm_amd import SVCConfig
    from dpsvm_amd._native import load

    C = load()
    n, d = 60000, 784
    out = {}
    for world, dp in ((1, "auto"), (2, "auto"), (2, "replicate")):
        p = SVCConfig(C=10.0, gamma=0.25, cache_mb=10000, dp=dp).to_native(d)  # 10 GB: 14.4 GB whole, 7.2 GB a shard
        if world == 1:
            out[(world, dp)] = [bool(C.shrink_auto(p, n, d, 0, None))]
            continue
        g = C.ThreadCommGroup(world)
        comms = [g.comm(r) for r in range(world)]
        res = [None] * world

        def work(r):
            res[r] = bool(C.shrink_auto(p, n, d, 0, comms[r]))

        ts = [threading.Thread(target=work, args=(r,)) for r in range(world)]
        [t.start() for t in ts]
        [t.join() for t in ts]
        out[(world, dp)] = res
    assert out[(1, "auto")] == [True]
    assert out[(2, "auto")] == [False, False]
    assert out[(2, "replicate")] == [True, True]


def test_shrinking_lends_the_whole_solvers_cache_bit_identically(monkeypatch):
    """A shrunk phase whose Gram does not fit the memory the whole-problem
    solver leaves gets that solver's cache (release_cache; the next whole phase
    allocates it again and recaptures its graphs).  Forced for every phase here
    (DPSVM_SHRINK_RELEASE=1, read once per process: a fresh interpreter): the
    run is bit-identical to one that keeps the cache."""
    import json
    import os
    import subprocess
    import sys

    code = ("import json, sys, hashlib; sys.path.insert(0, %r)\n"
            "from dpsvm_amd import SVC\nfrom dpsvm_amd.utils.datasets import synthetic\n"
            "X, y = synthetic('covtype', n=30000, seed=8)\n"
            "c = SVC(C=64.0, gamma=0.25, eps=1e-3, clip='box', device='cuda', solver='ws', max_iter=5_000_000,"
            " shrink='on', force_cache=True, cache_lines=20000).fit(X, y)\n"
            "print(json.dumps({'sha': hashlib.sha256(c.alpha_.tobytes()).hexdigest(), 'b': float(c.b_),"
            " 'phases': int(c.stats_['shrink_phases']), 'conv': bool(c.converged_)}))\n"
            % os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    outs = []
    for rel in ("0", "1"):
        env = dict(os.environ, DPSVM_SHRINK_RELEASE=rel)
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(json.loads(r.stdout.strip().splitlines()[-1]))
    assert outs[0]["phases"] >= 2 and outs[0]["conv"]
    assert outs[0] == outs[1]
