"""Device-resident SMO on MI355X vs the CPU oracle; cache modes; simulated
multi-rank on one GPU; checkpoint/resume; predictor; bench on GPU."""
import json
import os
import sys
import threading

import numpy as np
import pytest
import torch

from dpsvm_amd import SVC as _SVC
from dpsvm_amd import load_model
from dpsvm_amd.utils.datasets import synthetic

pytestmark = pytest.mark.gpu


def SVC(*args, **kw):
    """this module covers every device engine: the quarantined pair-at-a-time
    cache / partitioned-X engines included (engines=all; the production rows
    come first in the choice, so dense problems run the same engines)"""
    kw.setdefault("engines", "all")
    return _SVC(*args, **kw)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _worker_errors(out, world):
    msgs = []
    for k in range(world):
        p = f"{out}.rank{k}.err"
        if os.path.exists(p):
            msgs.append(f"rank {k}: " + open(p).read()[-1500:])
    return "\n".join(msgs) + "\n"


def _close(g, c, n):
    assert g.converged_ and c.converged_
    assert abs(g.n_iter_ - c.n_iter_) <= max(10, c.n_iter_ // 50)
    assert abs(g.n_support_ - c.n_support_) <= max(3, c.n_support_ // 100)
    assert abs(g.b_ - c.b_) < 1e-2


@pytest.mark.parametrize("mode", ["dense", "lru", "lru_tiny", "partitioned"])
def test_gpu_matches_cpu(mode):
    X, y = synthetic("adult", n=4000, seed=3)
    kw = dict(C=1.0, gamma=0.05, eps=1e-3)
    cpu = SVC(device="cpu", **kw).fit(X, y)
    extra = {"dense": {}, "lru": {"cache_lines": 256}, "lru_tiny": {"cache_lines": 2, "spec_rows": 0},
             "partitioned": {"x_mode": "partitioned"}}[mode]
    gpu = SVC(device="cuda", **kw, **extra).fit(X, y)
    _close(gpu, cpu, 4000)
    if mode == "dense":
        assert gpu.setup_info_["cache_lines"] == 4000
    else:
        assert gpu.stats_["cache_misses"] > 0
    assert abs(gpu.train_accuracy() - cpu.score(X, y)) < 0.01


def test_gpu_box_clip_and_max_iter():
    X, y = synthetic("blobs", n=3000, d=16, seed=5, sep=1.0)
    g = SVC(C=1.0, gamma=0.1, clip="box", device="cuda").fit(X, y)
    assert g.converged_ and abs(float((g.alpha_ * y).sum())) < 1e-2
    g2 = SVC(C=1.0, gamma=0.1, max_iter=1000, device="cuda").fit(X, y)
    assert g2.n_iter_ == 1000 and g2.status_ == 2
    g3 = SVC(C=1.0, gamma=0.1, max_iter=1000, use_graph=False, device="cuda").fit(X, y)
    assert np.array_equal(g2.alpha_, g3.alpha_)  # graph replay == eager launches


def test_simulated_ranks_one_gpu_identical(C):
    """P ranks as threads sharing the GPU (host-staged collectives) must make
    bit-identical decisions to one rank."""
    X, y = synthetic("covtype", n=6000, seed=2)
    kw = dict(C=4.0, gamma=0.5, eps=1e-3, device="cuda")
    # bitwise identity holds across rank counts within one cache mode (the Gram
    # GEMM and the row kernel accumulate dot products in different orders)
    for world, extra in ((2, {}), (3, {"x_mode": "partitioned"}), (4, {"cache_lines": 64})):
        ref = SVC(**kw, **extra).fit(X, y)
        g = C.ThreadCommGroup(world)
        comms = [g.comm(r) for r in range(world)]
        out = [None] * world
        errs = []

        def work(r):
            try:
                out[r] = SVC(**kw, **extra).fit(X, y, comm=comms[r])
            except Exception as e:  # pragma: no cover
                errs.append(e)

        ts = [threading.Thread(target=work, args=(r,)) for r in range(world)]
        [t.start() for t in ts]
        [t.join() for t in ts]
        assert not errs, errs
        for r in range(world):
            assert out[r].n_iter_ == ref.n_iter_, (world, extra)
            assert np.array_equal(out[r].alpha_, ref.alpha_)


def test_gpu_checkpoint_resume(tmp_path):
    X, y = synthetic("blobs", n=5000, d=24, seed=9, sep=1.0)
    full = SVC(C=1.0, gamma=0.05, device="cuda").fit(X, y)
    ck = str(tmp_path / "ck.bin")
    part = SVC(C=1.0, gamma=0.05, device="cuda", max_iter=full.n_iter_ // 2, checkpoint_path=ck,
               checkpoint_every=max(1, full.n_iter_ // 5)).fit(X, y)
    assert not part.converged_ and os.path.exists(ck)
    res = SVC(C=1.0, gamma=0.05, device="cuda").fit(X, y, resume=ck)
    assert res.n_iter_ == full.n_iter_
    assert np.array_equal(res.alpha_, full.alpha_)


def test_gpu_predictor_and_model_file(tmp_path):
    X, y = synthetic("mnist-parity", n=3000, seed=4)
    clf = SVC(C=10.0, gamma=0.02, device="cuda").fit(X, y)
    Xt, yt = synthetic("mnist-parity", n=1000, seed=5)
    dec_gpu = clf.decision_function(Xt)
    p = str(tmp_path / "m.txt")
    clf.save(p)
    m = load_model(p, device="cpu")
    dec_cpu = m.decision_function(Xt)
    assert np.allclose(dec_gpu, dec_cpu, atol=2e-4, rtol=1e-4)
    assert load_model(p, device="cuda").score(Xt, yt) > 0.9


def test_mnist_shape_headline_converges():
    """The BASELINE config (60000 x 784, C=10, gamma=0.25, tol=1e-3) on one GPU."""
    X, y = synthetic("mnist", n=60000, seed=0)
    # solver auto from 50k rows: ws-dense (here with 8 blocks per round, bench.py's setting)
    auto = SVC(C=10.0, gamma=0.25, eps=1e-3, device="cuda", ws_blocks=8).fit(X, y)
    assert auto.setup_info_["iteration"] == "ws-dense" and auto.converged_ and auto.n_rounds_ < 400
    assert auto.train_accuracy() > 0.99
    # the pair-at-a-time engine (the reference's trajectory)
    clf = SVC(C=10.0, gamma=0.25, eps=1e-3, device="cuda", solver="smo").fit(X, y)
    assert clf.converged_
    assert clf.fit_time_ < 30.0
    assert clf.train_accuracy() > 0.99
    assert abs(auto.b_ - clf.b_) < 2e-3
    # > 65535 iterations: the persistent engine's 16-bit exchange tags wrap;
    # one launch per iteration (no exchange) must give the same iterates
    assert clf.setup_info_["iteration"] == "persistent-dense" and clf.n_iter_ > 70000
    ref = SVC(C=10.0, gamma=0.25, eps=1e-3, device="cuda", persist="off", solver="smo").fit(X, y)
    assert ref.n_iter_ == clf.n_iter_ and np.array_equal(ref.alpha_, clf.alpha_) and ref.b_ == clf.b_


def test_bench_gpu_small():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    import subprocess

    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--samples", "8000", "--steps", "2",
                        "--warmup", "1"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    out = json.loads([l for l in r.stdout.split("\n") if l.startswith("{")][-1])
    assert out["converged"] and out["n_gpus"] == 1 and out["train_accuracy"] > 0.99


@pytest.mark.parametrize("extra", [{}, {"cache_lines": 128}, {"x_mode": "partitioned"}])
def test_rccl_one_rank_collective_path(C, extra):
    """The RCCL collective + hipGraph capture path, exercised on one GPU with a
    one-rank communicator (force_collectives): identical to the local path."""
    X, y = synthetic("adult", n=3000, seed=1)
    kw = dict(C=1.0, gamma=0.05, device="cuda", **extra)
    ref = SVC(**kw).fit(X, y)
    comm = C.rccl_comm(C.rccl_unique_id(), 0, 1, 0)
    assert comm.name == "rccl" and comm.device_memory
    got = SVC(force_collectives=True, **kw).fit(X, y, comm=comm)
    assert got.n_iter_ == ref.n_iter_
    assert np.array_equal(got.alpha_, ref.alpha_)
    assert abs(got.train_accuracy() - ref.train_accuracy()) < 1e-9


def test_cache_policies_bitwise_identical():
    """K(i, j) from the row kernel is bitwise independent of when/where it is
    computed, so every cache configuration (tiny device cache, speculation,
    host spill tier) must reproduce the same SMO trajectory exactly."""
    X, y = synthetic("covtype", n=5000, seed=6)
    kw = dict(C=4.0, gamma=0.5, device="cuda")
    ref = SVC(cache_lines=4096, **kw).fit(X, y)
    tiny = SVC(cache_lines=2, spec_rows=0, **kw).fit(X, y)
    spill = SVC(cache_lines=24, host_cache_lines=512, **kw).fit(X, y)
    for other in (tiny, spill):
        assert other.n_iter_ == ref.n_iter_
        assert np.array_equal(other.alpha_, ref.alpha_)
    assert spill.stats_["host_hits"] > 0
    assert tiny.stats_["cache_misses"] > ref.stats_["cache_misses"]


def test_gpu_fault_injection_and_verify(monkeypatch, C):
    X, y = synthetic("blobs", n=3000, d=8, seed=3, sep=1.0)
    monkeypatch.setenv("DPSVM_FAULT", "nan@200")
    clf = SVC(C=1.0, gamma=0.1, device="cuda", graph_block=16, persist_block=16).fit(X, y)
    assert clf.status_ == 4 and not clf.converged_ and clf.n_iter_ >= 200
    monkeypatch.delenv("DPSVM_FAULT")
    monkeypatch.setenv("DPSVM_VERIFY", "1")
    comm = C.rccl_comm(C.rccl_unique_id(), 0, 1, 0)
    ok = SVC(C=1.0, gamma=0.1, device="cuda", force_collectives=True).fit(X, y, comm=comm)
    assert ok.converged_


@pytest.mark.parametrize("engine", ["persistent", "fused", "cache", "fused-cache", "chain", "partitioned"])
def test_verify_invariants_every_engine(monkeypatch, engine):
    """DPSVM_VERIFY=1: alpha in [0, C] and the incrementally updated f equals f
    recomputed from alpha (predict GEMM) at the end of the run, for every engine."""
    monkeypatch.setenv("DPSVM_VERIFY", "1")
    X, y = synthetic("mnist-parity", n=3000, seed=2)
    kw = dict(C=10.0, gamma=0.25, device="cuda")
    if engine == "fused":
        kw["persist"] = "off"
    elif engine in ("cache", "fused-cache", "chain"):
        kw["cache_lines"] = 64
        if engine == "fused-cache":
            kw["persist"] = "off"
        if engine == "chain":
            kw["cache_engine"] = "chain"
    elif engine == "partitioned":
        kw["x_mode"] = "partitioned"
    clf = SVC(**kw).fit(X, y)
    assert clf.converged_
    assert 0.0 <= clf.stats_["verify_f_err"] < 1e-4
    # also mid-run (max_iter stop): f and alpha must agree after any iteration
    part = SVC(max_iter=777, **kw).fit(X, y)
    assert part.n_iter_ == 777 and 0.0 <= part.stats_["verify_f_err"] < 1e-4


@pytest.mark.parametrize("extra", [{"cache_lines": 64}, {"cache_lines": 2, "spec_rows": 0},
                                   {"cache_lines": 24, "host_cache_lines": 8}])
def test_fused_cache_iteration_matches_kernel_chain(monkeypatch, extra):
    """The one-launch cache-mode iteration (smo_fused_lru) and the
    rows/step/finalize chain compute bit-identical kernel rows, so they must
    follow the same SMO trajectory (whatever their cache decisions)."""
    X, y = synthetic("covtype", n=5000, seed=6)
    kw = dict(C=4.0, gamma=0.5, device="cuda", persist="off", **extra)
    fused = SVC(**kw).fit(X, y)
    assert fused.setup_info_["iteration"] == "fused-cache"
    chain = SVC(cache_engine="chain", **kw).fit(X, y)
    assert chain.setup_info_["iteration"] == "chain"
    assert fused.n_iter_ == chain.n_iter_
    assert np.array_equal(fused.alpha_, chain.alpha_)
    assert fused.stats_["cache_misses"] > 0
    if extra.get("host_cache_lines"):
        assert fused.stats_["host_hits"] > 0


def test_fused_cache_wide_features_and_checkpoint(monkeypatch, tmp_path):
    """d > one LDS k-chunk (multi-chunk X pass) + checkpoint/resume in cache mode."""
    X, y = synthetic("blobs", n=2500, d=1100, seed=8, sep=1.0)
    kw = dict(C=1.0, gamma=1.0 / 1100, device="cuda", cache_lines=48, persist="off")
    cpu = SVC(C=1.0, gamma=1.0 / 1100, device="cpu").fit(X, y)
    full = SVC(**kw).fit(X, y)
    assert full.setup_info_["iteration"] == "fused-cache"
    _close(full, cpu, 2500)
    ck = str(tmp_path / "ck.bin")
    part = SVC(max_iter=full.n_iter_ // 2, checkpoint_path=ck, checkpoint_every=max(1, full.n_iter_ // 4),
               **kw).fit(X, y)
    assert not part.converged_
    res = SVC(**kw).fit(X, y, resume=ck)
    assert res.n_iter_ == full.n_iter_
    assert np.array_equal(res.alpha_, full.alpha_)
    chain = SVC(cache_engine="chain", **kw).fit(X, y)
    assert np.array_equal(chain.alpha_, full.alpha_)


@pytest.mark.parametrize("case", ["covtype-spec", "covtype-nospec", "tiny-cache", "wide", "max-iter", "box"])
def test_persistent_cache_engine_matches_fused(monkeypatch, case):
    """Persistent cache engine (private per-workgroup CLOCK metadata, keys
    exchanged in-kernel, X pass per workgroup) == the one-launch-per-iteration
    cache engine, bit for bit: same kernel rows, same trajectory."""
    if case == "wide":
        X, y = synthetic("blobs", n=2500, d=1100, seed=8, sep=1.0)
        kw = dict(C=1.0, gamma=1.0 / 1100, cache_lines=48)
    else:
        X, y = synthetic("covtype", n=6000, seed=6)
        kw = dict(C=4.0, gamma=0.5, cache_lines=256)
    kw.update({"covtype-spec": {}, "covtype-nospec": {"spec_rows": 0}, "tiny-cache": {"cache_lines": 2, "spec_rows": 0},
               "wide": {}, "max-iter": {"max_iter": 1500}, "box": {"clip": "box"}}[case])
    got = SVC(device="cuda", persist_block=301, xch_timeout_s=30.0, **kw).fit(X, y)
    assert got.setup_info_["iteration"] == "persistent-cache"
    ref = SVC(device="cuda", persist="off", **kw).fit(X, y)
    assert ref.setup_info_["iteration"] == "fused-cache"
    assert got.n_iter_ == ref.n_iter_ and got.status_ == ref.status_
    assert np.array_equal(got.alpha_, ref.alpha_) and got.b_ == ref.b_
    assert got.stats_["cache_misses"] > 0 and got.stats_["x_passes"] > 0
    if case == "max-iter":
        assert got.n_iter_ == 1500 and got.status_ == 2


def test_peer_exchange_loopback_and_thread_ranks(monkeypatch, C):
    """In-kernel peer exchange of the selection keys (dense mode): a one-rank
    loopback reproduces the local run bit for bit; rank threads sharing one
    device in one process fall back to the all-reduce (their streams may share
    a hardware queue) with identical results."""
    X, y = synthetic("covtype", n=6000, seed=2)
    kw = dict(C=4.0, gamma=0.5, eps=1e-3, device="cuda", xch_timeout_s=30.0)
    ref = SVC(persist="off", **kw).fit(X, y)
    assert ref.setup_info_["exchange"] == "none"
    loop = SVC(exchange="peer", persist="off", **kw).fit(X, y)
    assert loop.setup_info_["exchange"] == "loopback" and loop.setup_info_["iteration"] == "fused-dense"
    assert loop.n_iter_ == ref.n_iter_ and np.array_equal(loop.alpha_, ref.alpha_)
    g = C.ThreadCommGroup(2)
    comms = [g.comm(r) for r in range(2)]
    out = [None, None]
    errs = []

    def work(r):
        try:
            out[r] = SVC(**kw).fit(X, y, comm=comms[r])
        except Exception as e:  # pragma: no cover
            errs.append(e)

    ts = [threading.Thread(target=work, args=(r,)) for r in range(2)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errs, errs
    for r in range(2):
        assert out[r].setup_info_["exchange"] == "allreduce"
        assert out[r].n_iter_ == ref.n_iter_ and np.array_equal(out[r].alpha_, ref.alpha_)


@pytest.mark.parametrize("block,rows", [(2048, None), (37, None), (501, 3072)])
def test_persistent_engine_matches_fused(monkeypatch, block, rows):
    """Persistent dense kernel (keys exchanged in-kernel, row state in
    registers) == one launch per iteration, bit for bit; also across launches
    of an odd block length, at max_iter, and with 12 rows per thread."""
    X, y = synthetic("covtype", n=6000, seed=2)
    kw = dict(C=4.0, gamma=0.5, eps=1e-3, device="cuda", xch_timeout_s=30.0, rows_per_group=rows or 0)
    ref = SVC(persist="off", **kw).fit(X, y)
    got = SVC(persist="on", persist_block=block, **kw).fit(X, y)
    assert got.setup_info_["iteration"] == "persistent-dense"
    assert got.n_iter_ == ref.n_iter_ and got.status_ == ref.status_
    assert np.array_equal(got.alpha_, ref.alpha_)
    assert got.b_ == ref.b_
    m = SVC(persist="on", persist_block=block, max_iter=1000, **kw).fit(X, y)
    m_ref = SVC(persist="off", max_iter=1000, **kw).fit(X, y)
    assert m.n_iter_ == 1000 and m.status_ == 2 and np.array_equal(m.alpha_, m_ref.alpha_)


@pytest.mark.parametrize("clip", ["independent", "box"])
def test_persistent_eta_from_gram_matches_to_tolerance(clip):
    """eta="gram": the persistent dense engine takes K(hi, lo) from the resident
    Gram instead of the two X rows (no sample-row reads, one barrier fewer).
    The GEMM rounds K differently from the explicit difference, so the run is
    pinned to the float64 oracle of the reference algorithm and to the default
    engine at tolerance level, not bit for bit; ignored (default path) in cache mode."""
    from ref_smo import decision, smo_reference
    X, y = synthetic("blobs", n=2500, d=12, seed=41, sep=1.2)
    C_, g = 2.0, 0.15
    kw = dict(C=C_, gamma=g, eps=1e-3, clip=clip, device="cuda", persist="on", xch_timeout_s=30.0)
    ref = SVC(**kw).fit(X, y)
    got = SVC(eta="gram", **kw).fit(X, y)
    assert got.setup_info_["iteration"] == "persistent-dense" and got.converged_
    assert abs(got.n_iter_ - ref.n_iter_) <= max(20, ref.n_iter_ // 20)
    assert abs(got.b_ - ref.b_) < 2e-3
    assert abs(got.n_support_ - ref.n_support_) <= max(3, ref.n_support_ // 50)
    a_o, b_o, it_o = smo_reference(X, y, C=C_, gamma=g, eps=1e-3, clip=clip)
    assert abs(got.n_iter_ - it_o) <= max(10, it_o // 20) and abs(got.b_ - b_o) < 5e-3
    assert np.abs(got.alpha_ - a_o).max() < 5e-2 * C_
    d_o = decision(X, y, a_o, b_o, g, X)
    assert np.mean(np.sign(got.decision_function(X)) == np.sign(d_o)) > 0.995
    # cache mode has no resident Gram: the flag changes nothing there
    c0 = SVC(cache_lines=256, **kw).fit(X, y)
    c1 = SVC(cache_lines=256, eta="gram", **kw).fit(X, y)
    assert c0.n_iter_ == c1.n_iter_ and np.array_equal(c0.alpha_, c1.alpha_)


@pytest.mark.parametrize("engine", ["fused", "persistent", "persistent-batches", "persistent-cache"])
def test_peer_exchange_two_processes_one_gpu(tmp_path, engine):
    """Two ranks as two processes sharing the GPU (gloo bootstrap, IPC-mapped
    receive buffers): in-kernel exchange, bit-identical to one rank.
    persistent-batches: 256-row workgroups and one publication per lane per
    poll round, so each poll sweeps its 2 x 40 publications in two batches."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    import subprocess

    n = 20000 if engine == "persistent-batches" else 6000
    env = dict(os.environ, DPSVM_FORCE_DEVICE="0", DPSVM_VERIFY="1")
    extra_json = json.dumps({"rows_per_group": 256, "xch_poll_batch": 1} if engine == "persistent-batches" else {})
    out = tmp_path / "mp"
    port = 29600 + ["fused", "persistent", "persistent-batches", "persistent-cache"].index(engine)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(root, "tests", "mp_exchange_worker.py"), str(out), engine, str(n), extra_json]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=root)
    assert r.returncode == 0, _worker_errors(out, 2) + r.stderr[-2000:]
    res = [json.load(open(f"{out}.rank{k}.json")) for k in range(2)]
    X, y = synthetic("covtype", n=n, seed=2)
    extra = {"cache_lines": 256} if engine == "persistent-cache" else {}
    ref = SVC(C=4.0, gamma=0.5, eps=1e-3, device="cuda", **extra).fit(X, y)
    want = {"fused": "fused-dense", "persistent-cache": "persistent-cache"}.get(engine, "persistent-dense")
    for k in range(2):
        assert res[k]["exchange"] == "peer" and res[k]["exchange_mem"] == "uncached"
        assert res[k]["iteration"] == want
        assert res[k]["iters"] == ref.n_iter_
        assert res[k]["alpha_sha"] == __import__("hashlib").sha256(ref.alpha_.tobytes()).hexdigest()


@pytest.mark.parametrize("world", [4, 8])
@pytest.mark.parametrize("engine", ["persistent", "persistent-cache"])
def test_peer_exchange_four_processes_one_gpu(tmp_path, engine, world):
    """Four (eight) ranks as four (eight) processes sharing the GPU: every
    workgroup pushes its publication to `world` receive buffers and polls
    world x G of them; the result is bit-identical to one rank (rehearsal of
    the 4- and 8-GPU runs: same rank count and shard geometry)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    import subprocess

    n = 8000
    env = dict(os.environ, DPSVM_FORCE_DEVICE="0", DPSVM_VERIFY="1")
    out = tmp_path / f"mp{world}"
    port = 29620 + ["persistent", "persistent-cache"].index(engine) + (4 if world == 8 else 0)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(root, "tests", "mp_exchange_worker.py"), str(out), engine, str(n)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=root)
    assert r.returncode == 0, _worker_errors(out, world) + r.stderr[-2000:]
    res = [json.load(open(f"{out}.rank{k}.json")) for k in range(world)]
    X, y = synthetic("covtype", n=n, seed=2)
    extra = {"cache_lines": 256} if engine == "persistent-cache" else {}
    ref = SVC(C=4.0, gamma=0.5, eps=1e-3, device="cuda", **extra).fit(X, y)
    sha = __import__("hashlib").sha256(ref.alpha_.tobytes()).hexdigest()
    for k in range(world):
        assert res[k]["exchange"] == "peer" and res[k]["exchange_mem"] == "uncached"
        assert res[k]["iteration"] == ("persistent-cache" if engine == "persistent-cache" else "persistent-dense")
        assert res[k]["iters"] == ref.n_iter_ and res[k]["alpha_sha"] == sha


def test_bench_two_processes_exchange_fallback(tmp_path):
    """bench.py with 2 ranks: a peer exchange that gives up (1 us poll bound)
    makes every rank fail the warmup run the same way; the bench falls back
    to the all-reduce path and still reports a verified time."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    import subprocess

    env = dict(os.environ, DPSVM_FORCE_DEVICE="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29611", os.path.join(root, "bench.py"), "--gpus", "2",
           "--samples", "4000", "--steps", "1", "--warmup", "1", "--comm", "gloo", "--xch-timeout", "0.000001",
           "--solver", "smo"]  # the pair-at-a-time engines' peer exchange
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=root)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.split("\n") if l.startswith("{")][-1])
    assert out["exchange"] == "allreduce" and out["converged"] and out["n_gpus"] == 2
    assert "falling back" in r.stderr


_SHARED = os.environ.get("DPSVM_TEST_SHARED_GPU") == "1"
_NDEV = torch.cuda.device_count() if torch.cuda.is_available() else 0
_MULTI = pytest.mark.skipif(not _SHARED and _NDEV < 2,
                            reason="needs >= 2 GPUs (DPSVM_TEST_SHARED_GPU=1 rehearses it on one)")


def _bench_multi(root, world, extra, port):
    import subprocess

    env = dict(os.environ)
    comm = ["--comm", "gloo"] if _SHARED else ["--comm", "rccl"]
    if _SHARED:
        env["DPSVM_FORCE_DEVICE"] = "0"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
           "--gpus", str(world), "--samples", "8000", "--steps", "1", "--warmup", "1", "--no-accuracy"] + comm + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=root)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return json.loads([l for l in r.stdout.split("\n") if l.startswith("{")][-1])


def _ref_8000():
    X, y = synthetic("mnist", n=8000, d=784, seed=0)
    return SVC(C=10.0, gamma=0.25, eps=1e-3, device="cuda").fit(X, y)


@_MULTI
def test_bench_multi_gpu_sharded_matches_one_gpu(tmp_path):
    """bench.py as one process per GPU with the rows SHARDED (RCCL communicator
    over xGMI, in-kernel peer exchange between devices) on up to 8 GPUs: same
    iteration count, b and SV count as the one-GPU solve, cross-rank verified.
    DPSVM_TEST_SHARED_GPU=1 runs the same ranks on one GPU over gloo."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    world = 2 if _SHARED else min(_NDEV, 8)
    out = _bench_multi(root, world, ["--dp", "shard", "--solver", "smo"], 29641)
    assert out["n_gpus"] == world and out["converged"] and out["exchange"] == "peer"
    assert out["dp_policy"] == "shard" and out["exchange_mem"] == "uncached"
    assert out["comm"] != "local" and out["config"]["parallelism"] == f"dp{world}"
    ref = _ref_8000()
    assert out["iterations"] == ref.n_iter_ and out["b"] == ref.b_
    assert out["n_sv"] == int((ref.alpha_ > 0).sum())


@pytest.mark.skipif(_NDEV < 2, reason="needs >= 2 GPUs (replication needs distinct devices)")
def test_bench_multi_gpu_auto_policy_replicates_and_checks_shards(tmp_path):
    """Default policy on distinct GPUs for a problem whose Gram fits one GPU:
    every rank solves it all (no per-iteration hop), and the untimed sharded
    check solve reports the same iterations and b."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    world = min(_NDEV, 8)
    out = _bench_multi(root, world, ["--solver", "smo"], 29651)
    ref = _ref_8000()
    # the timed runs use whichever policy measured faster on this node; the
    # pair-at-a-time engine is bit-identical to one GPU either way
    assert out["dp_autotune"]["chosen"] == out["dp_policy"]
    assert out["iterations"] == ref.n_iter_ and out["b"] == ref.b_
    sc = out["shard_check"]
    assert sc and "error" not in sc, sc
    assert sc["exchange"] == "peer" and sc["iterations"] == ref.n_iter_ and sc["b"] == ref.b_


@_MULTI
def test_bench_multi_gpu_ws_sharded_and_default(tmp_path):
    """bench.py defaults (working-set engine) on up to 8 GPUs: sharded rows
    (per-round candidate all-gather + sub-Gram sum over RCCL, graph-captured)
    converge to the one-GPU optimum, cross-rank verified; the default policy
    replicates on distinct GPUs and its untimed sharded check succeeds."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    world = 2 if _SHARED else min(_NDEV, 8)
    # bench.py's default: 8 sub-problems per round (multi-block rounds); sharded
    # ranks read other candidate lists than one GPU, so b agrees to the stop gap
    ref = SVC(C=10.0, gamma=0.25, eps=1e-3, device="cuda", solver="ws",
              ws_blocks=8).fit(*synthetic("mnist", n=8000, d=784, seed=0))
    out = _bench_multi(root, world, ["--dp", "shard"], 29661)
    assert out["iteration"] == "ws-dense" and out["dp_policy"] == "shard" and out["converged"]
    # RCCL: multi-block rounds; gloo rehearsal: one-block rounds over the peer exchange
    assert out["params"]["ws_blocks"] in (0, 8) and (_SHARED or "ws_blocks" not in out["engine_note"])
    assert abs(out["b"] - ref.b_) < 2e-3 and abs(out["n_sv"] - ref.n_support_) <= 8
    if _NDEV >= 2:
        dflt = _bench_multi(root, world, [], 29671)
        assert dflt["dp_autotune"]["chosen"] == dflt["dp_policy"]
        if dflt["dp_policy"] == "replicate":
            assert dflt["iterations"] == ref.n_iter_ and dflt["b"] == ref.b_
        assert abs(dflt["b"] - ref.b_) < 2e-3
        sc = dflt["shard_check"]
        assert sc and "error" not in sc and sc["engine"] == "ws-dense", sc
        assert abs(sc["b"] - ref.b_) < 2e-3


def test_bench_two_processes_measured_dp_policy(tmp_path):
    """--dp measure (the default's measured choice, forced on shared-GPU
    rehearsal ranks): the replicated solve and one sharded solve are both timed
    (max over ranks, identical on every rank), the timed runs use the faster,
    and the JSON line records both times and the choice."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    import subprocess

    env = dict(os.environ, DPSVM_FORCE_DEVICE="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29615", os.path.join(root, "bench.py"), "--gpus", "2",
           "--samples", "6000", "--steps", "1", "--warmup", "1", "--comm", "gloo", "--dp", "measure",
           "--no-accuracy", "--reference-check", "off"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=root)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.split("\n") if l.startswith("{")][-1])
    at, sc = out["dp_autotune"], out["shard_check"]
    assert sc and "error" not in sc, sc
    assert at and at["chosen"] in ("shard", "replicate") and at["replicate_s"] > 0 and at["shard_s"] > 0
    assert out["dp_policy"] == at["chosen"] and out["converged"] and out["n_gpus"] == 2
    assert abs(sc["b"] - out["b"]) < 1e-3


@pytest.mark.skipif(_NDEV < 2, reason="needs >= 2 GPUs (svmTrain -p N: one thread per device)")
@pytest.mark.parametrize("ranks", [2, 8])
@pytest.mark.parametrize("dp", ["shard", "auto"])
def test_svmtrain_in_process_multi_gpu(tmp_path, bin_dir, ranks, dp):
    """svmTrain -p N: one process, one thread per GPU, ncclCommInitAll, the
    in-kernel exchange over same-process peer pointers (hipDeviceEnablePeerAccess).
    Sharded: bit-identical iterations and b to one rank; auto: replicated solve.
    The cross-rank alpha digest runs by default."""
    if ranks > _NDEV:
        pytest.skip(f"needs {ranks} GPUs")
    import subprocess

    outs = {}
    for p_ in (1, ranks):
        mj = str(tmp_path / f"m{p_}.json")
        cmd = [os.path.join(bin_dir, "svmTrain"), "-a", "784", "-x", "8000", "--synthetic", "mnist", "-c", "10",
               "-g", "0.25", "-m", str(tmp_path / f"model{p_}.txt"), "-p", str(p_), "--dp", dp,
               "--metrics-json", mj, "--xch-timeout", "30"]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        outs[p_] = json.load(open(mj))
    one, many = outs[1], outs[ranks]
    assert many["world"] == ranks and many["iterations"] == one["iterations"] and many["b"] == one["b"]
    assert many["n_sv"] == one["n_sv"]
    if dp == "shard":
        assert many["dp_policy"] == "shard" and many["exchange"] == "peer"
        assert many["engine"] == "persistent-dense"
    else:
        assert many["dp_policy"] == "replicate"


def test_census_forced_oversubscription_falls_back():
    """A persistent grid that cannot be co-resident (here: a census grid of
    4096 workgroups, more than the device holds) is detected at setup within
    the census bound and the solver falls back to the one-launch-per-iteration
    engine, bit-identical, instead of spinning to the exchange timeout."""
    import time

    X, y = synthetic("covtype", n=6000, seed=2)
    kw = dict(C=4.0, gamma=0.5, eps=1e-3, device="cuda", xch_timeout_s=30.0)
    ref = SVC(**kw).fit(X, y)
    assert ref.setup_info_["iteration"] == "persistent-dense" and ref.setup_info_["census"] == "ok"
    assert ref.setup_info_["blocks_per_cu"] >= 1 and ref.setup_info_["cus"] >= 1
    t0 = time.perf_counter()
    got = SVC(census_groups=4096, **kw).fit(X, y)
    assert time.perf_counter() - t0 < 20.0
    assert got.setup_info_["census"] == "failed" and got.setup_info_["iteration"] == "fused-dense"
    assert "census" in got.setup_info_["engine_note"]
    assert got.n_iter_ == ref.n_iter_ and np.array_equal(got.alpha_, ref.alpha_)
    # cache mode: persistent cache engine -> fused cache engine
    cref = SVC(cache_lines=256, **kw).fit(X, y)
    assert cref.setup_info_["iteration"] == "persistent-cache"
    cgot = SVC(cache_lines=256, census_groups=4096, **kw).fit(X, y)
    assert cgot.setup_info_["iteration"] == "fused-cache" and cgot.setup_info_["census"] == "failed"
    assert cgot.n_iter_ == cref.n_iter_ and np.array_equal(cgot.alpha_, cref.alpha_)
    # persist="on" (required) refuses loudly instead of falling back
    with pytest.raises(Exception, match="co-resident"):
        SVC(persist="on", census_groups=4096, **kw).fit(X, y)


def test_gpu_resume_rejects_mismatched_problem(tmp_path):
    X, y = synthetic("blobs", n=3000, d=16, seed=9, sep=1.0)
    ck = str(tmp_path / "ck.bin")
    SVC(C=1.0, gamma=0.05, device="cuda", max_iter=300, checkpoint_path=ck, checkpoint_every=100).fit(X, y)
    with pytest.raises(Exception, match="gamma"):
        SVC(C=1.0, gamma=0.5, device="cuda").fit(X, y, resume=ck)
    with pytest.raises(Exception, match="C ="):
        SVC(C=0.5, gamma=0.05, device="cuda").fit(X, y, resume=ck)
    ok = SVC(C=1.0, gamma=0.05, eps=1e-2, device="cuda").fit(X, y, resume=ck)  # eps may differ
    assert ok.converged_


@pytest.mark.parametrize("p_from,p_to", [(2, 1), (2, 3)])
def test_gpu_checkpoint_resume_other_rank_count(tmp_path, C, p_from, p_to):
    """A checkpoint written by P simulated ranks (alpha + all-gathered f) resumes
    at P' ranks and finishes on the uninterrupted trajectory."""
    X, y = synthetic("covtype", n=6000, seed=2)
    kw = dict(C=4.0, gamma=0.5, eps=1e-3, device="cuda")
    full = SVC(**kw).fit(X, y)
    ck = str(tmp_path / "ck.bin")

    def run(world, resume=None, **extra):
        if world == 1:
            return [SVC(**kw, **extra).fit(X, y, resume=resume)]
        g = C.ThreadCommGroup(world)
        comms = [g.comm(r) for r in range(world)]
        out, errs = [None] * world, []

        def work(r):
            try:
                out[r] = SVC(**kw, **extra).fit(X, y, comm=comms[r], resume=resume)
            except Exception as e:  # pragma: no cover
                errs.append(e)

        ts = [threading.Thread(target=work, args=(r,)) for r in range(world)]
        [t.start() for t in ts]
        [t.join() for t in ts]
        assert not errs, errs
        return out

    part = run(p_from, max_iter=full.n_iter_ // 2, checkpoint_path=ck, checkpoint_every=max(1, full.n_iter_ // 5))
    assert not part[0].converged_ and os.path.exists(ck)
    assert C.read_checkpoint(ck).iter == full.n_iter_ // 2
    res = run(p_to, resume=ck)
    for r in res:
        assert r.n_iter_ == full.n_iter_ and np.array_equal(r.alpha_, full.alpha_)


_ORACLE_ENGINES = {
    "persistent-dense": {},
    "fused-dense": {"persist": "off"},
    "persistent-cache": {"cache_lines": 64},
    "fused-cache": {"cache_lines": 64, "persist": "off"},
    "chain": {"cache_lines": 64, "cache_engine": "chain"},
    "partitioned": {"x_mode": "partitioned"},
}


@pytest.mark.parametrize("clip", ["independent", "box"])
@pytest.mark.parametrize("engine", sorted(_ORACLE_ENGINES))
def test_gpu_engines_vs_float64_numpy_oracle(engine, clip):
    """Every device engine vs an independent float64 numpy model of the
    reference algorithm (tests/ref_smo.py: svmTrainMain.cpp:235-310), not the
    builder's own CPU solver: same iterations (fp32 vs fp64 arithmetic allow a
    small drift), same alphas, b and support set."""
    from ref_smo import smo_reference

    X, y = synthetic("blobs", n=2500, d=12, seed=41, sep=1.2)
    C_, g = 2.0, 0.15
    a_ref, b_ref, it_ref = smo_reference(X, y, C=C_, gamma=g, eps=1e-3, clip=clip)
    clf = SVC(C=C_, gamma=g, eps=1e-3, clip=clip, device="cuda", **_ORACLE_ENGINES[engine]).fit(X, y)
    want = "chain" if engine == "partitioned" else engine
    assert clf.setup_info_["iteration"] == want
    assert clf.converged_
    assert abs(clf.n_iter_ - it_ref) <= max(10, it_ref // 20), (clf.n_iter_, it_ref)
    assert np.abs(clf.alpha_ - a_ref).max() < 5e-2 * C_
    assert abs(clf.b_ - b_ref) < 5e-3
    sv_ours, sv_ref = set(np.nonzero(clf.alpha_ > 0)[0]), set(np.nonzero(a_ref > 0)[0])
    assert len(sv_ours ^ sv_ref) <= max(3, len(sv_ref) // 50)


def test_gpu_box_clip_vs_sklearn_libsvm():
    """Box clipping reaches LIBSVM's optimum (scikit-learn's libsvm, second-order
    working sets): SV count, intercept, and decision signs agree."""
    sk = pytest.importorskip("sklearn.svm")
    X, y = synthetic("adult", n=3000, seed=2)
    C_, g = 1.0, 0.05
    ref = sk.SVC(C=C_, gamma=g, kernel="rbf", tol=1e-3).fit(X, y)
    for extra in ({}, {"cache_lines": 64}):
        clf = SVC(C=C_, gamma=g, eps=1e-3, clip="box", device="cuda", **extra).fit(X, y)
        n_ref = int(ref.n_support_.sum())
        assert abs(clf.n_support_ - n_ref) <= max(5, n_ref // 50)
        assert abs(-clf.b_ - ref.intercept_[0]) < 0.05
        agree = np.mean(np.sign(clf.decision_function(X)) == np.sign(ref.decision_function(X)))
        assert agree > 0.99
        assert abs(float((clf.alpha_ * np.where(y > 0, 1, -1)).sum())) < 1e-2
