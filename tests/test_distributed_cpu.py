"""Multi-rank SMO on CPU: the native solver sharded over ranks must make the
same decisions as one rank (packed-key MIN all-reduce, deterministic ties).

  * in-process ranks (ThreadCommGroup — the CLI's --ranks)
  * multi-process ranks over torch.distributed/gloo (the bench/torchrun path)
"""
import os
import socket
import threading

import numpy as np
import pytest
import torch.multiprocessing as mp

from dpsvm_amd import SVC
from dpsvm_amd.utils.datasets import synthetic


def _fit_single(X, y, **kw):
    return SVC(device="cpu", **kw).fit(X, y)


def test_thread_ranks_identical(C):
    X, y = synthetic("blobs", n=700, d=6, seed=21, sep=1.2)
    kw = dict(C=1.5, gamma=0.3, eps=1e-3)
    ref = _fit_single(X, y, **kw)
    for world in (2, 3, 5):
        g = C.ThreadCommGroup(world)
        comms = [g.comm(r) for r in range(world)]
        out = [None] * world

        def work(r):
            out[r] = SVC(device="cpu", **kw).fit(X, y, comm=comms[r])

        ts = [threading.Thread(target=work, args=(r,)) for r in range(world)]
        [t.start() for t in ts]
        [t.join() for t in ts]
        for r in range(world):
            assert out[r].n_iter_ == ref.n_iter_
            assert np.array_equal(out[r].alpha_, ref.alpha_)
            assert out[r].b_ == ref.b_


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from dpsvm_amd.parallel import init_distributed, make_comm, shutdown

    ctx = init_distributed(device="cpu")
    comm = make_comm(ctx)
    assert comm.name == "callback" and comm.size == world and comm.rank == rank
    X, y = synthetic("adult", n=900, seed=4)
    clf = SVC(C=1.0, gamma=0.1, eps=1e-3, device="cpu").fit(X, y, comm=comm)
    q.put((rank, clf.n_iter_, clf.alpha_.tobytes(), clf.b_))
    del comm
    shutdown(ctx)


@pytest.mark.parametrize("world", [2, 3, 8])  # 8: the rank count of one MI355X node
def test_gloo_multiprocess_identical(world):
    X, y = synthetic("adult", n=900, seed=4)
    ref = _fit_single(X, y, C=1.0, gamma=0.1, eps=1e-3)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in procs]
    res = [q.get(timeout=300) for _ in range(world)]
    [p.join(timeout=60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    for rank, it, ab, b in res:
        assert it == ref.n_iter_
        assert np.array_equal(np.frombuffer(ab, dtype=np.float32), ref.alpha_)
        assert b == ref.b_


def _dying_worker(rank, world, port, ck, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), DPSVM_FAULT="exit@300:1")
    from dpsvm_amd.parallel import init_distributed, make_comm

    ctx = init_distributed(device="cpu", timeout_s=30)
    comm = make_comm(ctx)
    X, y = synthetic("blobs", n=800, d=6, seed=31, sep=1.0)
    try:
        SVC(device="cpu", C=1.0, gamma=0.3, checkpoint_path=ck, checkpoint_every=100).fit(X, y, comm=comm)
        q.put((rank, "finished"))
    except Exception as e:  # noqa: BLE001
        q.put((rank, "error: " + str(e)[:200]))


def test_dead_rank_fails_survivors_and_checkpoint_resumes(tmp_path):
    """rank 1's process dies mid-solve (DPSVM_FAULT=exit@300:1).
    The surviving rank must fail (collective error), not hang, and the last
    checkpoint resumes the job at another rank count on the same trajectory."""
    import time

    world, port, ck = 2, _free_port(), str(tmp_path / "ck.bin")
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    ps = [ctxm.Process(target=_dying_worker, args=(r, world, port, ck, q)) for r in range(world)]
    t0 = time.time()
    [p.start() for p in ps]
    [p.join(timeout=120) for p in ps]
    alive = [p for p in ps if p.is_alive()]
    for p in alive:
        p.kill()
    assert not alive, "a surviving rank hung after its peer died"
    assert time.time() - t0 < 120
    assert ps[1].exitcode == 3  # the injected death
    msgs = dict(q.get(timeout=5) for _ in range(1))
    assert msgs.get(0, "").startswith("error"), msgs
    from dpsvm_amd._native import load

    c = load().read_checkpoint(ck)
    assert 0 < c.iter <= 300
    X, y = synthetic("blobs", n=800, d=6, seed=31, sep=1.0)
    full = SVC(device="cpu", C=1.0, gamma=0.3).fit(X, y)
    res = SVC(device="cpu", C=1.0, gamma=0.3).fit(X, y, resume=ck)
    assert res.n_iter_ == full.n_iter_ and np.array_equal(res.alpha_, full.alpha_)
