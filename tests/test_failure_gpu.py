"""Rank death on the GPU path: with
DPSVM_FAULT=exit@K:1 rank 1's process dies mid-solve; the surviving rank must
fail on its own within 60 s (the in-kernel peer exchange gives up and the
solve raises).  In-process ranks (svmTrain --ranks / -p) whose rank 1 THROWS
(DPSVM_FAULT=throw@K:1, thread alive) must abort the peer's communicator and
report rank 1's error as the root cause."""
import os
import socket
import subprocess
import sys
import time

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_dead_rank_process_survivor_fails_within_60s():
    port = _free_port()
    procs = []
    t0 = time.time()
    for r in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE="2",
                   LOCAL_RANK=str(r), DPSVM_FORCE_DEVICE="0", DPSVM_FAULT="exit@2000:1")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "_fault_worker.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=150)
            outs.append(out)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    elapsed = time.time() - t0
    assert procs[1].returncode == 3, outs[1][-2000:]  # the injected death
    assert procs[0].returncode != 0, outs[0][-2000:]
    assert "rank 0: error" in outs[0], outs[0][-2000:]
    # process start-up (torch import, device init, setup) included
    assert elapsed < 90, elapsed


def _cli_throw(tmp_path, extra):
    exe = os.path.join(ROOT, "bin", "svmTrain")
    if not os.path.exists(exe):
        pytest.skip("bin/svmTrain not built")
    env = dict(os.environ, DPSVM_FAULT="throw@2000:1")
    t0 = time.time()
    r = subprocess.run([exe, "-a", "784", "-x", "12000", "--synthetic", "mnist", "-c", "10", "-g", "0.25", "-m",
                        str(tmp_path / "m.txt"), "--solver", "ws", "--dp", "shard", *extra],
                       capture_output=True, text=True, timeout=120, env=env)
    return r, time.time() - t0


def test_thread_rank_throw_cli_reports_root_cause(tmp_path):
    """DPSVM_FAULT=throw@K:1 inside rank 1's solve thread (process alive): the
    CLI aborts rank 0's communicator, rank 0 leaves its blocked collective
    through the abort, and the process exits non-zero with rank 1's error."""
    r, dt = _cli_throw(tmp_path, ["--ranks", "2", "--xch-timeout", "15"])
    assert r.returncode != 0 and dt < 60, (r.returncode, dt, r.stderr[-2000:])
    err = r.stderr
    assert "rank 1 failed first (root cause)" in err, err[-2000:]
    assert "fault injection: rank 1 throws" in err.strip().splitlines()[-1], err[-2000:]
    assert "rank 0 (after rank 1 failed)" in err and "aborted" in err, err[-2000:]


def test_rccl_rank_throw_cli_reports_root_cause(tmp_path):
    """The same over RCCL (-p 2, one GPU per rank thread): rank 0's owning
    thread carries out the requested ncclCommAbort and fails."""
    if torch.cuda.device_count() < 2:
        pytest.skip("needs 2 GPUs")
    r, dt = _cli_throw(tmp_path, ["-p", "2"])
    assert r.returncode != 0 and dt < 60, (r.returncode, dt, r.stderr[-2000:])
    err = r.stderr
    assert "rank 1 failed first (root cause)" in err, err[-2000:]
    assert "fault injection: rank 1 throws" in err.strip().splitlines()[-1], err[-2000:]
    assert "rank 0 (after rank 1 failed)" in err and "aborted" in err, err[-2000:]


def _cli_throw_phase(tmp_path, extra):
    exe = os.path.join(ROOT, "bin", "svmTrain")
    if not os.path.exists(exe):
        pytest.skip("bin/svmTrain not built")
    env = dict(os.environ, DPSVM_FAULT="throwphase@1:1")
    t0 = time.time()
    r = subprocess.run([exe, "-a", "54", "-x", "20000", "--synthetic", "covtype", "-c", "4", "-g", "0.5", "-m",
                        str(tmp_path / "m.txt"), "--shrink=on", "--clip", "box", *extra],
                       capture_output=True, text=True, timeout=180, env=env)
    return r, time.time() - t0


def test_thread_rank_throw_at_shrink_boundary_reports_root_cause(tmp_path):
    """DPSVM_FAULT=throwphase@1:1: rank 1 throws right after shrinking phase 1,
    while rank 0 goes on into the phase boundary's collectives (agreement,
    inactive-row gather) — it must leave them through the abort and the CLI
    must report rank 1 as the root cause, not hang."""
    r, dt = _cli_throw_phase(tmp_path, ["--ranks", "2", "--xch-timeout", "15"])
    assert r.returncode != 0 and dt < 150, (r.returncode, dt, r.stderr[-2000:])
    err = r.stderr
    assert "rank 1 failed first (root cause)" in err, err[-2000:]
    assert "throws after shrink phase 1" in err.strip().splitlines()[-1], err[-2000:]


def test_rccl_rank_throw_at_shrink_boundary_reports_root_cause(tmp_path):
    """The same over RCCL (-p 2): rank 0's waits on its device collectives are
    bounded (sync_collective polls the communicator's abort), so the owning
    thread leaves them once rank 1 failed."""
    if torch.cuda.device_count() < 2:
        pytest.skip("needs 2 GPUs")
    r, dt = _cli_throw_phase(tmp_path, ["-p", "2"])
    assert r.returncode != 0 and dt < 150, (r.returncode, dt, r.stderr[-2000:])
    assert "rank 1 failed first (root cause)" in r.stderr, r.stderr[-2000:]
