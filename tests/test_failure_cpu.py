"""In-process rank failure (VERDICT round 3 "what's weak" 6):
DPSVM_FAULT=throw@K:R makes rank R's solve throw while its thread lives on.
The CLI must abort the peers' communicators (a surviving rank blocked in a
collective leaves it through abort(), not a watchdog), exit non-zero well
within the bound, and name rank R's own error as the root cause."""
import os
import time

from conftest import ROOT, run


def test_thread_rank_throw_aborts_peers_and_reports_root_cause(tmp_path):
    exe = os.path.join(ROOT, "bin", "svmTrain")
    env = dict(os.environ, DPSVM_FAULT="throw@300:1")
    t0 = time.time()
    r = run([exe, "-a", "64", "-x", "3000", "--synthetic", "mnist", "-c", "10", "-g", "0.25",
             "-m", str(tmp_path / "m.txt"), "--cpu", "--ranks", "2"], env=env, timeout=120, cwd=str(tmp_path))
    assert r.returncode != 0
    assert time.time() - t0 < 60
    err = r.stderr
    # the process fails with rank 1's error, the root cause, reported last
    assert "rank 1 failed first (root cause)" in err, err
    assert err.strip().splitlines()[-1] == "svmTrain: fault injection: rank 1 throws at iteration 300", err
    # rank 0 was waiting in a collective on rank 1 and left it through the abort
    assert "rank 0 (after rank 1 failed): ThreadComm aborted" in err, err
    assert not (tmp_path / "m.txt").exists()


def test_throw_fault_ignores_other_ranks(tmp_path):
    exe = os.path.join(ROOT, "bin", "svmTrain")
    env = dict(os.environ, DPSVM_FAULT="throw@300:5")  # no rank 5: the run is unaffected
    r = run([exe, "-a", "64", "-x", "2000", "--synthetic", "mnist", "-c", "10", "-g", "0.25",
             "-m", str(tmp_path / "m.txt"), "--cpu", "--ranks", "2"], env=env, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr
    assert "Converged at iteration number" in r.stdout
