"""svmTrain / svmSeq / svmTest CLIs: reference flags, stdout lines, model file."""
import os

import numpy as np
import pytest

from conftest import run
from dpsvm_amd.utils import datasets


def _data(tmp_path, n=400):
    X, y = datasets.synthetic("blobs", n=n, d=5, seed=7, sep=1.5)
    p = str(tmp_path / "train.csv")
    datasets.write_csv(p, X, y)
    return p, X, y


def test_svmtrain_cpu_reference_output(tmp_path, bin_dir):
    p, X, y = _data(tmp_path)
    m = str(tmp_path / "model.txt")
    js = str(tmp_path / "metrics.json")
    r = run([os.path.join(bin_dir, "svmTrain"), "-a", "5", "-x", "400", "-f", p, "-c", "2", "-g", "0.4",
             "-e", "0.001", "-m", m, "--cpu", "--metrics-json", js])
    assert r.returncode == 0, r.stderr
    out = r.stdout
    for line in ("Populated Data from input file at node: 0", "SETUP DONE", "TOTAL TIME TAKEN in seconds:",
                 "Converged at iteration number:", "b: ", "Number of SVs:", "Training accuracy:",
                 f"Training model has been saved to the file {m}"):
        assert line in out, (line, out)
    assert "0\t400" in out  # shard table disp\tsize
    import json

    met = json.load(open(js))
    assert met["converged"] and met["n"] == 400 and met["iterations"] > 0
    lines = open(m).read().strip().split("\n")
    assert abs(float(lines[0]) - 0.4) < 1e-7 and len(lines) - 2 == met["n_sv"]


def test_svmtrain_simulated_ranks_cpu(tmp_path, bin_dir):
    p, X, y = _data(tmp_path)
    outs = []
    for ranks in ("1", "3"):
        m = str(tmp_path / f"m{ranks}.txt")
        r = run([os.path.join(bin_dir, "svmTrain"), "-a", "5", "-x", "400", "-f", p, "-c", "2", "-g", "0.4",
                 "-m", m, "--cpu", "--ranks", ranks])
        assert r.returncode == 0, r.stderr
        outs.append(open(m).read())
    assert outs[0] == outs[1]  # identical model from 1 and 3 ranks


def test_svmtrain_usage_errors(tmp_path, bin_dir):
    r = run([os.path.join(bin_dir, "svmTrain"), "-a", "5", "-x", "10"])
    assert r.returncode == 255 and "Enter a valid file name" in r.stderr
    r = run([os.path.join(bin_dir, "svmTrain"), "-f", "x.csv", "-m", "m.txt"])
    assert r.returncode == 255 and "Missing a required parameter" in r.stderr
    r = run([os.path.join(bin_dir, "svmTrain"), "--bogus"])
    assert r.returncode == 255
    r = run([os.path.join(bin_dir, "svmTrain"), "-f", "x.csv", "-m", "m.txt", "--eta", "bogus"])
    assert r.returncode == 255 and "--eta x|gram" in r.stderr


def test_svmtrain_params_roundtrip_new_knobs(tmp_path, bin_dir):
    """--eta and the exchange choice are recorded in --metrics-json and read back
    by --params-json (a run's engine is reproducible from its summary)."""
    import json

    p, X, y = _data(tmp_path)
    js, js2 = str(tmp_path / "a.json"), str(tmp_path / "b.json")
    base = [os.path.join(bin_dir, "svmTrain"), "-a", "5", "-x", "400", "-f", p, "-c", "2", "-g", "0.4",
            "-m", str(tmp_path / "m.txt"), "--cpu"]
    r = run(base + ["--eta", "gram", "--exchange", "peer", "--ws-blocks", "4", "--metrics-json", js])
    assert r.returncode == 0, r.stderr
    pa = json.load(open(js))["params"]
    assert pa["eta"] == 1 and pa["exchange"] == 2 and pa["ws_blocks"] == 4
    r = run(base + ["--params-json", js, "--metrics-json", js2])
    assert r.returncode == 0, r.stderr
    pb = json.load(open(js2))["params"]
    assert pb["eta"] == 1 and pb["exchange"] == 2 and pb["ws_blocks"] == 4


def test_svmseq_and_svmtest(tmp_path, bin_dir):
    p, X, y = _data(tmp_path)
    m = str(tmp_path / "model.txt")
    r = run([os.path.join(bin_dir, "svmSeq"), "-a", "5", "-x", "400", "-f", p, "-c", "2", "-g", "0.4",
             "-m", m])
    assert r.returncode == 0, r.stderr
    assert "Converged at iteration number:" in r.stdout and "Training accuracy:" in r.stdout
    dec_path = str(tmp_path / "dec.txt")
    r = run([os.path.join(bin_dir, "svmTest"), "-a", "5", "-x", "400", "-f", p, "-m", m, "--cpu",
             "--decision-out", dec_path])
    assert r.returncode == 0, r.stderr
    for line in ("Populated test data", "Total number of Support Vectors:", "Populated training model",
                 "Test accuracy:"):
        assert line in r.stdout
    acc = float(r.stdout.split("Test accuracy:")[1].split()[0])
    dec = np.loadtxt(dec_path)
    assert acc > 0.8 and dec.shape == (400,)


def test_svmtrain_synthetic_and_checkpoint_resume(tmp_path, bin_dir):
    m = str(tmp_path / "m.txt")
    ck = str(tmp_path / "ck.bin")
    base = [os.path.join(bin_dir, "svmTrain"), "-a", "4", "-x", "500", "--synthetic", "blobs", "--seed", "3",
            "-c", "1", "-g", "0.5", "--cpu", "-m", m]
    r = run(base + ["--skip-accuracy"])
    full_it = int(r.stdout.split("Converged at iteration number:")[1].split()[0])
    full_model = open(m).read()
    r = run(base + ["-n", str(full_it // 2), "--checkpoint", ck, "--checkpoint-every", str(full_it // 4)])
    assert "Could not converge in" in r.stdout and os.path.exists(ck)
    r = run(base + ["--resume", ck])
    assert r.returncode == 0, r.stderr
    assert f"Converged at iteration number: {full_it}" in r.stdout
    assert open(m).read() == full_model


@pytest.mark.gpu
def test_svmtrain_gpu_matches_cpu_and_svmtest(tmp_path, bin_dir):
    """svmTrain on the GPU (default device): reference stdout lines, the same
    SMO trajectory as --cpu within fp32 tolerance, model read back by svmTest."""
    p, X, y = _data(tmp_path, n=2000)
    outs = {}
    for dev in ("gpu", "cpu"):
        m = str(tmp_path / f"model_{dev}.txt")
        js = str(tmp_path / f"metrics_{dev}.json")
        cmd = [os.path.join(bin_dir, "svmTrain"), "-a", "5", "-x", "2000", "-f", p, "-c", "2", "-g", "0.4",
               "-e", "0.001", "-m", m, "--metrics-json", js] + (["--cpu"] if dev == "cpu" else [])
        r = run(cmd)
        assert r.returncode == 0, r.stderr
        for line in ("SETUP DONE", "Converged at iteration number:", "Training accuracy:"):
            assert line in r.stdout, (line, r.stdout)
        import json

        tr_acc = float([l for l in r.stdout.split("\n") if l.startswith("Training accuracy:")][-1].split()[-1])
        outs[dev] = (json.load(open(js)), m, tr_acc)
    g, c = outs["gpu"][0], outs["cpu"][0]
    assert g["converged"] and c["converged"]
    assert abs(g["iterations"] - c["iterations"]) <= max(10, c["iterations"] // 50)
    assert abs(g["n_sv"] - c["n_sv"]) <= max(3, c["n_sv"] // 100)
    r = run([os.path.join(bin_dir, "svmTest"), "-a", "5", "-x", "2000", "-f", p, "-m", outs["gpu"][1]])
    assert r.returncode == 0, r.stderr
    acc = float([l for l in r.stdout.split("\n") if "accuracy" in l.lower()][-1].split()[-1])
    assert abs(acc - outs["gpu"][2]) < 2e-3  # the predictor reproduces the trainer's accuracy


@pytest.mark.gpu
def test_svmtrain_shrink_matches_plain_box(tmp_path, bin_dir):
    """svmTrain --shrink (one GPU, LIBSVM-style shrinking phases) reaches the
    same joint-box optimum as the plain device run: reference stdout lines, b
    and the support-set size within the stop tolerance's reach."""
    import json

    outs = {}
    for mode in ("plain", "shrink"):
        m = str(tmp_path / f"model_{mode}.txt")
        js = str(tmp_path / f"metrics_{mode}.json")
        cmd = [os.path.join(bin_dir, "svmTrain"), "-a", "54", "-x", "20000", "--synthetic", "covtype", "-c", "32",
               "-g", "0.03125", "-e", "0.001", "-n", "10000000", "--clip", "box", "-m", m, "--metrics-json", js]
        r = run(cmd + (["--shrink"] if mode == "shrink" else []))
        assert r.returncode == 0, r.stderr
        for line in ("SETUP DONE", "Converged at iteration number:", "Training accuracy:"):
            assert line in r.stdout, (line, r.stdout)
        outs[mode] = json.load(open(js))
    p, s = outs["plain"], outs["shrink"]
    assert p["converged"] and s["converged"]
    assert s["engine"] == "ws+shrinking"
    assert abs(p["b"] - s["b"]) < 2e-2
    assert abs(p["n_sv"] - s["n_sv"]) <= max(5, p["n_sv"] // 50)
