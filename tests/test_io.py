"""CSV / LIBSVM readers, model files (dpsvm + legacy seq formats), converters."""
import os

import numpy as np
import pytest

from dpsvm_amd import SVC, load_model
from dpsvm_amd.utils import convert, datasets


def test_csv_roundtrip(tmp_path):
    X, y = datasets.synthetic("covtype", n=500, seed=1)
    p = str(tmp_path / "a.csv")
    datasets.write_csv(p, X, y)
    X2, y2 = datasets.read_csv(p)
    assert X2.shape == (500, 54) and np.array_equal(X, X2) and np.array_equal(y, y2)
    # first n rows only (parse.cpp:23)
    X3, _ = datasets.read_csv(p, n=10)
    assert X3.shape == (10, 54) and np.array_equal(X3, X[:10])
    X4, y4 = datasets.read_csv_rows(p, 100, 20, 54)
    assert np.array_equal(X4, X[100:120]) and np.array_equal(y4, y[100:120])


def test_csv_errors(tmp_path):
    p = tmp_path / "bad.csv"
    p.write_text("1,0.5,abc\n")
    with pytest.raises(RuntimeError):
        datasets.read_csv(str(p), d=2)
    with pytest.raises(RuntimeError):
        datasets.read_csv(str(tmp_path / "missing.csv"))
    p.write_text("1,1,2,3\n")
    with pytest.raises(RuntimeError):  # more features than d
        datasets.read_csv(str(p), d=2)


def test_synthetic_rank_slices_match():
    X, y = datasets.synthetic("mnist", n=1000, seed=9)
    Xs, ys = datasets.synthetic("mnist", n=1000, seed=9, row0=250, rows=300)
    assert np.array_equal(Xs, X[250:550]) and np.array_equal(ys, y[250:550])
    assert X.shape == (1000, 784) and 0.15 < (X > 0).mean() < 0.23
    assert set(np.unique(y)) == {-1.0, 1.0}


def test_model_file_format(tmp_path):
    X, y = datasets.synthetic("blobs", n=200, d=3, seed=2)
    clf = SVC(C=1.0, gamma=0.5, device="cpu").fit(X, y)
    p = str(tmp_path / "m.txt")
    clf.save(p)
    lines = open(p).read().strip().split("\n")
    assert abs(float(lines[0]) - 0.5) < 1e-7            # gamma
    assert abs(float(lines[1]) - clf.b_) < 1e-6         # b
    assert len(lines) - 2 == clf.n_support_             # one line per SV
    first = lines[2].split(",")
    assert len(first) == 2 + 3 and first[1] in ("1", "-1")
    m = load_model(p, device="cpu")
    assert m.n_support == clf.n_support_
    assert np.allclose(m.decision_function(X), clf.decision_function(X), atol=1e-5)
    # legacy seq format (no b line) is auto-detected
    pl = str(tmp_path / "legacy.txt")
    clf.save(pl, legacy=True)
    ml = load_model(pl, device="cpu")
    assert ml.b == 0.0 and ml.n_support == clf.n_support_
    # 6 significant digits = the reference's ostream default
    p6 = str(tmp_path / "m6.txt")
    clf.save(p6, precision=6)
    assert abs(load_model(p6, device="cpu").gamma - 0.5) < 1e-6


def test_libsvm_reader(tmp_path):
    p = tmp_path / "s.txt"
    p.write_text("+1 1:1 5:1 123:1\n-1 2:0.5\n")
    X, y = datasets.read_libsvm(str(p), d=123)
    assert X.shape == (2, 123) and X[0, 0] == 1 and X[0, 4] == 1 and X[0, 122] == 1 and X[1, 1] == 0.5
    assert list(y) == [1.0, -1.0]


def test_converters(tmp_path):
    src = tmp_path / "mnist_train.csv"
    src.write_text("4,0,255,51\n7,255,0,0\n")
    out = convert.convert_mnist(str(src))
    assert out.endswith("mnist_train_conv.csv")
    rows = [r.split(",") for r in open(out).read().strip().split("\n")]
    assert rows[0][0] == "1" and rows[1][0] == "-1"
    assert abs(float(rows[0][2]) - 1.0) < 1e-9 and abs(float(rows[0][3]) - 0.2) < 1e-9
    a9a = tmp_path / "a9a.txt"
    a9a.write_text("-1 3:1 11:1 123:1\n+1 1:1\n")
    o = convert.convert_adult(str(a9a))
    r = [x.split(",") for x in open(o).read().strip().split("\n")]
    assert len(r[0]) == 124 and r[0][0] == "-1" and r[0][3] == "1" and r[0][123] == "1" and r[1][1] == "1"
    # legacy shift: feature k lands one column right, 123 dropped
    ol = convert.convert_adult(str(a9a), str(tmp_path / "legacy.csv"), legacy_shift=True)
    rl = [x.split(",") for x in open(ol).read().strip().split("\n")]
    assert len(rl[0]) == 124 and rl[0][4] == "1" and rl[0][1] == "0" and rl[1][2] == "1"
    X, y = datasets.read_csv(o, d=123)
    assert X.shape == (2, 123) and X[0, 2] == 1.0
