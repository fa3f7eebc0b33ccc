"""Native C++ unit tests (bin/dpsvm_unit): keys, sharding, I/O, checkpoints,
CPU solver rank invariance; `--gpu` adds the device solver modes."""
import os

import pytest

from conftest import run


def test_native_unit_cpu(bin_dir):
    r = run([os.path.join(bin_dir, "dpsvm_unit")])
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed" in r.stdout


@pytest.mark.gpu
def test_native_unit_gpu(bin_dir):
    r = run([os.path.join(bin_dir, "dpsvm_unit"), "--gpu"])
    assert r.returncode == 0, r.stdout + r.stderr
    assert "gpu                          ok" in r.stdout


def test_host_asan_build_unit_and_cpu_cli(tmp_path):
    """Host AddressSanitizer build (`python -m dpsvm_amd.build --asan`, SURVEY
    §5.2; GPU ASan is not available on this pool): the native unit suite, the
    CPU trainer (checkpoint + model write) and the predictor run clean under it."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = run([sys.executable, "-m", "dpsvm_amd.build", "--asan", "-q"], cwd=root)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    b = os.path.join(root, "build", "rel-asan", "bin")
    # leak checking off: the HIP runtime keeps process-lifetime allocations
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1")
    r = run([os.path.join(b, "dpsvm_unit")], env=env)
    assert r.returncode == 0 and "0 failed" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
    model = str(tmp_path / "m.txt")
    r = run([os.path.join(b, "svmTrain"), "-a", "32", "-x", "2000", "--synthetic", "blobs", "-c", "1",
             "-g", "0.05", "-m", model, "--cpu", "--checkpoint", str(tmp_path / "ck.bin")], env=env)
    assert r.returncode == 0 and "Number of SVs:" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
    assert "AddressSanitizer" not in r.stderr
    from dpsvm_amd.utils.datasets import synthetic, write_csv

    X, y = synthetic("blobs", n=500, d=32, seed=3)
    csv = str(tmp_path / "t.csv")
    write_csv(csv, X, y)
    r = run([os.path.join(b, "svmTest"), "-a", "32", "-x", "500", "-f", csv, "-m", model], env=env)
    assert r.returncode == 0 and "AddressSanitizer" not in r.stderr, r.stdout[-3000:] + r.stderr[-3000:]
