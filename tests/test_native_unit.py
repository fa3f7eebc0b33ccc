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
