"""dpsvm_amd — MI355X-native distributed RBF C-SVM trainer (modified SMO).

Capabilities of farshid83/dpsvm (binary RBF C-SVM, first-order maximal
violating pair SMO, row-sharded data parallelism, LRU kernel-row cache, text
model files, CPU trainer + predictor), re-designed for AMD Instinct MI355X:
hand-written CDNA4 HIP kernels (fp32 MFMA kernel rows / Gram / predict, wave-64
selection reductions, device-resident iteration captured in hipGraphs), RCCL
over xGMI for the per-iteration collective, one process (or thread) per GPU.

Quick start::

    from dpsvm_amd import SVC, datasets
    X, y = datasets.synthetic("mnist", n=60000)
    clf = SVC(C=10, gamma=0.25, eps=1e-3).fit(X, y)     # GPU if present
    clf.save("model.txt"); print(clf.n_iter_, clf.n_support_, clf.score(X, y))
"""
from __future__ import annotations

__version__ = "0.1.0"

from .models.svc import SVC, SVCConfig, load_model  # noqa: E402
from .utils import datasets  # noqa: E402
from . import parallel  # noqa: E402

__all__ = ["SVC", "SVCConfig", "load_model", "datasets", "parallel", "native"]


def native():
    """The native extension module (built in-tree on first use)."""
    from ._native import load

    return load()
