"""Loader for the in-tree native extension ``dpsvm_amd._C``.

torch is imported first when available so that torch's bundled HIP runtime
(same soname ``libamdhip64.so.7``) is the single HIP runtime in the process.
On a machine with a GPU the extension is REQUIRED: a missing or stale build
raises instead of silently falling back to Python code.
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import sys

_C = None
_ERR: Exception | None = None


def _try_import_torch() -> None:
    try:
        import torch  # noqa: F401
    except Exception:  # torch is optional for the CPU-only native paths
        pass


def load(build_if_missing: bool = True):
    """Return the native module, building it in-tree if it is absent."""
    global _C, _ERR
    if _C is not None:
        return _C
    _try_import_torch()
    alt = os.environ.get("DPSVM_NATIVE_SO")  # A/B runs: another in-tree build of the same module
    if alt:
        spec = importlib.util.spec_from_file_location("dpsvm_amd._C", alt)
        _C = importlib.util.module_from_spec(spec)
        sys.modules["dpsvm_amd._C"] = _C
        spec.loader.exec_module(_C)
        return _C
    try:
        _C = importlib.import_module("dpsvm_amd._C")
        return _C
    except ImportError as e:
        _ERR = e
    if build_if_missing and os.environ.get("DPSVM_NO_AUTOBUILD", "0") != "1":
        from . import build as _build

        _build.build(clis=True)
        importlib.invalidate_caches()
        _C = importlib.import_module("dpsvm_amd._C")
        return _C
    raise ImportError(f"dpsvm_amd native extension not built: {_ERR}. Run `python -m dpsvm_amd.build`.")


_PAIRQ = None


def load_quarantine():
    """Load the plugin with the quarantined pair-at-a-time cache /
    partitioned-X engines (libdpsvm_pairq.so, next to the module; it registers
    them with the solver when loaded).  engines="all" needs it (tests, A/B
    probes); the production module never does."""
    global _PAIRQ
    if _PAIRQ is not None:
        return _PAIRQ
    C = load()
    import ctypes

    path = os.path.join(os.path.dirname(os.path.abspath(C.__file__)), "libdpsvm_pairq.so")
    if not os.path.exists(path):
        raise ImportError(f"the pair-cache plugin is not built ({path}); run `python -m dpsvm_amd.build`")
    _PAIRQ = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    if not C.quarantine_loaded():
        raise ImportError(f"{path} loaded but did not register its engines")
    return _PAIRQ


def gpu_available() -> bool:
    """True when a HIP device is usable (via torch when present)."""
    try:
        import torch

        return bool(torch.cuda.is_available()) and torch.cuda.device_count() > 0
    except Exception:
        try:
            return load().device_count() > 0
        except Exception:
            return False


def require_gpu() -> None:
    if not gpu_available():
        raise RuntimeError("dpsvm_amd: no HIP device available (device='cuda' requested)")
    load()


def is_loaded_from_tree() -> bool:
    m = sys.modules.get("dpsvm_amd._C")
    return m is not None and os.path.dirname(os.path.abspath(m.__file__)) == os.path.dirname(__file__)
