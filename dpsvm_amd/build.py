"""Build the native core for MI355X (gfx950) in-tree.

Products (all git-ignored, shipped to the GPU box with the snapshot):
  dpsvm_amd/_C<EXT_SUFFIX>   pybind11 module (solver, kernels, comm, I/O): the production engines
  dpsvm_amd/libdpsvm_pairq.so  plugin: the quarantined pair-at-a-time cache / partitioned-X
                             engines (loaded for engines="all"; linked into bin/svmTrainPairq
                             and bin/dpsvm_unit only)
  bin/svmTrain               distributed trainer CLI  (reference: svmTrainMain.cpp)
  bin/svmTest                predictor CLI            (reference: seq_test.cpp / Makefile:104)
  bin/svmSeq                 CPU trainer CLI          (reference: seq.cpp)
  bin/dpsvm_unit             native unit tests (CTest-style, run by pytest)
  bin/svmTrainPairq          svmTrain with the quarantined engines linked in (--engines all)

Usage:  python -m dpsvm_amd.build [-j N] [--force] [--debug] [--asan]
Everything is compiled by hipcc (ROCm 7.2) with --offload-arch=gfx950; .cpp files
are host-only C++20, .hip files carry the device code.  Incremental: an object
is rebuilt when its source or any header under csrc/ is newer.
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
BUILD = ROOT / "build"
BIN = ROOT / "bin"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"

LIB_SOURCES = [
    "io/csv.cpp",
    "io/model_io.cpp",
    "io/synth.cpp",
    "comm/comm_host.cpp",
    "comm/comm_rccl.cpp",
    "solver/smo_cpu.cpp",
    "solver/checkpoint.cpp",
    "solver/gpu_setup.hip",
    "solver/gpu_exchange.hip",
    "solver/gpu_engines.hip",
    "solver/gpu_solve.hip",
    "solver/gpu_predict.hip",
    "solver/ws_kernel_entry.hip",
    "solver/gpu_shrink.cpp",
    "kernels/setup_kernels.hip",
    "kernels/rbf_gemm.hip",
    "kernels/rbf_gemm_split.hip",
    "kernels/smo_fused.hip",
    "kernels/microbench.hip",
    "kernels/compact.hip",
    "kernels/smo_persist.hip",
    "kernels/ws_select.hip",
    "kernels/ws_merge.hip",
    "kernels/ws_solve.hip",
    "kernels/ws_recompute.hip",
]
# the quarantined engines (solver/gpu_engines_pairq.hip registers them): a plugin
# library for the Python module, linked into the CLIs (svmTrain --engines all)
PLUGIN_SOURCES = [
    "kernels/smo_kernels.hip",
    "kernels/smo_fused_lru.hip",
    "kernels/smo_persist_lru.hip",
    "solver/gpu_engines_pairq.hip",
]
CLI = {
    "svmTrain": "cli/svm_train.cpp",
    "svmTest": "cli/svm_test.cpp",
    "svmSeq": "cli/svm_seq.cpp",
    "dpsvm_unit": "cli/unit_tests.cpp",
    "svmTrainPairq": "cli/svm_train.cpp",
}
# the CLIs that link the quarantined engines in: the native unit tests and a
# separate trainer for `--engines all`; the default CLIs are production-only
CLI_WITH_PLUGIN = {"dpsvm_unit", "svmTrainPairq"}
BINDINGS = "python/bindings.cpp"


def hipcc() -> str:
    p = ROCM / "bin" / "hipcc"
    return str(p) if p.exists() else (shutil.which("hipcc") or "hipcc")


def ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def module_path() -> Path:
    return PKG / ("_C" + ext_suffix())


def plugin_path() -> Path:
    return PKG / "libdpsvm_pairq.so"


def _headers_mtime() -> float:
    m = 0.0
    for p in CSRC.rglob("*"):
        if p.suffix in (".hpp", ".h", ".cuh"):
            m = max(m, p.stat().st_mtime)
    return m


def _flags(debug: bool, asan: bool) -> list[str]:
    f = ["-std=c++20", "-fPIC", f"-I{CSRC / 'include'}", f"-I{CSRC}", f"-I{ROCM / 'include'}",
         "-Wall", "-Wno-unused-function", "-Wno-unused-variable", "-Wno-unused-result"]
    f += ["-O0", "-g"] if debug else ["-O3"]
    if asan:
        # host-only sanitizer: GPU ASan/xnack+ is not available on this pool
        f += ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer"]
    return f


def _compile(src: Path, obj: Path, flags: list[str], extra: list[str], force: bool, hdr_m: float) -> str:
    if (not force and obj.exists() and obj.stat().st_mtime >= src.stat().st_mtime
            and obj.stat().st_mtime >= hdr_m):
        return f"up-to-date {src.name}"
    obj.parent.mkdir(parents=True, exist_ok=True)
    if src.suffix == ".hip":
        cmd = [hipcc(), "-x", "hip", f"--offload-arch={ARCH}"] + flags + extra + ["-c", str(src), "-o", str(obj)]
    else:
        cmd = [hipcc(), "-x", "c++", "-D__HIP_PLATFORM_AMD__"] + flags + extra + ["-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return f"compiled {src.name}"


def _link(out: Path, objs: list[Path], shared: bool, flags: list[str], extra: list[str] | None = None) -> None:
    out.parent.mkdir(parents=True, exist_ok=True)
    cmd = [hipcc(), f"--offload-arch={ARCH}"] + [str(o) for o in objs] + ["-o", str(out)]
    if shared:
        cmd += ["-shared", f"-Wl,-soname,{out.name}"]
    cmd += extra or []
    cmd += [f"-L{ROCM / 'lib'}", "-lamdhip64", "-lrccl", "-lpthread", f"-Wl,-rpath,{ROCM / 'lib'}"]
    # sanitizer runtimes: each -fsanitize= stays paired with the -Xarch_host before it
    for i, x in enumerate(flags[:-1]):
        if x == "-Xarch_host" and flags[i + 1].startswith("-fsanitize"):
            cmd += [x, flags[i + 1]]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {out}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def build(jobs: int | None = None, force: bool = False, debug: bool = False, asan: bool = False,
          verbose: bool = False, clis: bool = True) -> Path:
    jobs = jobs or min(8, os.cpu_count() or 4)
    flags = _flags(debug, asan)
    tag = ("dbg" if debug else "rel") + ("-asan" if asan else "")
    objdir = BUILD / tag
    hdr_m = _headers_mtime()
    import pybind11

    py_inc = [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]
    tasks = [(CSRC / s, objdir / (s.replace("/", "_") + ".o"), []) for s in LIB_SOURCES + PLUGIN_SOURCES]
    tasks.append((CSRC / BINDINGS, objdir / "bindings.o", py_inc + ["-fvisibility=hidden"]))
    if clis:
        tasks += [(CSRC / s, objdir / (s.replace("/", "_") + ".o"), []) for s in sorted(set(CLI.values()))]
    with ThreadPoolExecutor(jobs) as ex:
        futs = [ex.submit(_compile, s, o, flags, e, force, hdr_m) for s, o, e in tasks]
        for f in futs:
            msg = f.result()
            if verbose:
                print(msg, flush=True)
    lib_objs = [objdir / (s.replace("/", "_") + ".o") for s in LIB_SOURCES]
    mod = module_path() if not (debug or asan) else objdir / ("_C" + ext_suffix())
    newest = max(o.stat().st_mtime for o in lib_objs + [objdir / "bindings.o"])
    if force or not mod.exists() or mod.stat().st_mtime < newest:
        _link(mod, lib_objs + [objdir / "bindings.o"], True, flags)
        if verbose:
            print(f"linked {mod}")
    # the plugin resolves the solver's symbols from the module it sits next to
    plug_objs = [objdir / (s.replace("/", "_") + ".o") for s in PLUGIN_SOURCES]
    plug = plugin_path() if not (debug or asan) else objdir / "libdpsvm_pairq.so"
    newest_p = max([o.stat().st_mtime for o in plug_objs] + [mod.stat().st_mtime])
    if force or not plug.exists() or plug.stat().st_mtime < newest_p:
        _link(plug, plug_objs, True, flags, [str(mod), "-Wl,-rpath,$ORIGIN"])
        if verbose:
            print(f"linked {plug}")
    if clis:
        bindir = BIN if not (debug or asan) else objdir / "bin"
        for name, src in CLI.items():
            o = objdir / (src.replace("/", "_") + ".o")
            out = bindir / name
            extra = plug_objs if name in CLI_WITH_PLUGIN else []
            if force or not out.exists() or out.stat().st_mtime < max(newest, newest_p, o.stat().st_mtime):
                _link(out, lib_objs + extra + [o], False, flags)
                if verbose:
                    print(f"linked {out}")
    return mod


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--asan", action="store_true", help="host-only AddressSanitizer build (build/<tag>/bin)")
    ap.add_argument("--no-cli", action="store_true")
    ap.add_argument("-q", "--quiet", action="store_true")
    a = ap.parse_args(argv)
    mod = build(a.jobs, a.force, a.debug, a.asan, verbose=not a.quiet, clis=not a.no_cli)
    print(f"dpsvm_amd native build OK ({ARCH}): {mod}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
