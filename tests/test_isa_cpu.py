"""Register-spill guard for the production device kernels (CPU only: hipcc
cross-compiles gfx950 here).

Each listed translation unit is compiled to gfx950 assembly with
``--offload-device-only -S`` and every kernel in it must have a zero private
(scratch) segment: a spilled accumulator or index array costs scratch loads in
the hot loop (round-4 review: ``rbf_gemm_split_w64_kernel<0>`` carried 396 B /
175 scratch instructions in the headline's Gram epilogue).
"""
import os
import re
import subprocess

import pytest

from conftest import ROOT

CSRC = os.path.join(ROOT, "dpsvm_amd", "csrc")
HIPCC = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")

# every kernel of these TUs runs on a production path (Gram / row / predict
# GEMMs, the working-set rounds, the pair-at-a-time dense engines)
SPILL_FREE = [
    "kernels/rbf_gemm_split.hip",
    "kernels/ws_select.hip",
    "kernels/ws_merge.hip",
    "kernels/ws_solve.hip",
    "kernels/ws_recompute.hip",
    "kernels/smo_persist.hip",
    "kernels/compact.hip",
]


def kernel_scratch(tu, tmp_path):
    out = tmp_path / (os.path.basename(tu) + ".s")
    cmd = [HIPCC, "-x", "hip", "--offload-arch=gfx950", "-std=c++20", "-O3", f"-I{CSRC}/include", f"-I{CSRC}",
           "--offload-device-only", "-S", os.path.join(CSRC, tu), "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    s = out.read_text()
    res = {}
    for blk in re.split(r"\n\t\.amdhsa_kernel ", s)[1:]:
        name = blk.split("\n", 1)[0]
        m = re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", blk)
        res[name] = int(m.group(1)) if m else -1
    n_scratch = len(re.findall(r"\bscratch_(?:load|store)_", s))
    return res, n_scratch


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
@pytest.mark.parametrize("tu", SPILL_FREE)
def test_production_kernels_do_not_spill(tu, tmp_path):
    res, n_scratch = kernel_scratch(tu, tmp_path)
    assert res, f"no kernels found in {tu}"
    spilled = {k: v for k, v in res.items() if v != 0}
    assert not spilled and n_scratch == 0, f"{tu}: scratch segments {spilled}, {n_scratch} scratch instructions"
