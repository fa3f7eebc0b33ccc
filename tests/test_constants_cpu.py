"""Python mirrors of device_state.hpp constants stay in step with the header."""
import re
from pathlib import Path

HDR = Path(__file__).resolve().parents[1] / "dpsvm_amd/csrc/include/dpsvm/device_state.hpp"


def header_int(name):
    m = re.search(rf"constexpr int {name} = (\d+);", HDR.read_text())
    assert m, name
    return int(m.group(1))


def test_candidate_list_width_matches_header():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "k", Path(__file__).resolve().parents[1] / "dpsvm_amd/ops/kernels.py")
    src = Path(spec.origin).read_text()
    m = re.search(r"^WS_CAND = (\d+)", src, re.M)
    assert m and int(m.group(1)) == header_int("kWsCand")
    t = (Path(__file__).resolve().parent / "test_ws_kernels_gpu.py").read_text()
    m = re.search(r"^KC = (\d+)", t, re.M)
    assert m and int(m.group(1)) == header_int("kWsCand")
