"""The device solver's engine choice is one table (device_state.hpp kEngineTable,
evaluated by choose_engine() in gpu_setup.hip; kQuarantineTable after it only
with engines=all); docs/DESIGN.md §2 lists the same rows.  CPU only: the table
is host code."""
import os
import re

import pytest

C = pytest.importorskip("dpsvm_amd._C")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRODUCTION = ["ws-dense", "ws-cache", "persistent-dense", "fused-dense"]
QUARANTINE = ["persistent-cache", "fused-cache", "chain"]


def _doc_rows(doc, start, stop):
    sec = doc[doc.index(start):doc.index(stop)]
    rows = re.findall(r"^\| ([a-z-]+)(?: \(§[^)]*\))? \|", sec, flags=re.M)
    return [r for r in rows if r != "engine"]


def test_engine_table_matches_design_doc():
    table = C.engine_table()
    assert [n for n, _ in table] == PRODUCTION  # <= 4 production rows
    full = C.engine_table(quarantine=True)
    assert [n for n, _ in full] == PRODUCTION + QUARANTINE
    with open(os.path.join(ROOT, "docs", "DESIGN.md")) as fh:
        doc = fh.read()
    assert _doc_rows(doc, "**Engine choice**", "**Quarantined rows**") == PRODUCTION, \
        "DESIGN.md §2 engine table out of sync with kEngineTable"
    assert _doc_rows(doc, "**Quarantined rows**", "## 2a.") == QUARANTINE, \
        "DESIGN.md §2 quarantine table out of sync with kQuarantineTable"
    for _, use in full:
        assert use
    for _, use in full[len(PRODUCTION):]:
        assert use.startswith("engines=all")


@pytest.mark.parametrize("facts,want", [
    (dict(ws_dense=True, dense=True, persistent=True), "ws-dense"),
    (dict(ws_cache=True, cache_replicated=True, persistent=True), "ws-cache"),
    (dict(dense=True, persistent=True), "persistent-dense"),
    (dict(dense=True), "fused-dense"),
    (dict(cache_replicated=True, persistent=True), None),
    (dict(cache_replicated=True), None),
    (dict(), None),
    (dict(cache_replicated=True, persistent=True, quarantine=True), "persistent-cache"),
    (dict(cache_replicated=True, quarantine=True), "fused-cache"),
    (dict(quarantine=True), "chain"),
    (dict(persistent=True, quarantine=True), "chain"),
    (dict(ws_cache=True, cache_replicated=True, quarantine=True), "ws-cache"),
])
def test_choose_engine_first_match(facts, want):
    """None: no production row matches — the setup refuses the configuration
    and names engines=all"""
    assert C.choose_engine(**facts) == want


def test_quarantined_engines_are_a_plugin_not_the_production_module():
    """The production module carries no code of the quarantined pair-at-a-time
    cache / partitioned-X engines: their kernels and
    engine classes live in libdpsvm_pairq.so, which registers them when loaded
    (engines="all"); of the CLIs only bin/svmTrainPairq and the native unit
    tests link them in (hygiene)."""
    import subprocess

    from dpsvm_amd import build
    from dpsvm_amd._native import load_quarantine

    def defined(path):
        out = subprocess.run(["nm", "-D", "--defined-only", "-C", str(path)], capture_output=True, text=True)
        assert out.returncode == 0, out.stderr
        return out.stdout

    def defined_all(path):  # executables: the static symbol table
        out = subprocess.run(["nm", "--defined-only", "-C", str(path)], capture_output=True, text=True)
        assert out.returncode == 0, out.stderr
        return out.stdout

    prod = defined(build.module_path())
    for sym in ("smo_fused_lru_kernel", "smo_persist_lru_kernel", "smo_rows_kernel", "smo_finalize_kernel",
                "launch::smo_fused_lru(", "launch::smo_persist_lru(", "launch::smo_rows("):
        assert sym not in prod, f"{sym} is in the production module"
    plug = defined(build.plugin_path())
    for sym in ("launch::smo_fused_lru(", "launch::smo_persist_lru(", "launch::smo_rows("):
        assert sym in plug
    for cli in ("svmTrain", "svmTest", "svmSeq"):
        exe = os.path.join(ROOT, "bin", cli)
        if os.path.exists(exe):
            assert "smo_fused_lru_kernel" not in defined_all(exe), f"{cli} links the quarantined engines"
    exe = os.path.join(ROOT, "bin", "svmTrainPairq")
    if os.path.exists(exe):
        assert "smo_fused_lru_kernel" in defined_all(exe)
    load_quarantine()
    assert C.quarantine_loaded()


def test_reference_cache_size_floor_on_production_engines():
    """-s N: the reference runs any line count (svmTrainMain.cpp:71, default 10).
    The production engines raise a count below the working-set cache's minimum
    (2 ws_size + 512 lines) to that minimum (the setup prints a note and records
    it as setup_info_["cache_note"]); engines=all keeps it for the pair cache
    engines; 0 (no cap) and counts above the minimum pass through."""
    lo = C.ws_cache_min_lines(192)
    assert lo == 2 * 192 + 512
    assert C.production_line_cap(10, 192) == lo
    assert C.production_line_cap(10, 48) == 2 * 48 + 512
    assert C.production_line_cap(lo - 1, 192) == lo
    assert C.production_line_cap(5000, 192) == 5000
    assert C.production_line_cap(0, 192) == 0
    assert C.production_line_cap(10, 192, engines=1) == 10
    with open(os.path.join(ROOT, "README.md")) as fh:
        assert "2 x ws_size + 512" in fh.read()  # the deviation list states the rule
