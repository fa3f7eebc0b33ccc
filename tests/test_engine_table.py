"""The device solver's engine choice is one table (device_state.hpp kEngineTable,
evaluated by choose_engine() in gpu_setup.hip); docs/DESIGN.md §2 lists the same
rows.  CPU only: the table is host code."""
import os
import re

import pytest

C = pytest.importorskip("dpsvm_amd._C")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_engine_table_matches_design_doc():
    table = C.engine_table()
    names = [n for n, _ in table]
    assert names == ["ws-dense", "ws-cache", "persistent-dense", "fused-dense", "persistent-cache", "fused-cache",
                     "chain"]
    with open(os.path.join(ROOT, "docs", "DESIGN.md")) as fh:
        doc = fh.read()
    sec = doc[doc.index("**Engine choice**"):doc.index("## 2a.")]
    doc_rows = re.findall(r"^\| ([a-z-]+)(?: \(§[^)]*\))? \|", sec, flags=re.M)
    doc_rows = [r for r in doc_rows if r != "engine"]
    assert doc_rows == names, "DESIGN.md §2 engine table out of sync with kEngineTable"
    for _, use in table:
        assert use


@pytest.mark.parametrize("facts,want", [
    (dict(ws_dense=True, dense=True, persistent=True), "ws-dense"),
    (dict(ws_cache=True, cache_replicated=True, persistent=True), "ws-cache"),
    (dict(dense=True, persistent=True), "persistent-dense"),
    (dict(dense=True), "fused-dense"),
    (dict(cache_replicated=True, persistent=True), "persistent-cache"),
    (dict(cache_replicated=True), "fused-cache"),
    (dict(), "chain"),
    (dict(persistent=True), "chain"),
])
def test_choose_engine_first_match(facts, want):
    assert C.choose_engine(**facts) == want
