"""CPU tests: the oracle and the host-side parser of libpqgpu.so against the
reference's own test vectors (transcribed as data by
tests/golden/make_ref_vectors.py):

* Dremel level KATs, data_store_test.go:18-477 — 17 leaf columns of 9 tests,
  each with the asserted MaxDefinitionLevel / MaxRepetitionLevel, dense values
  and def / rep level arrays (34 `toArray()` assertions).  A file holding
  exactly those levels and values (tests/pqwrite.py) must decode to them.
* Fuzz-crash regressions (readAllData, schema_test.go:366-381): malformed
  files that must give an error, never a crash.  No test in the reference
  pins the error class, so the oracle's class is the expectation the GPU
  tests compare against (tests/test_gpu_parity.py).
"""
import json
import os

import numpy as np
import pytest

import oracle
import pqgpu
import pqwrite
from conftest import GOLDEN

KAT = json.load(open(os.path.join(GOLDEN, "kat_levels.json")))["tests"]
CRASH = json.load(open(os.path.join(GOLDEN, "crash", "index.json")))


def kat_file(name):
    t = KAT[name]
    return pqwrite.write(t["schema"], t["columns"])


def dense_values(out, max_def, max_rep):
    """The column store's dense values (values.assemble()) from the canonical
    layout: slots with validity set (every slot is a value for max_rep >= 2)."""
    v = out["values"].view("<i4")
    if max_rep >= 2:
        return v.tolist()
    bits = np.unpackbits(out["validity"], bitorder="little")[:v.size] if max_def > 0 else np.ones(v.size, np.uint8)
    return v[bits.astype(bool)].tolist()


def test_level_kats_transcribed():
    assert len(KAT) == 9
    assert sum(len(t["columns"]) for t in KAT.values()) == 17  # x2 toArray() assertions = 34


@pytest.mark.parametrize("name", sorted(KAT))
def test_level_kats_oracle(name):
    """Oracle: schema.go:789-823 levels, page_v1.go:27-55 level streams and
    values, dense values as the column store holds them (data_store.go:158-203)."""
    f = oracle.File(kat_file(name))
    leaves = f.leaves()
    assert sorted(L["name"] for L in leaves) == sorted(KAT[name]["columns"])
    for i, L in enumerate(leaves):
        want = KAT[name]["columns"][L["name"]]
        assert (L["max_def"], L["max_rep"]) == (want["max_def"], want["max_rep"]), (name, L["name"])
        out = f.decode(i)
        assert out["def"].tolist() == want["def"], (name, L["name"])
        assert out["rep"].tolist() == want["rep"], (name, L["name"])
        assert dense_values(out, L["max_def"], L["max_rep"]) == want["values"], (name, L["name"])


@pytest.mark.parametrize("name", sorted(KAT))
def test_level_kats_host_schema(name):
    """libpqgpu.so's footer and schema walk (host only, no GPU): the same
    MaxDefinitionLevel / MaxRepetitionLevel per leaf (Column, schema.go:70-93)."""
    r = pqgpu.FileReader(kat_file(name))
    got = {c["name"]: (c["max_def"], c["max_rep"]) for c in r.Columns()}
    want = {k: (c["max_def"], c["max_rep"]) for k, c in KAT[name]["columns"].items()}
    assert got == want
    assert r.NumRows() == sum(1 for x in next(iter(KAT[name]["columns"].values()))["rep"] if x == 0)


def oracle_outcome(data):
    """('open_error', code) or ('ok', [per (rg, leaf) status])."""
    try:
        f = oracle.File(data)
    except oracle.OracleError as e:
        return ("open_error", e.code)
    res = []
    for rg in range(f.num_row_groups):
        for leaf in range(len(f.leaves())):
            try:
                f.decode(leaf, rg, rg + 1)
                res.append(0)
            except oracle.OracleError as e:
                res.append(e.code)
    return ("ok", res)


@pytest.mark.parametrize("case", CRASH, ids=[c["test"] for c in CRASH])
def test_crash_inputs_oracle_and_host(case):
    """readAllData on the reference's fuzz-crash inputs: an error, not a crash.
    The oracle must come back with a status, and libpqgpu.so's host parser
    must agree on whether the footer opens (and with which class if not)."""
    data = open(os.path.join(GOLDEN, "crash", case["file"]), "rb").read()
    assert data[:4] == b"PAR1" and len(data) == case["bytes"]
    kind, res = oracle_outcome(data)
    try:
        r = pqgpu.FileReader(data)
        host = ("ok", r.RowGroupCount(), len(r.Columns()))
    except pqgpu.PqgError as e:
        host = ("open_error", e.code)
    if kind == "open_error":
        assert host == ("open_error", res), case["test"]
    else:
        f = oracle.File(data)
        assert host == ("ok", f.num_row_groups, len(f.leaves())), case["test"]
        assert any(s != 0 for s in res), case["test"]  # every transcribed input is malformed somewhere
