"""The k_inflate cases (tests/gzcases.py) against the oracle on the CPU: each
hand-built or zlib-built gzip page has the outcome the case names (the
oracle's zlib call, oracle/pqref.c:1107-1134: PQG_ERR_CODEC for
Z_DATA_ERROR, PQG_ERR_SIZE for Z_BUF_ERROR or a short result), and a valid
page decodes to its body.  This pins the cases before tests/test_gpu_inflate.py
runs them through k_inflate."""
import numpy as np
import pytest

import gzcases
import oracle

CODES = {"ok": 0, "codec": 5, "size": 8}
CASES = gzcases.cases()


@pytest.mark.parametrize("name,expected,data", CASES, ids=[c[0] for c in CASES])
def test_case_outcome(name, expected, data):
    o = oracle.File(data)
    try:
        got = o.decode(0, 0, 1)
        rc = 0
    except oracle.OracleError as e:
        rc = e.code
    assert rc == CODES[expected], (name, rc, expected)
    if rc == 0:
        assert got["values"].size % 8 == 0
