"""The max_rep >= 2 list-structure restatement (tests/nestref.py) pinned on
the CPU: built from the oracle's decoded rep / def levels (oracle/pqref.c),
it equals pyarrow's own nested ListArray offsets and validity, level by
level, for lists of lists with nulls and empty lists at every level."""
import io

import numpy as np
import pytest

import nestref
import oracle


def _bytes(t, **kw):
    pq = pytest.importorskip("pyarrow.parquet")
    b = io.BytesIO()
    pq.write_table(t, b, **kw)
    return b.getvalue()


# (V2 pages under Snappy are avoided: pyarrow stores some small ones with
# is_compressed = false, which the reference decompresses anyway — D4 — and
# the oracle reports that error)
@pytest.mark.parametrize("ver,comp", [("1.0", "snappy"), ("2.0", "none"), ("1.0", "gzip")])
def test_restatement_matches_pyarrow(ver, comp):
    rng = np.random.default_rng(91)
    for name, t, depth, rdefs, max_def in nestref.nested_tables(rng):
        data = _bytes(t, data_page_version=ver, compression=comp, row_group_size=1000, data_page_size=4096)
        o = oracle.File(data)
        assert o.leaves()[0]["max_rep"] == depth and o.leaves()[0]["max_def"] == max_def, name
        got = o.decode(0, 0, o.num_row_groups)
        mine = nestref.nest_from_levels(got["def"], got["rep"], rdefs, max_def)
        ref = nestref.nest_from_arrow(t.column(0).combine_chunks(), depth)
        assert len(mine) == len(ref) == depth + 1
        for k, (a, b) in enumerate(zip(mine, ref)):
            assert a["count"] == b["count"], (name, k)
            assert np.array_equal(a["validity"], b["validity"]), (name, k)
            if "offsets" in b:
                assert np.array_equal(a["offsets"], b["offsets"]), (name, k)
