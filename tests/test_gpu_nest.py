"""Columns with max_rep >= 2 on the GPU (k_nest_count / k_nest_write,
pq_nest.hip; pqg_batch_column_nest): every level's offsets and validity and
the leaf slots' validity equal the restatement built from the oracle's
levels (tests/nestref.py, pinned against pyarrow by tests/test_nest_ref.py)
and pyarrow's own arrays — lists of lists with nulls and empty lists at
every level, 2 and 3 levels, required and optional outer lists, strings,
V1 / V2 pages, several row groups and pages, and a column long enough for
many scan blocks.  The rest of each column (values, levels) is checked by
check_file as before."""
import io

import numpy as np
import pytest

import nestref
import oracle
import pqgpu
from test_gpu_parity import check_file

pytestmark = pytest.mark.gpu


def _bytes(t, **kw):
    pq = pytest.importorskip("pyarrow.parquet")
    b = io.BytesIO()
    pq.write_table(t, b, **kw)
    return b.getvalue()


def _gpu_nest(data, flags):
    r = pqgpu.FileReader(data)
    b = r.batch(0, r.RowGroupCount(), [0], flags)
    b.decode()
    assert b.sync(raise_on_error=False) == 0, pqgpu.last_error()
    out = b.nest(0)
    b.decode()  # a second decode rebuilds the same structure
    assert b.sync(raise_on_error=False) == 0
    again = b.nest(0)
    b.close()
    for x, y in zip(out, again):
        for k in x:
            assert np.array_equal(np.asarray(x[k]), np.asarray(y[k])), ("second decode", k)
    return out


def _same(got, exp, ctx):
    assert len(got) == len(exp), ctx
    for k, (a, b) in enumerate(zip(got, exp)):
        assert a["count"] == b["count"], (ctx, k, a["count"], b["count"])
        assert np.array_equal(a["validity"], b["validity"]), (ctx, k, "validity")
        if "offsets" in b:
            assert np.array_equal(a["offsets"], b["offsets"]), (ctx, k, "offsets")
        else:
            assert np.asarray(a.get("offsets", np.empty(0))).size == 0, (ctx, k)


@pytest.mark.parametrize("ver,comp", [("1.0", "snappy"), ("2.0", "none"), ("1.0", "gzip")])
def test_nested_offsets(ver, comp):
    rng = np.random.default_rng(92)
    for name, t, depth, rdefs, max_def in nestref.nested_tables(rng):
        data = _bytes(t, data_page_version=ver, compression=comp, row_group_size=1000, data_page_size=4096)
        ctx = "%s v%s %s" % (name, ver, comp)
        check_file(data, ctx)
        o = oracle.File(data)
        lv = o.decode(0, 0, o.num_row_groups)
        exp = nestref.nest_from_levels(lv["def"], lv["rep"], rdefs, max_def)
        _same(nestref.nest_from_arrow(t.column(0).combine_chunks(), depth), exp, ctx + " (pyarrow)")
        for flags in (0, pqgpu.BATCH_LEVELS):
            _same(_gpu_nest(data, flags), exp, "%s flags %d" % (ctx, flags))


def test_nested_offsets_many_blocks():
    """~180 k level entries (about 45 scan blocks of 4,096) in one batch."""
    rng = np.random.default_rng(93)
    name, t, depth, rdefs, max_def = nestref.nested_tables(rng, rows=40000)[0]
    data = _bytes(t, compression="snappy", row_group_size=15000)
    o = oracle.File(data)
    lv = o.decode(0, 0, o.num_row_groups)
    assert len(lv["def"]) > 150000
    exp = nestref.nest_from_levels(lv["def"], lv["rep"], rdefs, max_def)
    _same(_gpu_nest(data, 0), exp, name + " many blocks")


def test_nest_arguments():
    """pqg_batch_column_nest rejects flat and max_rep == 1 columns and levels
    outside 1..max_rep + 1."""
    pa = pytest.importorskip("pyarrow")
    t = pa.table({"flat": pa.array([1, 2, 3]), "l1": pa.array([[1], [], None], type=pa.list_(pa.int64())),
                  "l2": pa.array([[[1]], [], None], type=pa.list_(pa.list_(pa.int64())))})
    r = pqgpu.FileReader(_bytes(t))
    b = r.batch(0, 1, [0, 1, 2], 0)
    b.decode()
    assert b.sync(raise_on_error=False) == 0
    for i in (0, 1):
        with pytest.raises(pqgpu.PqgError):
            b.nest(i)
    got = b.nest(2)
    assert [g["count"] for g in got] == [3, 1, 1]
    assert list(got[0]["offsets"]) == [0, 1, 1, 1] and list(got[1]["offsets"]) == [0, 1]
    b.close()
