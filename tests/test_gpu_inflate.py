"""k_inflate (GZIP pages on the GPU, pq_inflate.hip) against the oracle's zlib
call, bit-exact, outcome for outcome:

* every case of tests/gzcases.py — zlib-built members (levels 0/1/6/9, the
  fixed / Huffman-only / RLE / filtered strategies, five data shapes) and
  hand-built ones (long codes past both root tables, a 1-bit distance code,
  an empty distance code, distances of 32768, stored / fixed / dynamic blocks
  in one member, header fields, trailing bytes, and the errors: header,
  block, code, symbol, distance, size and trailer checks), whose outcomes
  tests/test_gzip_cases.py pins on the CPU;
* the same pages inflated by zlib on the host (PQG_BATCH_HOST_INFLATE) give
  the same status and bytes;
* pyarrow-written GZIP files (V1 / V2 pages, dictionaries, strings, nulls,
  lists);
* seeded corruption (byte flips, truncation) of zlib members.
"""
import io

import numpy as np
import pytest

import gzcases
import oracle
import pqgpu
from test_gpu_parity import KEYS, _pq_bytes, check_file

pytestmark = pytest.mark.gpu
CASES = gzcases.cases()


def _decode(data, flags):
    r = pqgpu.FileReader(data)
    leaves = list(range(len(r.Columns())))
    b = r.batch(0, r.RowGroupCount(), leaves, flags)
    st = b.stats()
    b.decode()
    rc = b.sync(raise_on_error=False)
    out = [b.column(i) for i in leaves] if rc == 0 else None
    b.close()
    return rc, out, st


@pytest.mark.parametrize("name,expected,data", CASES, ids=[c[0] for c in CASES])
def test_inflate_case(name, expected, data):
    check_file(data, name)
    rc, out, st = _decode(data, 0)
    assert st["gzip_device_pages"] == st["pages"] > 0  # every page through k_inflate
    assert st["host_inflated_pages"] == 0
    rc_h, out_h, st_h = _decode(data, pqgpu.BATCH_HOST_INFLATE)
    assert st_h["gzip_device_pages"] == 0
    assert rc == rc_h, (name, rc, rc_h)
    assert rc == {"ok": 0, "codec": 5, "size": 8}[expected], (name, rc)
    if rc == 0:
        for a, h in zip(out, out_h):
            for k in KEYS:
                assert np.array_equal(a[k], h[k]), (name, k)


@pytest.mark.parametrize("version", ["1.0", "2.0"])
@pytest.mark.parametrize("level", [1, 9])
def test_inflate_pyarrow_files(version, level):
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(81 + level)
    n = 60000
    words = np.array(["w%05d" % i for i in rng.integers(0, 3000, 500)])
    ints = rng.integers(0, 1 << 40, n)
    t = pa.table({
        "i": pa.array(ints),
        "small": pa.array(rng.integers(0, 9, n).astype(np.int32)),
        "d": pa.array(rng.random(n), mask=rng.random(n) < 0.2),
        "s": pa.array(words[rng.integers(0, 500, n)], mask=rng.random(n) < 0.1),
        "l": pa.array([list(range(int(k))) for k in rng.integers(0, 4, n)], type=pa.list_(pa.int64())),
    })
    for dic in (True, False):
        data = _pq_bytes(t, compression="gzip", compression_level=level, data_page_version=version,
                         use_dictionary=dic, data_page_size=1 << 16, row_group_size=n // 2)
        check_file(data, "pyarrow gzip v%s level %d dict %s" % (version, level, dic))


def test_inflate_corrupted_members():
    """Seeded damage to zlib members: 1-3 byte flips anywhere in the member
    (header, blocks, trailer) or a cut at a random length.  The GPU reports
    the oracle's status and, when the page still inflates, its bytes."""
    rng = np.random.default_rng(83)
    sets = gzcases.data_sets(seed=84, n=1 << 13)
    names = sorted(sets)
    for trial in range(120):
        d = sets[names[trial % len(names)]]
        m = bytearray(gzcases.zgz(d, level=int(rng.integers(1, 10))))
        if trial % 4 == 3:
            m = m[: int(rng.integers(0, len(m)))]
        else:
            for _ in range(int(rng.integers(1, 4))):
                p = int(rng.integers(0, len(m)))
                m[p] ^= int(rng.integers(1, 256))
        data = gzcases.file_of([(d, bytes(m))])
        check_file(data, "corrupt member %d" % trial)
