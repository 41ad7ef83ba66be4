"""GPU parity: libpqgpu.so (HIP kernels on cuda:0) against the CPU oracle and the
committed golden fixtures.  Bit-exact on every output buffer."""
import io
import json
import os

import numpy as np
import pytest

import oracle
import pqgpu
from conftest import GOLDEN, golden_bytes

pytestmark = pytest.mark.gpu

KEYS = ("values", "validity", "list_offsets", "list_validity", "str_offsets", "def", "rep")


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if pqgpu.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")


@pytest.fixture(params=["k_snappy", "k_snappy_wg"])
def snappy_kernel(request, monkeypatch):
    """Run a Snappy test with both decoders: the wave-per-page k_snappy (the
    default) and the workgroup-per-page k_snappy_wg (PQG_SNAPPY_WG=1, read by
    the library at every decode)."""
    if request.param == "k_snappy_wg":
        monkeypatch.setenv("PQG_SNAPPY_WG", "1")
    else:
        monkeypatch.delenv("PQG_SNAPPY_WG", raising=False)
    return request.param


def assert_same(gpu, ora, max_def, max_rep, ctx=""):
    for k in KEYS:
        if k == "validity" and max_def == 0:
            continue
        if k in ("list_offsets", "list_validity") and max_rep != 1:
            continue
        a, b = gpu[k], ora[k]
        if k in ("def", "rep") and a.size == 0:
            continue
        assert a.size == b.size, (ctx, k, a.size, b.size)
        if not np.array_equal(a, b):
            bad = np.nonzero(a != b)[0]
            raise AssertionError("%s %s: %d bytes differ, first at %d (gpu %d, oracle %d)"
                                 % (ctx, k, bad.size, bad[0], a[bad[0]], b[bad[0]]))
    for k in ("slots", "str_bytes"):
        assert gpu[k] == ora[k], (ctx, k)
    if max_rep == 1:
        assert gpu["rows"] == ora["rows"], ctx


def gpu_decode_all(data, levels=True, rg0=0, rg1=None, leaves=None):
    r = pqgpu.FileReader(data)
    rg1 = r.RowGroupCount() if rg1 is None else rg1
    leaves = list(range(len(r.Columns()))) if leaves is None else leaves
    b = r.batch(rg0, rg1, leaves, pqgpu.BATCH_LEVELS if levels else 0)
    # the first decode resumes from the batch's counting pass (strings /
    # lists), the second runs the whole pipeline again: both must agree
    b.decode()
    rc = b.sync(raise_on_error=False)
    out = {leaf: b.column(i) for i, leaf in enumerate(leaves)} if rc == 0 else None
    b.decode()
    rc2 = b.sync(raise_on_error=False)
    assert rc2 == rc, ("second decode", rc, rc2)
    if rc == 0:
        for i, leaf in enumerate(leaves):
            again = b.column(i)
            for k in KEYS:
                assert np.array_equal(again[k], out[leaf][k]), ("second decode differs", leaf, k)
    b.close()
    return rc, out, r.Columns()


def check_file(data, ctx, rg0=0, rg1=None):
    o = oracle.File(data)
    rg1 = o.num_row_groups if rg1 is None else rg1
    exp, first_err = {}, None
    for leaf, info in enumerate(o.leaves()):
        try:
            exp[leaf] = o.decode(leaf, rg0, rg1)
        except oracle.OracleError as e:
            # first error in (row group, leaf) order is what the batch must report
            key = (e.rg, leaf)
            if first_err is None or key < first_err[0]:
                first_err = (key, e.code)
    # with level output (k_decode<0> for every page) and without it (the
    # routes a reader takes: tiled pages, k_decode<1..3>, k_plain_str)
    for levels in (True, False):
        rc, got, cols = gpu_decode_all(data, levels, rg0, rg1)
        if first_err is not None:
            assert rc == first_err[1], (ctx, levels, rc, first_err)
            continue
        assert rc == 0, (ctx, levels, rc, pqgpu.last_error())
        for leaf, info in enumerate(o.leaves()):
            assert_same(got[leaf], exp[leaf], info["max_def"], info["max_rep"],
                        "%s leaf %d levels=%s" % (ctx, leaf, levels))


def fixture_names():
    return sorted(json.load(open(os.path.join(GOLDEN, "manifest.json"))))


@pytest.mark.parametrize("name", fixture_names())
def test_golden_fixture_parity(name, manifest):
    data = golden_bytes(name + ".parquet")
    check_file(data, name)
    # and against the committed pyarrow expectations
    e = manifest[name]
    cols = [c for c in e["columns"].values()]
    if any("error" in c for c in cols):
        rc, _, _ = gpu_decode_all(data)
        assert rc == [c["error"] for c in cols if "error" in c][0]
        return
    exp = np.load(os.path.join(GOLDEN, name + ".npz"))
    rc, got, info = gpu_decode_all(data, levels=False)
    assert rc == 0
    for key, c in e["columns"].items():
        g = got[c["leaf"]]
        for k in ("values", "validity", "list_offsets", "list_validity", "str_offsets"):
            ek = "%s_%s" % (key, k)
            if ek not in exp or (k == "validity" and info[c["leaf"]]["max_def"] == 0):
                continue
            assert np.array_equal(g[k], exp[ek].view(np.uint8).ravel()), (name, key, k)


def test_stats_get_old_caller_size():
    """ABI 2: a caller whose pqg_batch_stats is the version-1 struct (eleven
    int64 counters, 88 bytes) passes that size and gets exactly those bytes —
    the same counters as a full-size call — and nothing past them is written;
    a size short of the prefix is PQG_ERR_ARG."""
    import ctypes
    data = golden_bytes("c4_list_str.parquet")
    r = pqgpu.FileReader(data)
    b = r.batch(0, r.RowGroupCount(), list(range(len(r.Columns()))), 0)
    try:
        full = b.stats()
        L = pqgpu.lib()
        buf = (ctypes.c_uint8 * 160)(*([0xAB] * 160))
        assert L.pqg_batch_stats_get(b._h, ctypes.cast(buf, ctypes.POINTER(pqgpu.BatchStats)), 88) == 0
        got = np.frombuffer(bytes(buf), np.int64, 11)
        names = [f for f, _ in pqgpu.BatchStats._fields_][:11]
        assert list(got) == [full[k] for k in names]
        assert bytes(buf)[88:] == b"\xab" * 72
        assert L.pqg_batch_stats_get(b._h, ctypes.cast(buf, ctypes.POINTER(pqgpu.BatchStats)), 80) == pqgpu.ERR_ARG
    finally:
        b.close()


def test_row_group_subsets():
    data = golden_bytes("c4_list_str.parquet")
    check_file(data, "c4 rg1", 1, 2)
    check_file(data, "c4 rg1-3", 1, 3)
    data = golden_bytes("c1_int64_plain.parquet")
    check_file(data, "c1 rg2", 2, 3)


def test_snappy_block_roundtrip(snappy_kernel):
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(5)
    for n in (0, 1, 5, 64, 65, 4095, 8192, 8193, 70000, 300000):
        for kind in ("rand", "rep", "mixed"):
            if kind == "rand":
                data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            elif kind == "rep":
                data = (b"0123456789abcdefXYZ" * (n // 19 + 1))[:n]
            else:
                data = np.round(rng.standard_normal(n // 8 + 1), 2).tobytes()[:n]
            comp = pa.compress(data, codec="snappy", asbytes=True)
            assert pqgpu.DecompressBlock(pqgpu.CompressionCodec_SNAPPY, comp, n) == data, (n, kind)
    # a literal long enough to be deferred to k_copy, then far copies that reach back
    # into it (offset > the 8 KB LDS history), hand-assembled: google snappy never
    # emits offsets beyond its 64 KB block, other encoders may
    lit = rng.integers(0, 256, 70000, dtype=np.uint8).tobytes()
    stream = bytearray()
    total = 70000 + 40 + 64 + 5
    v = total
    while True:
        b = v & 0x7f
        v >>= 7
        stream.append(b | (0x80 if v else 0))
        if not v:
            break
    stream += bytes([62 << 2]) + (70000 - 1).to_bytes(3, "little") + lit
    stream += bytes([((40 - 1) << 2) | 3]) + (68000).to_bytes(4, "little")   # copy4 into the literal
    stream += bytes([((64 - 1) << 2) | 3]) + (9000).to_bytes(4, "little")    # far copy
    stream += bytes([((5 - 1) << 2) | 2]) + (3).to_bytes(2, "little")         # overlapping near copy
    want = bytearray(lit)
    for off, ln in ((68000, 40), (9000, 64), (3, 5)):
        for _ in range(ln):
            want.append(want[len(want) - off])
    assert len(want) == total
    rc_o, got_o, _ = oracle.snappy_decode(bytes(stream), total)
    assert rc_o == 0 and got_o == bytes(want)
    assert pqgpu.DecompressBlock(pqgpu.CompressionCodec_SNAPPY, bytes(stream), total) == bytes(want)
    # far back-references (offset > the 8 KB LDS history): repeat a random 20 KB block
    blk = rng.integers(0, 256, 20000, dtype=np.uint8).tobytes()
    data = blk * 3
    comp = pa.compress(data, codec="snappy", asbytes=True)
    assert pqgpu.DecompressBlock(pqgpu.CompressionCodec_SNAPPY, comp, len(data)) == data


def _uvarint(v):
    out = bytearray()
    while True:
        b = v & 0x7f
        v >>= 7
        out.append(b | (0x80 if v else 0))
        if not v:
            return bytes(out)


def test_snappy_segments_and_fallback(snappy_kernel):
    """Blocks longer than 64 KiB are decoded by one wave per 64 KiB segment
    (k_snappy_walk finds the token at each boundary); streams without that
    structure fall back to the serial decode.  Every case against the oracle."""
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(9)

    def both(stream, n, expect_n=None):
        expect_n = n if expect_n is None else expect_n
        rc_o, got_o, n_o = oracle.snappy_decode(stream, max(n, expect_n) + 64)
        want = rc_o if rc_o else (pqgpu.ERR_SIZE if n_o != expect_n else 0)
        try:
            got = pqgpu.DecompressBlock(pqgpu.CompressionCodec_SNAPPY, stream, expect_n)
            rc_g = 0
        except pqgpu.PqgError as e:
            rc_g, got = e.code, None
        assert rc_g == want, (rc_g, want)
        if want == 0:
            assert got == got_o[:expect_n]
    # google snappy output (64 KiB blocks): segments
    for n in (65536, 65537, 200000, 1 << 20, (1 << 20) + 12345):
        data = (np.round(rng.standard_normal(n // 8 + 1), 2).tobytes() + b"x" * 7)[:n]
        both(pa.compress(data, codec="snappy", asbytes=True), n)
        if n >= 200000:
            # bytes or a token after the decoded length end the stream corrupt
            # (decode_other.go:16-99), segmented or not
            s = pa.compress(data, codec="snappy", asbytes=True)
            both(s + b"\x00", n)
            both(s + bytes([0x01, 0x05]), n)
            both(s + bytes([0x00, 0x41]), n)
    # a copy that reaches back across the 64 KiB boundary (a token starts there): fallback
    lit = rng.integers(0, 256, 65536, dtype=np.uint8).tobytes()
    stream = _uvarint(65536 + 64) + bytes([62 << 2]) + (65536 - 1).to_bytes(3, "little") + lit
    stream += bytes([((64 - 1) << 2) | 2]) + (60000).to_bytes(2, "little")
    both(stream, 65536 + 64)
    # a token crossing the boundary: fallback
    stream = _uvarint(65600) + bytes([62 << 2]) + (65530 - 1).to_bytes(3, "little") + lit[:65530]
    stream += bytes([60 << 2, 70 - 1]) + lit[:70]
    both(stream, 65600)
    # corrupt inside the second segment (offset 0), and a size mismatch
    good = pa.compress(lit + lit[:40000], codec="snappy", asbytes=True)
    bad = bytearray(good)
    bad[-3:] = bytes([0x01, 0x00, 0x00])
    both(bytes(bad), len(lit) + 40000)
    both(good, len(lit) + 40000, expect_n=len(lit) + 39999)


def test_snappy_block_errors_match_oracle(snappy_kernel):
    """DecompressBlock = snappy.Decode + the exact-size check of newBlockReader
    (compress.go:112-119): class SNAPPY if the stream is corrupt, else SIZE if
    the decoded length differs from the page header's."""
    cases = [bytes([4, 0b01, 0]), bytes([4, 0x0c, 1, 2, 3]), bytes([5, 0x0c, 1, 2, 3]), b"", bytes([0x80]),
             bytes([3, 0x08, 1, 2, 3]), bytes([2, 0x04, 7, 8, 0x01, 1]), bytes([6, 0x04, 7, 8, 0x05, 1]),
             bytes([8, 0x04, 7, 8, 0x0a, 2, 0]), bytes([0xff] * 11)]
    for c in cases:
        for expect in (8, 6, 4, 3, 2):
            rc_o, _, n = oracle.snappy_decode(c, 64)
            want = rc_o if rc_o else (pqgpu.ERR_SIZE if n != expect else 0)
            try:
                pqgpu.DecompressBlock(pqgpu.CompressionCodec_SNAPPY, c, expect)
                rc_g = 0
            except pqgpu.PqgError as e:
                rc_g = e.code
            assert rc_g == want, (c, expect, rc_g, want)


def _pq_bytes(table, **kw):
    pq = pytest.importorskip("pyarrow.parquet")
    buf = io.BytesIO()
    pq.write_table(table, buf, **kw)
    return buf.getvalue()


@pytest.mark.parametrize("bw", [3, 7, 13, 17, 20])
def test_generated_dictionary_widths(bw):
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(bw)
    K = 1 << bw
    rows = max(3 * K // 2, 50000) if bw <= 17 else 700000
    dvals = rng.permutation(K).astype(np.int32) * 3 - 7
    t = pa.table({"v": pa.array(dvals[rng.integers(0, K, rows)])},
                 schema=pa.schema([pa.field("v", pa.int32(), nullable=False)]))
    check_file(_pq_bytes(t, compression="snappy", dictionary_pagesize_limit=1 << 30, row_group_size=1 << 18),
               "dict bw%d" % bw)


@pytest.mark.parametrize("bw", [13, 14, 15])
def test_tiled_big_dictionary_groups(bw):
    """Wide dictionaries (2^13..2^15 entries): k_expand_wg, a CU's workgroup
    holding the dictionary in LDS (PQG_BIG=1), INT32 and INT64 columns side
    by side, against the oracle; and the mixed launch's L1/L2 path
    (PQG_NO_BIG=1)."""
    rng = np.random.default_rng(200 + bw)
    K = 1 << bw
    rows = 600000
    d32 = rng.permutation(K).astype(np.int32) * 5 - 11
    d64 = rng.permutation(K >> 1).astype(np.int64) * 0x1234567 - (1 << 35)
    t = _req_table({"a": d32[rng.integers(0, K, rows)], "b": d64[rng.integers(0, K >> 1, rows)]})
    data = _pq_bytes(t, compression="snappy", dictionary_pagesize_limit=1 << 30, row_group_size=300000)
    for env in ("PQG_BIG", "PQG_NO_BIG"):
        os.environ[env] = "1"
        try:
            check_file(data, "big dict bw%d %s" % (bw, env))
        finally:
            del os.environ[env]


@pytest.mark.parametrize("bw", [13, 16])
@pytest.mark.parametrize("comp", ["none", "snappy"])
def test_tiled_wg_dictionary_layouts(bw, comp):
    """k_expand_wg: a dictionary resident in a CU's LDS (bit width 13) and one
    streamed through it in slices (16: two slices), INT32 and INT64 columns;
    uncompressed dictionaries sit 16-byte aligned (copied by LDS-DMA), Snappy
    single-literal ones are read in place at any alignment (register copy
    with a funnel shift); every page's last rows take the general key path."""
    rng = np.random.default_rng(300 + bw)
    K = 1 << bw
    rows = 3 * K + 777
    d32 = rng.permutation(K).astype(np.int32) * 7 - 3
    d64 = rng.permutation(K >> 2).astype(np.int64) * 0x10001 - (1 << 40)
    t = _req_table({"a": d32[rng.integers(0, K, rows)], "b": d64[rng.integers(0, K >> 2, rows)]})
    data = _pq_bytes(t, compression=comp, dictionary_pagesize_limit=1 << 30, row_group_size=rows // 2 + 5)
    os.environ["PQG_BIG"] = "1"
    try:
        check_file(data, "wg bw%d %s" % (bw, comp))
    finally:
        del os.environ["PQG_BIG"]


def test_segment_times_route():
    """PQG_SEGMENT_TIMES=1 (bench.py's phase timing) launches k_copy, the
    string walks, k_dict_prepare and k_prepare one by one instead of fused:
    the same outputs on every config shape."""
    os.environ["PQG_SEGMENT_TIMES"] = "1"
    try:
        for name in ("c1_int64_plain", "c2_dict_bw8", "c2_dict_bw12", "c3_delta_v2", "c4_list_str", "plain_strings",
                     "gzip_int64"):
            check_file(golden_bytes(name + ".parquet"), name + " segment times")
    finally:
        del os.environ["PQG_SEGMENT_TIMES"]


def test_generated_nullable_mix():
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(11)
    n = 120000
    ts = (1_600_000_000_000_000 + np.cumsum(np.where(rng.random(n) < 0.95, 1000, rng.integers(0, 4096, n)))).astype(np.int64)
    t = pa.table({
        "ts": pa.array(ts),
        "x": pa.array(np.round(rng.standard_normal(n), 2), mask=rng.random(n) < 0.1),
        "i": pa.array(rng.integers(-5, 5, n).astype(np.int32), mask=rng.random(n) < 0.5),
        "s": pa.array(["k%d" % v if v % 7 else None for v in rng.integers(0, 500, n)]),
    })
    for ver in ("1.0", "2.0"):
        check_file(_pq_bytes(t, compression="snappy", data_page_version=ver, use_dictionary=["s", "i"],
                             column_encoding={"ts": "DELTA_BINARY_PACKED", "x": "PLAIN"}, row_group_size=50000),
                   "mix v" + ver)


def test_flat_level_bitmaps():
    """Flat pages without level output keep their definition levels as a
    bitmap (def == max_def) written in order by k_levels (BitOut): null
    densities from none to all (RLE-only streams, long bit-packed runs on the
    serial path, short mixed runs through the run tables, bit width 1 and
    the per-value path of an optional field inside an optional struct,
    max_def 2), V1 and V2, against the oracle — with and without level
    output (check_file), and with the byte scratch (PQG_LEVEL_BYTES=1)."""
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(13)
    n = 90000
    cols = {}
    for name, frac in (("none", 0.0), ("all", 1.0), ("rare", 0.001), ("half", 0.5), ("dense", 0.97)):
        cols[name] = pa.array(rng.integers(-9, 9, n).astype(np.int64), mask=rng.random(n) < frac)
    # runs: blocks of nulls and values of random lengths (long RLE and bit-packed runs)
    blk = np.repeat(rng.random(n // 300) < 0.5, 300)[:n]
    cols["blocks"] = pa.array(rng.standard_normal(n), mask=np.pad(blk, (0, n - len(blk))))
    inner = pa.array(rng.integers(0, 100, n).astype(np.int32), mask=rng.random(n) < 0.2)
    cols["st"] = pa.StructArray.from_arrays([inner], names=["v"], mask=pa.array(rng.random(n) < 0.1))
    t = pa.table(cols)
    for ver in ("1.0", "2.0"):
        data = _pq_bytes(t, compression="snappy", data_page_version=ver, use_dictionary=False, row_group_size=40000)
        check_file(data, "level bitmaps v" + ver)
        os.environ["PQG_LEVEL_BYTES"] = "1"
        try:
            check_file(data, "level bytes v" + ver)
        finally:
            del os.environ["PQG_LEVEL_BYTES"]


def test_generated_lists():
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(12)
    n = 60000
    lists = [None if rng.random() < 0.05 else [None if rng.random() < 0.05 else int(v)
                                                for v in rng.integers(0, 100, rng.poisson(4))] for _ in range(n)]
    strs = [None if rng.random() < 0.1 else ["w%d" % v for v in rng.integers(0, 50, rng.poisson(2))] for _ in range(n)]
    t = pa.table({"l": pa.array(lists, pa.list_(pa.int32())), "ls": pa.array(strs, pa.list_(pa.string()))})
    check_file(_pq_bytes(t, compression="snappy", row_group_size=25000), "lists v1")
    check_file(_pq_bytes(t, compression="snappy", row_group_size=25000, data_page_version="2.0"), "lists v2")


@pytest.mark.parametrize("part", ["256", "768", "0"])
def test_list_page_parts(part):
    """k_decode<3> over parts of list pages (PQG_NEST_PART level entries a
    wave; 0 = a wave per page): each part counts the rows / slots / values
    before it from k_levels' bytes and seeks the key stream (HybS::skip,
    trains of identical bit-packed headers 64 runs a step).  Dictionary and
    PLAIN values, nulls at both levels, V1 and V2, bit-exact against the
    oracle; then seeded corruptions of uncompressed list pages, where a part
    after the first that fails leaves the page to the whole-page redo launch:
    the GPU reports the oracle's first error."""
    pa = pytest.importorskip("pyarrow")
    pq = pytest.importorskip("pyarrow.parquet")
    rng = np.random.default_rng(60)
    n = 30000
    lists = [None if rng.random() < 0.05 else [None if rng.random() < 0.05 else int(v)
                                                for v in rng.integers(-3000, 3000, rng.poisson(4))] for _ in range(n)]
    l64 = [None if x is None else [None if v is None else v * 977 for v in x] for x in lists]
    t = pa.table({"d": pa.array(lists, pa.list_(pa.int32())), "p": pa.array(l64, pa.list_(pa.int64()))})
    os.environ["PQG_NEST_PART"] = part
    try:
        for ver in ("1.0", "2.0"):
            check_file(_pq_bytes(t, compression="snappy", row_group_size=15000, data_page_version=ver,
                                 use_dictionary=["d"]), "list parts %s v%s" % (part, ver))
        base = _pq_bytes(t.select(["d"]), compression="none", row_group_size=n, data_page_size=16 << 10)
        cc = pq.ParquetFile(io.BytesIO(base)).metadata.row_group(0).column(0)
        lo, hi = cc.data_page_offset, cc.dictionary_page_offset + cc.total_compressed_size
        outcomes = set()
        for trial in range(16):
            data = bytearray(base)
            for _ in range(int(rng.integers(1, 3))):
                p = int(rng.integers(lo + 32, hi))
                data[p] ^= int(rng.integers(1, 256))
            check_file(bytes(data), "list parts %s corrupt %d" % (part, trial))
            try:
                oracle.File(bytes(data)).decode(0)
                outcomes.add(0)
            except oracle.OracleError as e:
                outcomes.add(e.code)
        assert len(outcomes) >= 2, outcomes
    finally:
        del os.environ["PQG_NEST_PART"]


@pytest.mark.parametrize("part", ["256", ""])
def test_list_parts_beside_unsplit_pages(part):
    """A batch where one list column's pages are split into k_decode<5> parts
    and another list column's pages stay whole because the planner does not
    split them: DELTA_BINARY_PACKED list<int64> / list<int32> values
    (deltabp_decoder.go), which <5> has no path for.  Those pages ride in the
    part list unsplit, are handed to the whole-page redo launch
    (k_decode<3>) and decode bit-exact against the oracle, V1 and V2, with and
    without nulls; a corrupted DELTA list page reports the oracle's error."""
    pa = pytest.importorskip("pyarrow")
    pq = pytest.importorskip("pyarrow.parquet")
    rng = np.random.default_rng(61)
    n = 40000
    lists = [None if rng.random() < 0.05 else [None if rng.random() < 0.05 else int(v)
                                                for v in rng.integers(-3000, 3000, rng.poisson(4))] for _ in range(n)]
    z64 = [None if x is None else [None if v is None else v * 1000003 + 7 for v in x] for x in lists]
    z32 = [None if x is None else [None if v is None else v * 13 for v in x] for x in lists]
    t = pa.table({"d": pa.array(lists, pa.list_(pa.int32())), "z": pa.array(z64, pa.list_(pa.int64())),
                  "y": pa.array(z32, pa.list_(pa.int32()))})
    if part:
        os.environ["PQG_NEST_PART"] = part
    try:
        for ver in ("1.0", "2.0"):
            check_file(_pq_bytes(t, compression="snappy", row_group_size=20000, data_page_version=ver,
                                 use_dictionary=["d"], column_encoding={"z": "DELTA_BINARY_PACKED",
                                                                        "y": "DELTA_BINARY_PACKED"}),
                       "delta lists beside parts %s v%s" % (part, ver))
        base = _pq_bytes(t, compression="none", row_group_size=n, use_dictionary=["d"], data_page_size=16 << 10,
                         column_encoding={"z": "DELTA_BINARY_PACKED", "y": "DELTA_BINARY_PACKED"})
        cc = pq.ParquetFile(io.BytesIO(base)).metadata.row_group(0).column(1)
        lo, hi = cc.data_page_offset, cc.data_page_offset + cc.total_compressed_size
        for trial in range(6):
            data = bytearray(base)
            p = int(rng.integers(lo + 32, hi))
            data[p] ^= int(rng.integers(1, 256))
            check_file(bytes(data), "delta lists beside parts %s corrupt %d" % (part, trial))
    finally:
        os.environ.pop("PQG_NEST_PART", None)


def _req_table(cols):
    pa = pytest.importorskip("pyarrow")
    return pa.table({k: pa.array(v) for k, v in cols.items()},
                    schema=pa.schema([pa.field(k, pa.array(v).type, nullable=False) for k, v in cols.items()]))


@pytest.mark.parametrize("bw", [1, 4, 12, 15])
def test_tiled_int64_dictionary(bw):
    """k_expand_mix<8>: required INT64 dictionary columns (LDS groups for the
    small dictionaries, L1/L2 blocks for the large), beside an INT32 one."""
    rng = np.random.default_rng(100 + bw)
    K = 1 << bw
    rows = max(2 * K, 60000)
    d64 = rng.permutation(K).astype(np.int64) * 0x12345679 - (1 << 40)
    d32 = rng.permutation(K).astype(np.int32) - 3
    t = _req_table({"a": d64[rng.integers(0, K, rows)], "b": d32[rng.integers(0, K, rows)]})
    check_file(_pq_bytes(t, compression="snappy", dictionary_pagesize_limit=1 << 30, row_group_size=1 << 16),
               "int64 dict bw%d" % bw)


def test_tiled_dictionary_fallback_to_plain():
    """A chunk whose dictionary overflows mid-way: RLE_DICTIONARY pages, then
    PLAIN pages with the same dictionary page in the chunk (LDS groups run both)."""
    rng = np.random.default_rng(21)
    rows = 400000
    t = _req_table({"v": rng.integers(-(1 << 31), 1 << 31, rows, dtype=np.int64).astype(np.int32),
                    "w": rng.integers(0, 1 << 40, rows, dtype=np.int64)})
    check_file(_pq_bytes(t, compression="snappy", dictionary_pagesize_limit=64 << 10, row_group_size=1 << 18),
               "dict fallback")


def test_tiled_dictionary_fallback_to_plain_strings():
    """BYTE_ARRAY chunks whose dictionary overflows mid-way (chunk_reader.go:206-283,
    type_bytearray.go:13-55): RLE_DICTIONARY string pages, then PLAIN string pages,
    flat required / nullable and beside a fixed-width fallback column."""
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(24)
    rows = 120000
    words = ["%08x-%s" % (v, "q" * int(v % 23)) for v in rng.integers(0, 1 << 32, rows)]
    t = pa.table({"s": pa.array(words), "n": pa.array(words, mask=rng.random(rows) < 0.2),
                  "i": pa.array(rng.integers(-(1 << 40), 1 << 40, rows))})
    for ver in ("1.0", "2.0"):
        check_file(_pq_bytes(t, compression="snappy", dictionary_pagesize_limit=48 << 10, row_group_size=50000,
                             data_page_version=ver), "string dict fallback v" + ver)


@pytest.mark.parametrize("maxlen", [16, 40, 300])
def test_nullable_dictionary_strings_staged(maxlen):
    """Nullable RLE_DICTIONARY BYTE_ARRAY pages on k_decode<2> (type_bytearray.go:
    57-80 dictionary lookups; chunk_reader.go:206-283): a step's strings go
    through the wave's LDS stage when its bytes fit (empty strings, <= 16-byte
    strings from six dwords, longer ones a dword at a time) and the per-string
    copies when they do not (maxlen 300: ~38 KB steps); nulls every density."""
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(31 + maxlen)
    rows = 60000
    lens = rng.integers(0, maxlen + 1, 700)
    vocab = ["".join(chr(97 + int(c)) for c in rng.integers(0, 26, n)) for n in lens]
    idx = rng.integers(0, len(vocab), rows)
    words = [vocab[i] for i in idx]
    t = pa.table({"a": pa.array(words, mask=rng.random(rows) < 0.3),
                  "b": pa.array(words, mask=rng.random(rows) < 0.97)})
    for ver in ("1.0", "2.0"):
        check_file(_pq_bytes(t, compression="snappy", row_group_size=25000, data_page_version=ver),
                   "nullable dict strings maxlen %d v%s" % (maxlen, ver))


@pytest.mark.parametrize("maxlen", [12, 200])
def test_string_page_parts(maxlen):
    """Flat nullable dictionary-string pages of >= 8,192 entries run as
    k_decode<2> parts of ~4,096 entries on the column's 256-slot grid: each
    part counts the values before it from k_levels' bitmap, takes their string
    bytes from k_prepare's per-256-value prefix table and seeks the key stream
    (HybS::skip).  Row groups of 23,457 rows put every page's first slot off
    the grid; stretches with no nulls, with every entry null, and mixed put
    part starts on null and non-null entries; V1 and V2, Snappy and not.
    Every buffer bit-exact against the oracle (offsets, bytes, validity)."""
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(71 + maxlen)
    rows = 70001
    lens = rng.integers(0, maxlen + 1, 900)
    vocab = ["".join(chr(97 + int(c)) for c in rng.integers(0, 26, n)) for n in lens]
    words = [vocab[i] for i in rng.integers(0, len(vocab), rows)]
    mask = rng.random(rows) < 0.2
    mask[9000:15000] = True    # every entry null
    mask[30000:41000] = False  # no nulls
    mask[50000:50300] = True
    t = pa.table({"s": pa.array(words, mask=mask), "r": pa.array(words, mask=rng.random(rows) < 0.01)})
    for ver in ("1.0", "2.0"):
        for comp in ("snappy", "none"):
            check_file(_pq_bytes(t, compression=comp, row_group_size=23457, data_page_version=ver),
                       "string parts maxlen %d v%s %s" % (maxlen, ver, comp))


def _c5_bytes(tmp_path, rows, rg_rows, **kw):
    import synth
    path = str(tmp_path / "c5_small.parquet")
    synth.make("c5", path, rows, rg_rows, **kw)
    return open(path, "rb").read()


def test_c5_lineitem_shape(tmp_path, snappy_kernel):
    """Config C5's file shape at small scale (tools/synth.py c5: 16 leaves, 4 INT64 /
    4 DOUBLE / 4 INT32 / 4 dictionary STRING): small dictionary pages make
    l_comment (and the high-cardinality numeric columns) fall back from
    RLE_DICTIONARY to PLAIN mid-chunk; every leaf bit-exact against the oracle."""
    pytest.importorskip("pyarrow")
    data = _c5_bytes(tmp_path, 90000, 30000, dictionary_pagesize_limit=64 << 10, data_page_size=256 << 10)
    check_file(data, "c5 small dict")
    # every Snappy page over 64 KiB in segments (k_snappy_walk + one wave per
    # segment), and none (one wave per page)
    for env, val in (("PQG_SNAPPY_SEG_MIN", "65537"), ("PQG_SNAPPY_SEGMENTS", "0")):
        os.environ[env] = val
        try:
            check_file(data, "c5 small dict %s=%s" % (env, val))
        finally:
            del os.environ[env]


def test_c5_lineitem_large_string_dictionary(tmp_path):
    """C5 with the writer's default 1 MiB dictionary limit: l_comment's
    dictionary page holds ~30k strings (k_dict_prepare on a large string
    dictionary) before the PLAIN fallback; 16 leaves side by side."""
    pytest.importorskip("pyarrow")
    data = _c5_bytes(tmp_path, 80000, 40000)
    check_file(data, "c5 default dict")
    # the ~1 MiB string dictionary pages themselves cut into Snappy segments:
    # k_dict_prepare must follow the segment chain (an early, side-stream
    # k_dict_prepare read them undecoded: an illegal access on the full C5)
    os.environ["PQG_SNAPPY_SEG_MIN"] = "65537"
    try:
        check_file(data, "c5 default dict, segmented dictionary pages")
    finally:
        del os.environ["PQG_SNAPPY_SEG_MIN"]


def _walked_dict_column_bytes(compression):
    """A required string column whose first 30,000 rows (a 100-word vocabulary)
    are RLE_DICTIONARY pages (bit width 7) of 20,000 / 10,000 values; 16
    5,000-byte strings then overflow the 64 KiB dictionary limit (116 entries:
    keys 116-127 are out of range), and 40-byte strings after them are PLAIN
    pages of 20,000 values (880 KB: region-parallel length walk); beside a
    required INT64 column."""
    rng = np.random.default_rng(43)
    letters = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz", np.uint8)
    word = lambda n: bytes(letters[rng.integers(0, 26, n)]).decode()
    vocab = [word(12) for _ in range(100)]
    rows = 90000
    w = [vocab[i] for i in rng.integers(0, 100, 30000)] + [word(5000) for _ in range(16)]
    w += [word(40) for _ in range(rows - len(w))]
    t = _req_table({"x": rng.integers(-2**40, 2**40, rows, dtype=np.int64), "w": w})
    return _pq_bytes(t, compression=compression, row_group_size=rows, dictionary_pagesize_limit=64 << 10,
                     data_page_size=1 << 20, write_batch_size=16)


def test_walked_column_dictionary_parts_corrupted():
    """Walk split (pq_host.cpp: a column with region-parallel-walked PLAIN
    pages is scanned and decoded after the walk, on side streams 0 / 2): that
    column's dictionary pages go to k_decode<4> in parts of ~2,048 values.
    Snappy and uncompressed, then seeded corruptions of the first dictionary
    page's key stream past its first part — a later part's error sends the
    page to the whole-page redo launch — against the oracle's outcome
    (type_dict.go:44-53, hybrid_decoder.go:82-166)."""
    pq = pytest.importorskip("pyarrow.parquet")
    check_file(_walked_dict_column_bytes("snappy"), "walked dict column, snappy")
    base = _walked_dict_column_bytes("none")
    check_file(base, "walked dict column")
    cc = pq.ParquetFile(io.BytesIO(base)).metadata.row_group(0).column(1)
    lo = cc.dictionary_page_offset if cc.has_dictionary_page else cc.data_page_offset
    assert cc.data_page_offset > lo  # (the dictionary page, then the key streams)
    rng = np.random.default_rng(41)
    outcomes = set()
    for trial in range(10):
        data = bytearray(base)
        for _ in range(2):
            p = cc.data_page_offset + int(rng.integers(4000, 16000))
            data[p] = 0xff if trial % 2 == 0 else data[p] ^ int(rng.integers(1, 256))  # 0xff: a key of 127
        check_file(bytes(data), "corrupt %d" % trial)
        try:
            oracle.File(bytes(data)).decode(1)
            outcomes.add(0)
        except oracle.OracleError as e:
            outcomes.add(e.code)
    assert len(outcomes - {0}) >= 1, outcomes  # some corruption is an error the redo launch reports


@pytest.mark.parametrize("per,depth,ramp", [(1, 2, False), (2, 1, False), (3, 3, False), (4, 3, True)])
def test_stream_slices_match_oracle(tmp_path, per, depth, ramp):
    """pqg_stream: row-group slices planned and uploaded by the host worker
    while the previous slice decodes; every slice bit-exact against the oracle's
    decode of the same row-group range (C5 shape: 16 leaves, strings, fallback
    to PLAIN; C4 golden: lists and nullable strings); with STREAM_RAMP the
    first two slices hold a quarter and a half of `per` row groups."""
    pytest.importorskip("pyarrow")
    for data, ctx in ((_c5_bytes(tmp_path, 70000, 10000, dictionary_pagesize_limit=64 << 10), "c5"),
                      (golden_bytes("c4_list_str.parquet"), "c4")):
        o = oracle.File(data)
        r = pqgpu.FileReader(data)
        leaves = list(range(len(r.Columns())))
        seen = []
        starts, rg = [], 0
        while rg < o.num_row_groups:
            starts.append(rg)
            k = len(starts) - 1
            rg += per if not ramp or k >= 2 else max(1, per // (4 if k == 0 else 2))
        with r.stream(0, None, per, leaves, depth, pqgpu.STREAM_RAMP if ramp else 0) as st:
            for b in st:
                rc = b.sync(raise_on_error=False)
                assert rc == 0, (ctx, b.rg0, pqgpu.last_error())
                rg1 = b.rg1
                k = starts.index(b.rg0)
                assert rg1 == (starts[k + 1] if k + 1 < len(starts) else o.num_row_groups), (ctx, b.rg0, rg1)
                for i, leaf in enumerate(leaves):
                    info = o.leaves()[leaf]
                    assert_same(b.column(i), o.decode(leaf, b.rg0, rg1), info["max_def"], info["max_rep"],
                                "%s stream slice %d leaf %d" % (ctx, b.rg0, leaf))
                seen.append(b.rg0)
        assert seen == starts, (ctx, seen)


@pytest.mark.parametrize("maxlen", [0, 3, 20, 60, 300])
def test_plain_required_strings_items(maxlen):
    """k_plain_str: flat required PLAIN BYTE_ARRAY pages of many items (several
    waves per page), short strings (steps staged in LDS and copied by output
    dword) and long ones (per-value copies), empty strings, against the oracle."""
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(300 + maxlen)
    rows = 30000
    lens = rng.integers(0, maxlen + 1, rows)
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789", np.uint8)
    offs = np.zeros(rows + 1, np.int32)
    offs[1:] = np.cumsum(lens)
    data = alpha[rng.integers(0, len(alpha), int(offs[-1]))]
    arr = pa.StringArray.from_buffers(rows, pa.py_buffer(offs.tobytes()), pa.py_buffer(data.tobytes()))
    t = pa.table({"s": arr}, schema=pa.schema([pa.field("s", pa.string(), nullable=False)]))
    for comp in ("snappy", "none"):
        check_file(_pq_bytes(t, compression=comp, use_dictionary=False, row_group_size=12000,
                             data_page_size=1 << 20), "plain strings maxlen %d %s" % (maxlen, comp))


def test_c5_small_row_groups(tmp_path):
    """C5 shape with 10k-row row groups: l_comment's RLE_DICTIONARY pages then a
    PLAIN page of several k_plain_str items, whole file and single row groups."""
    pytest.importorskip("pyarrow")
    data = _c5_bytes(tmp_path, 70000, 10000, dictionary_pagesize_limit=64 << 10)
    check_file(data, "c5 10k rg0", 0, 1)
    check_file(data, "c5 10k")


def test_two_live_batches_resume(tmp_path):
    """Two batches of one file alive together (as a stream holds them), the
    second created before the first is decoded: each decode bit-exact."""
    pytest.importorskip("pyarrow")
    data = _c5_bytes(tmp_path, 70000, 10000, dictionary_pagesize_limit=64 << 10)
    o = oracle.File(data)
    r = pqgpu.FileReader(data)
    leaves = list(range(len(r.Columns())))
    b0 = r.batch(0, 1, leaves)
    b1 = r.batch(1, 2, leaves)
    errs = []
    for b, rg in ((b0, 0), (b1, 1), (b0, 0)):
        b.decode()
        assert b.sync(raise_on_error=False) == 0
        for i, leaf in enumerate(leaves):
            info = o.leaves()[leaf]
            try:
                assert_same(b.column(i), o.decode(leaf, rg, rg + 1), info["max_def"], info["max_rep"],
                            "two batches rg %d leaf %d" % (rg, leaf))
            except AssertionError as e:
                errs.append(str(e))
    assert not errs, errs
    b0.close()
    b1.close()


def test_stream_reports_slice_errors():
    """A slice whose pages fail to decode reports the batch's first error; a
    stream over a file with an unsupported slice stops there."""
    data = golden_bytes("err_delta_1.parquet")
    o = oracle.File(data)
    r = pqgpu.FileReader(data)
    leaves = list(range(len(r.Columns())))
    codes = []
    with r.stream(0, None, 1, leaves) as st:
        try:
            for b in st:
                codes.append(b.sync(raise_on_error=False))
        except pqgpu.PqgError as e:  # an error found while planning a slice
            codes.append(e.code)
    want = None
    for leaf in leaves:
        try:
            o.decode(leaf)
        except oracle.OracleError as e:
            want = e.code if want is None else want
    assert want is not None and want in codes, (codes, want)


def test_tiled_rle_heavy_keys():
    """Bit width 1 and 2 key streams that alternate RLE and short bit-packed
    runs (the run walk's chain mode; k_expand's general rows)."""
    rng = np.random.default_rng(22)
    rows = 300000
    runs = np.repeat(rng.integers(0, 2, rows // 4), rng.integers(1, 12, rows // 4))[:rows]
    runs4 = np.repeat(rng.integers(0, 4, rows // 3), rng.integers(1, 20, rows // 3))[:rows]
    t = _req_table({"a": (runs * 7 - 1).astype(np.int32), "b": (runs4 * 11 + 5).astype(np.int32),
                    "c": (runs4 * 3).astype(np.int64)})
    check_file(_pq_bytes(t, compression="snappy", row_group_size=100000), "rle heavy")


def test_tiled_corrupted_key_streams_match_oracle():
    """Seeded corruption of uncompressed dictionary data pages (bytes after the
    page headers): whatever the oracle reports — a clean decode, an index out
    of range (type_dict.go:51-53) or a run-header error — the GPU reports the
    same, or decodes the same bytes."""
    pq = pytest.importorskip("pyarrow.parquet")
    rng = np.random.default_rng(23)
    K = 5  # bit width 3: keys 5..7 are out of range
    rows = 40000
    d = np.array([11, -4, 90, 7, 123456], np.int32)
    t = _req_table({"v": d[rng.integers(0, K, rows)]})
    base = _pq_bytes(t, compression="none", row_group_size=rows, data_page_size=8 << 10)
    md = pq.ParquetFile(io.BytesIO(base)).metadata
    cc = md.row_group(0).column(0)
    start = cc.dictionary_page_offset if cc.has_dictionary_page else cc.data_page_offset
    lo, hi = cc.data_page_offset, start + cc.total_compressed_size  # the data pages
    outcomes = set()
    for trial in range(24):
        data = bytearray(base)
        for _ in range(int(rng.integers(1, 4))):
            p = int(rng.integers(lo + 32, hi))
            data[p] ^= int(rng.integers(1, 256))
        check_file(bytes(data), "corrupt %d" % trial)
        o = oracle.File(bytes(data))
        try:
            o.decode(0)
            outcomes.add(0)
        except oracle.OracleError as e:
            outcomes.add(e.code)
    assert len(outcomes) >= 2, outcomes  # the corruptions reach more than one outcome


def test_snappy_literal_train_pages(snappy_kernel):
    """Incompressible Snappy pages longer than one 64 KiB encoder block are a
    train of literals: the host plan copies them with k_copy (no k_snappy).
    Data pages (required, and nullable with their levels inside the V1 body),
    big fixed-width dictionaries, and corrupted literal headers — which leave
    the page to k_snappy and its error classes — against the oracle."""
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(31)
    rows = 300000
    K = 1 << 17
    dvals = rng.integers(-2**31, 2**31 - 1, K, dtype=np.int64).astype(np.int32)
    t = pa.table({
        "r": pa.array(rng.integers(-2**63, 2**63 - 1, rows, dtype=np.int64)),
        "n": pa.array(rng.integers(-2**63, 2**63 - 1, rows, dtype=np.int64), mask=rng.random(rows) < 0.2),
        "d": pa.array(dvals[rng.integers(0, K, rows)]),
    }, schema=pa.schema([pa.field("r", pa.int64(), nullable=False), pa.field("n", pa.int64()),
                         pa.field("d", pa.int32(), nullable=False)]))
    for ver in ("1.0",):  # (pyarrow writes incompressible V2 pages uncompressed: D4)
        base = _pq_bytes(t, compression="snappy", row_group_size=rows // 2, data_page_size=1 << 20,
                         use_dictionary=["d"], dictionary_pagesize_limit=1 << 30, data_page_version=ver)
        check_file(base, "train v" + ver)
        # 64 KiB literal headers (tag 61, length 0xffff): corrupt the tag / length
        hits = [m for m in range(len(base) - 3) if base[m:m + 3] == b"\xf4\xff\xff"]
        assert len(hits) > 20, len(hits)
        for trial in range(10):
            data = bytearray(base)
            m = hits[int(rng.integers(0, len(hits)))]
            data[m + int(rng.integers(0, 3))] ^= int(rng.integers(1, 256))
            check_file(bytes(data), "train v%s corrupt %d" % (ver, trial))


def _snappy_one_literal(body, varint_len):
    """A raw Snappy block that is one literal holding `body`, its decoded-length
    uvarint padded to `varint_len` bytes (binary.Uvarint accepts non-minimal
    encodings, decode.go:38-46)."""
    n, vb = len(body), bytearray()
    for i in range(varint_len):
        b = (n >> (7 * i)) & 0x7F
        vb.append(b | (0x80 if i < varint_len - 1 else 0))
    assert n >> (7 * varint_len) == 0
    x = n - 1
    extra = (x.bit_length() + 7) // 8
    tag = bytes([x << 2]) if x < 60 else bytes([(59 + extra) << 2]) + x.to_bytes(extra, "little")
    return bytes(vb) + tag + body


def test_snappy_single_literal_padded_varint(snappy_kernel):
    """Flat required PLAIN INT64 / INT32 Snappy pages written as one literal
    whose length uvarint is non-minimal (3..10 bytes): the host plan and
    k_snappy must read the varint by the same rules, or a page the host left to
    k_snappy but planned records for (tiled PLAIN) reads unstaged bytes."""
    import pqwrite
    rng = np.random.default_rng(77)
    for ptype, width in ((2, 8), (1, 4)):
        for vlen in (3, 5, 6, 7, 9, 10):
            pages = []
            for n in (8000, 3, 20000):
                vals = rng.integers(-2**62, 2**62, n, dtype=np.int64)
                body = (vals if width == 8 else vals.astype(np.int32)).tobytes()
                pages.append((n, None, body))
            data = pqwrite.write_column(pages, ptype=ptype, encoding=0, codec=1,
                                        compress=lambda b, v=vlen: _snappy_one_literal(b, v))
            check_file(data, "padded varint %d type %d" % (vlen, ptype))
    # an 11-byte (over-long) varint is ErrCorrupt in both
    data = pqwrite.write_column([(100, None, bytes(800))], ptype=2, encoding=0, codec=1,
                                compress=lambda b: b"\x80" * 10 + b"\x00" + _snappy_one_literal(b, 2)[2:])
    check_file(data, "varint 11 bytes")


def test_boolean_columns_generated():
    """BOOLEAN (type_boolean.go): PLAIN bit-packed and RLE pages, nullable,
    required and inside lists, V1 and V2."""
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(31)
    n = 70000
    runs = np.repeat(rng.random(n // 5) < 0.5, rng.integers(1, 20, n // 5))[:n]
    lists = [None if rng.random() < 0.05 else [bool(x) if rng.random() > 0.1 else None
                                                for x in rng.random(rng.poisson(3)) < 0.5] for _ in range(n // 4)]
    t = pa.table({"b": pa.array(rng.random(n) < 0.3, mask=rng.random(n) < 0.1),
                  "r": pa.array(runs)})
    tl = pa.table({"l": pa.array(lists, pa.list_(pa.bool_()))})
    for ver, comp, enc in (("1.0", "snappy", None), ("1.0", "none", "RLE"), ("2.0", "none", None),
                           ("2.0", "none", "PLAIN")):
        kw = dict(compression=comp, data_page_version=ver, use_dictionary=False, row_group_size=30000)
        if enc:
            kw["column_encoding"] = {"b": enc, "r": enc}
        check_file(_pq_bytes(t, **kw), "bool %s %s %s" % (ver, comp, enc))
        kw.pop("column_encoding", None)
        if enc:
            kw["column_encoding"] = {"l": enc}
        check_file(_pq_bytes(tl, **kw), "bool list %s %s %s" % (ver, comp, enc))


def test_boolean_corrupted_pages_match_oracle():
    """Seeded byte corruption of uncompressed BOOLEAN pages (PLAIN V1 and RLE
    V2): the GPU reports the oracle's first error or decodes the same bytes."""
    pq = pytest.importorskip("pyarrow.parquet")
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(32)
    n = 20000
    runs = np.repeat(rng.random(n // 4) < 0.5, rng.integers(1, 16, n // 4))[:n]
    t = pa.table({"r": pa.array(runs)}, schema=pa.schema([pa.field("r", pa.bool_(), nullable=False)]))
    for ver, enc in (("1.0", "PLAIN"), ("2.0", "RLE")):
        base = _pq_bytes(t, compression="none", data_page_version=ver, use_dictionary=False,
                         column_encoding={"r": enc}, row_group_size=n, data_page_size=1 << 10)
        cc = pq.ParquetFile(io.BytesIO(base)).metadata.row_group(0).column(0)
        lo, hi = cc.data_page_offset, cc.data_page_offset + cc.total_compressed_size
        for trial in range(16):
            data = bytearray(base)
            for _ in range(int(rng.integers(1, 4))):
                p = int(rng.integers(lo + 8, hi))
                data[p] ^= int(rng.integers(1, 256))
            check_file(bytes(data), "bool corrupt %s %d" % (enc, trial))


@pytest.mark.parametrize("enc", ["DELTA_LENGTH_BYTE_ARRAY", "DELTA_BYTE_ARRAY"])
def test_delta_strings_generated(enc):
    """DELTA_LENGTH_BYTE_ARRAY / DELTA_BYTE_ARRAY (type_bytearray.go:98-240):
    page sizes around the length streams' block and miniblock edges (the
    reference's lookahead, D3, included), nulls, long values, V1 and V2, lists."""
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(41)
    for n in (1, 2, 63, 64, 65, 129, 130, 700, 25000):
        words = sorted("p%04d:%s" % (rng.integers(0, 500), "xyz" * int(rng.integers(0, 30))) for _ in range(n))
        if n == 700:  # long values, shared prefixes
            words = [w * int(rng.integers(1, 60)) for w in words]
        for nulls in (0.0, 0.2):
            t = pa.table({"s": pa.array(words, type=pa.string(), mask=rng.random(n) < nulls)})
            for ver in ("1.0", "2.0"):
                check_file(_pq_bytes(t, compression="none" if ver == "2.0" else "snappy", data_page_version=ver,
                                     use_dictionary=False, column_encoding={"s": enc}), "%s n%d %.1f v%s" % (enc, n, nulls, ver))
    lists = [None if rng.random() < 0.05 else ["q%d" % v for v in sorted(rng.integers(0, 300, rng.poisson(3)))]
             for _ in range(20000)]
    tl = pa.table({"l": pa.array(lists, pa.list_(pa.string()))})
    check_file(_pq_bytes(tl, compression="snappy", use_dictionary=False, column_encoding={"l": enc}), enc + " list")


@pytest.mark.parametrize("enc", ["DELTA_LENGTH_BYTE_ARRAY", "DELTA_BYTE_ARRAY"])
def test_delta_strings_corrupted_match_oracle(enc):
    """Seeded corruption of uncompressed DELTA string pages: the GPU reports the
    oracle's first error (length-stream init errors, EOF, invalid prefix
    lengths) or decodes the same bytes."""
    pq = pytest.importorskip("pyarrow.parquet")
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(42 if enc[6] == "L" else 43)
    n = 3000
    words = sorted("k%03d/%s" % (rng.integers(0, 300), "ab" * int(rng.integers(0, 6))) for _ in range(n))
    t = pa.table({"s": pa.array(words, type=pa.string())}, schema=pa.schema([pa.field("s", pa.string(), nullable=False)]))
    base = _pq_bytes(t, compression="none", use_dictionary=False, column_encoding={"s": enc}, data_page_size=4 << 10)
    cc = pq.ParquetFile(io.BytesIO(base)).metadata.row_group(0).column(0)
    lo, hi = cc.data_page_offset, cc.data_page_offset + cc.total_compressed_size
    for trial in range(20):
        data = bytearray(base)
        for _ in range(int(rng.integers(1, 4))):
            p = int(rng.integers(lo + 8, hi))
            data[p] ^= int(rng.integers(1, 256))
        check_file(bytes(data), "%s corrupt %d" % (enc, trial))


@pytest.mark.parametrize("shape", ["flat", "list"])
def test_plain_strings_corrupted_match_oracle(shape):
    """Seeded corruption of uncompressed PLAIN BYTE_ARRAY pages, flat and
    list<string> (type_bytearray.go:24-45: u32 length prefixes; a negative
    length is an error, a chain running past the page is EOF): the GPU
    reports the oracle's first error or decodes the same bytes.  k_decode
    reads the (offset, length) pairs k_prepare's walk left in page scratch,
    so this pins that a failed walk never lets stale scratch through."""
    pq = pytest.importorskip("pyarrow.parquet")
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(44 if shape == "flat" else 45)
    n = 4000
    words = ["w%05d%s" % (rng.integers(0, 99999), "z" * int(rng.integers(0, 12))) for _ in range(n)]
    if shape == "flat":
        t = pa.table({"s": pa.array(words, mask=rng.random(n) < 0.1)})
    else:
        lists = [None if rng.random() < 0.05 else words[i:i + int(rng.integers(0, 4))] for i in range(0, n, 2)]
        t = pa.table({"s": pa.array(lists, pa.list_(pa.string()))})
    base = _pq_bytes(t, compression="none", use_dictionary=False, data_page_size=2 << 10)
    cc = pq.ParquetFile(io.BytesIO(base)).metadata.row_group(0).column(0)
    lo, hi = cc.data_page_offset, cc.data_page_offset + cc.total_compressed_size
    outcomes = set()
    for trial in range(24):
        data = bytearray(base)
        for _ in range(int(rng.integers(1, 4))):
            p = int(rng.integers(lo + 8, hi))
            data[p] ^= int(rng.integers(1, 256))
        check_file(bytes(data), "plain strings %s corrupt %d" % (shape, trial))
        try:
            oracle.File(bytes(data)).decode(0)
            outcomes.add(0)
        except oracle.OracleError as e:
            outcomes.add(e.code)
    assert len(outcomes) >= 2, outcomes


def _plain_string_cases(rng):
    """Long PLAIN BYTE_ARRAY pages (>= 64 KiB: the region-parallel length walk,
    k_sw_regions / k_sw_link / k_sw_emit)."""
    pa = pytest.importorskip("pyarrow")
    letters = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz     ", np.uint8)
    n = 60000
    # l_comment-like text
    lens = rng.integers(10, 44, n)
    offs = np.zeros(n + 1, np.int32)
    offs[1:] = np.cumsum(lens)
    text = pa.StringArray.from_buffers(n, pa.py_buffer(offs.tobytes()),
                                       pa.py_buffer(letters[rng.integers(0, len(letters), int(offs[-1]))].tobytes()))
    # binary values: short, empty, longer than a region, longer than a 64-region chunk
    lens = rng.integers(0, 20, n)
    lens[rng.random(n) < 0.02] = rng.integers(300, 3000, int((rng.random(n) < 0.02).sum()) or 1)[0]
    lens[rng.integers(0, n, 3)] = 20000
    offs = np.zeros(n + 1, np.int32)
    offs[1:] = np.cumsum(lens)
    blob = pa.BinaryArray.from_buffers(pa.binary(), n, [None, pa.py_buffer(offs.tobytes()),
                                       pa.py_buffer(rng.integers(0, 256, int(offs[-1]), dtype=np.uint8).tobytes())])
    # values that hold well-formed length prefixes themselves: candidates inside
    # values survive, so regions are walked again from the true entry
    fake = b"\x04\x00\x00\x00abcd\x00\x00\x00\x00"
    adv = pa.array([fake * int(k) for k in rng.integers(0, 6, n)], pa.binary())
    mask = rng.random(n) < 0.15
    return {
        "text": pa.table({"s": text}, schema=pa.schema([pa.field("s", pa.string(), nullable=False)])),
        "blob_nullable": pa.table({"s": pa.array(blob.to_pylist(), pa.binary(), mask=mask)}),
        "adversarial": pa.table({"s": adv}, schema=pa.schema([pa.field("s", pa.binary(), nullable=False)])),
    }


@pytest.mark.parametrize("case", ["text", "blob_nullable", "adversarial"])
def test_plain_strings_region_walk(case):
    """Long PLAIN string pages walked region by region: V1 and V2, Snappy and
    uncompressed, required and nullable, values longer than a region and than
    a chunk of regions, values holding fake length prefixes; then seeded
    corruptions of the uncompressed pages (errors or other chains) — every
    outcome the oracle's."""
    pq = pytest.importorskip("pyarrow.parquet")
    rng = np.random.default_rng(61)
    t = _plain_string_cases(rng)[case]
    for ver in ("1.0", "2.0"):
        for comp in ("none", "snappy"):
            data = _pq_bytes(t, compression=comp, use_dictionary=False, data_page_size=1 << 20,
                             data_page_version=ver, row_group_size=40000)
            check_file(data, "%s v%s %s" % (case, ver, comp))
    base = _pq_bytes(t, compression="none", use_dictionary=False, data_page_size=1 << 20, row_group_size=40000)
    cc = pq.ParquetFile(io.BytesIO(base)).metadata.row_group(0).column(0)
    lo, hi = cc.data_page_offset, cc.data_page_offset + cc.total_compressed_size
    for trial in range(8):
        data = bytearray(base)
        for _ in range(int(rng.integers(1, 3))):
            p = int(rng.integers(lo + 64, hi))
            data[p] ^= int(rng.integers(1, 256))
        check_file(bytes(data), "%s corrupt %d" % (case, trial))
    # one dictionary page per row group holding every distinct value (>= 64 KiB:
    # walked region-parallel before k_dict_prepare), Snappy and uncompressed,
    # and corruptions inside the dictionary page
    for comp in ("none", "snappy"):
        data = _pq_bytes(t, compression=comp, use_dictionary=True, dictionary_pagesize_limit=1 << 30,
                         data_page_size=1 << 20, row_group_size=40000)
        check_file(data, "%s dictionary %s" % (case, comp))
    base = _pq_bytes(t, compression="none", use_dictionary=True, dictionary_pagesize_limit=1 << 30,
                     data_page_size=1 << 20, row_group_size=40000)
    cc = pq.ParquetFile(io.BytesIO(base)).metadata.row_group(0).column(0)
    lo, hi = cc.dictionary_page_offset, cc.data_page_offset
    for trial in range(6 if hi - lo > 64 << 10 else 0):  # (the fake-prefix values have 6 distinct)
        data = bytearray(base)
        p = int(rng.integers(lo + 64, hi))
        data[p] ^= int(rng.integers(1, 256))
        check_file(bytes(data), "%s dictionary corrupt %d" % (case, trial))


# ---------------------------------------------------------------------------
# the reference's own vectors (tests/golden/make_ref_vectors.py)
# ---------------------------------------------------------------------------
import test_reference_vectors as refvec  # noqa: E402


@pytest.mark.parametrize("name", sorted(refvec.KAT))
def test_level_kats_gpu(name):
    """Dremel level KATs (data_store_test.go:18-477) through libpqgpu.so: the
    GPU's def / rep levels and dense values equal the reference's asserted
    arrays, maxR 0, 1 and 2 alike, and every buffer equals the oracle's."""
    data = refvec.kat_file(name)
    rc, got, cols = gpu_decode_all(data, levels=True)
    assert rc == 0, (name, pqgpu.last_error())
    for leaf, c in enumerate(cols):
        want = refvec.KAT[name]["columns"][c["name"]]
        g = got[leaf]
        assert g["def"].tolist() == want["def"], (name, c["name"])
        assert g["rep"].tolist() == want["rep"], (name, c["name"])
        assert refvec.dense_values(g, c["max_def"], c["max_rep"]) == want["values"], (name, c["name"])
    check_file(data, "kat " + name)


@pytest.mark.parametrize("case", refvec.CRASH, ids=[c["test"] for c in refvec.CRASH])
def test_crash_inputs_gpu(case):
    """The reference's fuzz-crash inputs (readAllData) through the whole GPU
    pipeline: no fault, and the first error class equals the oracle's."""
    data = open(os.path.join(GOLDEN, "crash", case["file"]), "rb").read()
    kind, res = refvec.oracle_outcome(data)
    if kind == "open_error":
        with pytest.raises(pqgpu.PqgError) as ei:
            pqgpu.FileReader(data)
        assert ei.value.code == res
        return
    check_file(data, case["test"])


def test_dictionary_page_at_data_page_offset():
    """A chunk whose metadata leaves dictionary_page_offset unset, with the
    dictionary page first at data_page_offset (some writers do): decoded
    from there, bit-exact against the oracle, RLE runs and bit-packed keys."""
    import pqwrite
    rng = np.random.default_rng(45)
    for dn, bw in ((5, 3), (3000, 12), (20000, 15)):
        keys = rng.integers(0, dn, 50000)
        dvals = rng.integers(-2**31, 2**31, dn).astype("<i4").tobytes()
        body = bytes([bw]) + pqwrite.hybrid_bitpacked(keys, bw)
        rgs = [{"dict_page": dvals, "dict_count": dn, "pages": [(50000, None, body), (50000, None, body)]}]
        check_file(pqwrite.write_row_groups(rgs, ptype=1, encoding=8, dict_offset_field=False),
                   "dictionary at data_page_offset, %d entries" % dn)


def test_dict_index_error_before_bad_header():
    """The tiled path's error order in a batch without level streams (C2's
    shape, no k_level_check): the run walk sets a corrupt run header's error
    at once (with E_LATE), and a dictionary-index error k_expand finds among
    the values before that header must still win, as in the reference
    (keys read before a stream error are range-checked first,
    type_dict.go:44-53).  The status is the oracle's in every layout."""
    import pqwrite
    dn, bw = 3, 2  # key 3 is out of range
    good = [0, 1, 2, 1, 0, 2, 1, 0] * 8
    bad = list(good)
    bad[13] = 3
    rle = lambda v, cnt: pqwrite._uvar(cnt << 1) + bytes([v])
    cases = {
        # a bad key, then a run header past the stream (bit-packed groups beyond it)
        "bad key, then truncated run": pqwrite.hybrid_bitpacked(bad, bw) + pqwrite._uvar((40 << 1) | 1) + b"\x00",
        # a bad key, then an empty RLE run
        "bad key, then empty run": pqwrite.hybrid_bitpacked(bad, bw) + b"\x00",
        # good keys, then the bad header alone
        "truncated run alone": pqwrite.hybrid_bitpacked(good, bw) + pqwrite._uvar((40 << 1) | 1) + b"\x00",
        # a bad RLE key after good runs, then the bad header
        "bad RLE key, then empty run": pqwrite.hybrid_bitpacked(good, bw) + rle(3, 8) + b"\x00",
    }
    dvals = np.array([7, -9, 11], "<i4").tobytes()
    for name, keys in cases.items():
        n = 64 + 64
        body = bytes([bw]) + keys
        rgs = [{"dict_page": dvals, "dict_count": dn, "pages": [(n, None, body)]}]
        data = pqwrite.write_row_groups(rgs, ptype=1, encoding=8)
        with pytest.raises(oracle.OracleError):
            oracle.File(data).decode(0)
        check_file(data, name)
