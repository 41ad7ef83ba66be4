"""DELTA encodings at the edges of what the reference decodes.

* DELTA_BINARY_PACKED headers no conformant writer emits but the reference
  reads (deltabp_decoder.go:52-87, :114-175, :211-246, :273-334): miniblock
  sizes that are not a multiple of 8 (read 8 values a group, a miniblock
  started only where the position is a multiple of both), more than 64 (and
  more than 256) miniblocks per block, and the padding check of :150-155 that
  fails for some of them.  Pages are hand-built (tests/deltagen.py lays the
  values out as the reader reads them; tests/pqwrite.py writes the file); the
  oracle must return the encoder's values (or the reader model's error), and
  on the GPU box libpqgpu.so must equal the oracle bit for bit.
* DELTA_LENGTH_BYTE_ARRAY / DELTA_BYTE_ARRAY whose length streams use such
  layouts (the string bytes start where the reader is left, D5 included).
* FIXED_LEN_BYTE_ARRAY columns in DELTA_BYTE_ARRAY (chunk_reader.go:86-96 ->
  byteArrayDeltaDecoder, type_bytearray.go:195-240).
* DELTA_BYTE_ARRAY values longer than 16 KiB (type_bytearray.go:226).
"""
import io

import numpy as np
import pytest

import deltagen
import oracle
import pqwrite

# (block size, miniblocks): conformant, miniblock sizes not a multiple of 8,
# odd sizes, > 64 and > 256 miniblocks, a miniblock longer than most pages
LAYOUTS = [(128, 4), (256, 4), (12, 1), (48, 4), (20, 2), (21, 3), (24, 8), (800, 100), (2400, 300),
           (1040, 65), (1001, 1), (8, 8)]
SIZES = [1, 2, 7, 8, 9, 17, 100, 1000, 2500]
ERR = {"EOF": 10, "DELTA": 13, "BITWIDTH": 15}


def _values(rng, n, bits):
    steps = rng.integers(-3, 40, n)
    big = rng.random(n) < 0.05
    steps[big] = rng.integers(-(1 << 20), 1 << 20, int(big.sum()))
    v = np.cumsum(steps).astype(object) + int(rng.integers(-(1 << (bits - 2)), 1 << (bits - 2)))
    mask = (1 << bits) - 1
    out = []
    for x in v:
        x = int(x) & mask
        out.append(x - (1 << bits) if x >> (bits - 1) else x)
    return out


def _cases():
    rng = np.random.default_rng(71)
    out = []
    for bs, m in LAYOUTS:
        for bits in (32, 64):
            for n in SIZES:
                vals = _values(rng, n, bits)
                if n > 2 and rng.random() < 0.3:  # a wide jump: miniblocks of different widths
                    j = int(rng.integers(1, n))
                    vals[j] = int(rng.integers(-(1 << (bits - 2)), 1 << (bits - 2)))
                out.append((bs, m, bits, n, vals, int(rng.integers(0, 1 << 30))))
    return out


CASES = _cases()


def _file(bs, m, bits, n, vals, seed):
    stream = deltagen.encode(vals, bs, m, bits, rng=np.random.default_rng(seed))
    return pqwrite.write_column([(n, None, stream)], ptype=1 if bits == 32 else 2, encoding=5), stream


def _expect(stream, n, bits):
    try:
        got, _ = deltagen.read(stream, 0, n, bits)
        return got, None
    except deltagen.DeltaError as e:
        return None, ERR[e.kind]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_oracle_delta_layouts(case):
    """The oracle decodes every layout the reference reads, and fails where it fails."""
    bs, m, bits, n, vals, seed = CASES[case]
    data, stream = _file(bs, m, bits, n, vals, seed)
    want, err = _expect(stream, n, bits)
    if err is None:
        assert want == vals, "encoder / reader model disagree"
    try:
        got = oracle.File(data).decode(0)
        assert err is None, ("oracle decoded, reader model fails", err)
        assert got["values"].view(np.int32 if bits == 32 else np.int64).tolist() == vals
    except oracle.OracleError as e:
        assert e.code == err, (e.code, err)


def test_oracle_delta_padding_error_is_reached():
    """At least one layout ends in the padding error of :150-155 (sl < 0)."""
    errs = set()
    for bs, m, bits, n, vals, seed in CASES:
        _, stream = _file(bs, m, bits, n, vals, seed)
        errs.add(_expect(stream, n, bits)[1])
    assert ERR["DELTA"] in errs and None in errs


def _string_page(rng, enc, bs, m, n):
    """values section of a DELTA_LENGTH_BYTE_ARRAY / DELTA_BYTE_ARRAY page whose
    length streams use layout (bs, m); returns (section, values)."""
    words = sorted(bytes(rng.integers(97, 100, int(rng.integers(0, 9)), dtype=np.uint8)) + b"%d" % i for i in range(n))
    if enc == 6:
        suf, pre = words, None
    else:
        pre, suf, prev = [], [], b""
        for w in words:
            k = 0
            while k < min(len(w), len(prev)) and w[k] == prev[k]:
                k += 1
            pre.append(k)
            suf.append(w[k:])
            prev = w
    return length_streams(([pre] if pre is not None else []) + [[len(x) for x in suf]], bs, m, rng) + b"".join(suf), words


def length_streams(streams, bs, m, rng=None):
    """Length streams back to back, each padded to where the reader leaves it."""
    sec = b""
    for lens in streams:
        st = deltagen.encode(lens, bs, m, 32, rng=rng)
        try:  # the reader's skips past the stream are not clamped by what follows
            _, end = deltagen.read(st + bytes(1 << 20), 0, len(lens), 32)
        except deltagen.DeltaError:
            end = len(st)
        sec += deltagen.pad_tail(st, end)
    return sec


@pytest.mark.parametrize("enc", [6, 7])
def test_oracle_delta_string_layouts(enc):
    """Length streams in non-conformant layouts: the strings start where the
    reader is left (its padding skips, D5 included)."""
    rng = np.random.default_rng(72 + enc)
    decoded = 0
    for bs, m in LAYOUTS:
        for n in (1, 9, 100, 700):
            sec, words = _string_page(rng, enc, bs, m, n)
            data = pqwrite.write_column([(n, None, sec)], ptype=6, encoding=enc)
            try:
                got = oracle.File(data).decode(0)
            except oracle.OracleError:
                continue
            offs = got["str_offsets"].view(np.int64)
            vals = got["values"].tobytes()
            assert [vals[offs[i]:offs[i + 1]] for i in range(n)] == words, (bs, m, n)
            decoded += 1
    assert decoded >= len(LAYOUTS)


def _flba_table(pa, n, width, nulls, rng):
    base = rng.integers(97, 123, width, dtype=np.uint8).tobytes()
    vals = []
    for i in range(n):
        k = int(rng.integers(0, width))
        vals.append(base[:k] + rng.integers(97, 123, width - k, dtype=np.uint8).tobytes())
        if rng.random() < 0.3:
            base = vals[-1]
    mask = rng.random(n) < nulls
    return pa.table({"f": pa.array(vals, pa.binary(width), mask=mask)}), vals, mask


def _pq_bytes(t, **kw):
    import pyarrow.parquet as pq
    b = io.BytesIO()
    pq.write_table(t, b, **kw)
    return b.getvalue()


@pytest.mark.parametrize("width", [1, 4, 8, 16, 37])
def test_oracle_flba_delta_byte_array(width):
    """FIXED_LEN_BYTE_ARRAY in DELTA_BYTE_ARRAY (pyarrow-written, nulls, V1 and V2):
    the oracle's slots equal pyarrow's values, nulls zeroed."""
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(80 + width)
    decoded = 0
    for n, nulls in ((1, 0.0), (300, 0.0), (5000, 0.2)):
        t, vals, mask = _flba_table(pa, n, width, nulls, rng)
        for ver in ("1.0", "2.0"):
            data = _pq_bytes(t, use_dictionary=False, column_encoding={"f": "DELTA_BYTE_ARRAY"},
                             data_page_version=ver, compression="none" if ver == "2.0" else "snappy",
                             data_page_size=4096)
            try:
                got = oracle.File(data).decode(0)
            except oracle.OracleError as e:
                # pyarrow writes no block for a single length (D3): the
                # reference's init reads past the stream
                assert n == 1 and e.code in (10, 13, 15), e
                continue
            decoded += 1
            want = b"".join(b"\x00" * width if mk else v for v, mk in zip(vals, mask))
            assert got["values"].tobytes() == want
            if nulls:
                bits = np.unpackbits(got["validity"], bitorder="little")[:n]
                assert (bits == ~mask).all()
    assert decoded >= 4


def _flba_odd_length_file(width, n_ok):
    """A hand-built FLBA DELTA_BYTE_ARRAY page whose value n_ok has width + 1 bytes."""
    words = [b"%0*d" % (width, i) for i in range(n_ok)] + [b"x" * (width + 1)]
    sec = length_streams([[0] * len(words), [len(w) for w in words]], 128, 4) + b"".join(words)
    return pqwrite.write_column([(len(words), None, sec)], ptype=7, encoding=7, type_length=width)


def test_oracle_flba_delta_odd_length_is_an_error():
    with pytest.raises(oracle.OracleError) as ei:
        oracle.File(_flba_odd_length_file(6, 10)).decode(0)
    assert ei.value.code == 14  # PQG_ERR_BYTE_ARRAY (the documented deviation)


def long_value_table(pa, rng):
    words, prev = [], b"q" * 30000
    for i in range(40):
        k = int(rng.integers(0, len(prev) + 1))
        w = prev[:k] + rng.integers(97, 123, int(rng.integers(0, 70000)), dtype=np.uint8).tobytes()
        words.append(w)
        prev = w
    return pa.table({"s": pa.array(words, pa.binary())}), words


def test_oracle_delta_byte_array_long_values():
    pa = pytest.importorskip("pyarrow")
    t, words = long_value_table(pa, np.random.default_rng(90))
    data = _pq_bytes(t, use_dictionary=False, column_encoding={"s": "DELTA_BYTE_ARRAY"}, compression="snappy")
    got = oracle.File(data).decode(0)
    offs = got["str_offsets"].view(np.int64)
    assert [got["values"].tobytes()[offs[i]:offs[i + 1]] for i in range(len(words))] == words


# ---------------------------------------------------------------------------
# the same files through libpqgpu.so (GPU box)
# ---------------------------------------------------------------------------
def _gpu_check(data, ctx):
    import test_gpu_parity as gp
    gp.check_file(data, ctx)


@pytest.mark.gpu
def test_gpu_delta_layouts():
    for i, (bs, m, bits, n, vals, seed) in enumerate(CASES):
        data, _ = _file(bs, m, bits, n, vals, seed)
        _gpu_check(data, "delta layout %d (%d/%d, %d-bit, n %d)" % (i, bs, m, bits, n))
    # several pages of different layouts in one chunk
    rng = np.random.default_rng(73)
    pages = []
    for bs, m in LAYOUTS[:6]:
        vals = _values(rng, 333, 64)
        st = deltagen.encode(vals, bs, m, 64, rng=rng)
        pages.append((333, None, st))
    _gpu_check(pqwrite.write_column(pages, ptype=2, encoding=5), "delta layouts, one chunk")


@pytest.mark.gpu
@pytest.mark.parametrize("enc", [6, 7])
def test_gpu_delta_string_layouts(enc):
    rng = np.random.default_rng(72 + enc)
    for bs, m in LAYOUTS:
        for n in (1, 9, 100, 700):
            sec, _ = _string_page(rng, enc, bs, m, n)
            _gpu_check(pqwrite.write_column([(n, None, sec)], ptype=6, encoding=enc), "strings %d %d/%d n%d" % (enc, bs, m, n))


@pytest.mark.gpu
@pytest.mark.parametrize("width", [1, 4, 8, 16, 37])
def test_gpu_flba_delta_byte_array(width):
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(80 + width)
    for n, nulls in ((1, 0.0), (300, 0.0), (5000, 0.2)):
        t, _, _ = _flba_table(pa, n, width, nulls, rng)
        for ver in ("1.0", "2.0"):
            data = _pq_bytes(t, use_dictionary=False, column_encoding={"f": "DELTA_BYTE_ARRAY"},
                             data_page_version=ver, compression="none" if ver == "2.0" else "snappy",
                             data_page_size=4096)
            _gpu_check(data, "flba %d n%d v%s" % (width, n, ver))
    lists = [None if rng.random() < 0.1 else [bytes([97 + i % 26]) * width for i in range(int(rng.integers(0, 4)))]
             for _ in range(2000)]
    tl = pa.table({"l": pa.array(lists, pa.list_(pa.binary(width)))})
    _gpu_check(_pq_bytes(tl, use_dictionary=False, column_encoding={"l": "DELTA_BYTE_ARRAY"}), "flba list %d" % width)
    _gpu_check(_flba_odd_length_file(width, 70), "flba odd length %d" % width)


@pytest.mark.gpu
def test_gpu_delta_byte_array_long_values():
    pa = pytest.importorskip("pyarrow")
    t, _ = long_value_table(pa, np.random.default_rng(90))
    for ver in ("1.0", "2.0"):
        _gpu_check(_pq_bytes(t, use_dictionary=False, column_encoding={"s": "DELTA_BYTE_ARRAY"}, compression="snappy",
                             data_page_version=ver), "long DBA values v" + ver)
    w = 20000  # FLBA values past the LDS copy of the previous value
    rng = np.random.default_rng(91)
    t2, _, _ = _flba_table(pa, 30, w, 0.1, rng)
    _gpu_check(_pq_bytes(t2, use_dictionary=False, column_encoding={"f": "DELTA_BYTE_ARRAY"}), "flba 20000")
