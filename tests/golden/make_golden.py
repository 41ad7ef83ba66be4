"""Generate the committed golden fixtures under tests/golden/.

Run in the build container (needs pyarrow 25 and, for the KAT tables, a
readable /root/reference).  The GPU box never runs this script: it only reads
the committed outputs.

1. kat_bitpack.json — the reference's own bit-unpacking known-answer tables,
   transcribed verbatim (data only) from
     /root/reference/bitpacking32_test.go:25-654  (unpack8int32Tests, widths 0-32)
     /root/reference/bitpacking64_test.go:25-1744 (unpack8int64Tests, widths 0-64)
2. *.parquet + *.npz — small Parquet files written by pyarrow 25.0.0 (an
   independent, spec-conformant writer/reader) and their decoded outputs in the
   canonical layout both decoders emit (values spaced over slots with nulls
   zeroed, LSB-first validity bitmaps, int32 list offsets, int64 string offsets).
3. manifest.json — per file/column: expected npz keys, or the expected error
   class for files the reference decoder rejects (defects D3/D4 in SURVEY.md).
"""
import io
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


# ----------------------------------------------------------------------------
# 1. KAT tables
# ----------------------------------------------------------------------------
def _parse_kat(path, bits):
    src = open(path).read()
    start = src.index("unpack8int%dTests" % bits)
    body = src[start:]
    # entries look like {W, []byte{...}, [8]intNN{...}} possibly over several lines
    pat = re.compile(r"\{\s*(\d+),\s*\[\]byte\{([^}]*)\},\s*\[8\]int%d\{([^}]*)\},?\s*\}" % bits, re.S)
    out = []
    for m in pat.finditer(body):
        width = int(m.group(1))
        data = [int(x, 0) for x in m.group(2).replace("\n", " ").split(",") if x.strip()]
        vals = [int(x, 0) for x in m.group(3).replace("\n", " ").split(",") if x.strip()]
        assert len(vals) == 8 and len(data) == width, (width, data, vals)
        out.append({"width": width, "data": bytes(data).hex(), "values": vals})
    return out


def make_kat():
    k32 = _parse_kat(os.path.join(REF, "bitpacking32_test.go"), 32)
    k64 = _parse_kat(os.path.join(REF, "bitpacking64_test.go"), 64)
    with open(os.path.join(HERE, "kat_bitpack.json"), "w") as f:
        json.dump({"source": {"int32": "bitpacking32_test.go:25-654", "int64": "bitpacking64_test.go:25-1744"},
                   "int32": k32, "int64": k64}, f, indent=0)
    print("kat: %d int32 vectors, %d int64 vectors" % (len(k32), len(k64)))


# ----------------------------------------------------------------------------
# 2. canonical expected layout from a pyarrow array
# ----------------------------------------------------------------------------
def _bits(mask):
    return np.packbits(np.asarray(mask, dtype=np.uint8), bitorder="little")


def canon_flat(arr, width=None):
    """Flat (maxR == 0) column -> dict of canonical buffers."""
    import pyarrow as pa
    arr = arr.combine_chunks() if hasattr(arr, "combine_chunks") else arr
    n = len(arr)
    valid = np.ones(n, bool) if arr.null_count == 0 else ~np.asarray(arr.is_null())
    out = {"slots": np.int64(n), "validity": _bits(valid)}
    t = arr.type
    if pa.types.is_string(t) or pa.types.is_binary(t) or pa.types.is_large_string(t):
        vals = arr.to_pylist()
        bs = [(v.encode() if isinstance(v, str) else v) if v is not None else b"" for v in vals]
        offs = np.zeros(n + 1, np.int64)
        offs[1:] = np.cumsum([len(b) for b in bs])
        out["str_offsets"] = offs.view(np.uint8)
        out["values"] = np.frombuffer(b"".join(bs), np.uint8)
    else:
        np_t = {8: None}
        filled = arr.fill_null(False if pa.types.is_boolean(t) else 0) if arr.null_count else arr
        v = np.asarray(filled.to_numpy(zero_copy_only=False))
        out["values"] = np.ascontiguousarray(v).view(np.uint8).ravel()
    return out


def canon_list(arr):
    """LIST<primitive> column (maxR == 1) -> canonical buffers."""
    import pyarrow as pa
    arr = arr.combine_chunks()
    n = len(arr)
    lvalid = np.ones(n, bool) if arr.null_count == 0 else ~np.asarray(arr.is_null())
    lens = np.asarray(arr.value_lengths().fill_null(0))
    offs = np.zeros(n + 1, np.int32)
    offs[1:] = np.cumsum(lens)
    # flatten the present elements in row order (null rows contribute nothing)
    elems = pa.concat_arrays([arr[i].values for i in range(n) if arr[i].is_valid]) if n else pa.array([], arr.type.value_type)
    e = canon_flat(elems)
    return {"rows": np.int64(n), "list_offsets": offs.view(np.uint8), "list_validity": _bits(lvalid),
            "slots": e["slots"], "validity": e["validity"], "values": e["values"]}


# ----------------------------------------------------------------------------
# 3. fixtures
# ----------------------------------------------------------------------------
def write(name, table, **kw):
    import pyarrow.parquet as pq
    path = os.path.join(HERE, name + ".parquet")
    pq.write_table(table, path, **kw)
    return path


def fixtures():
    import pyarrow as pa
    manifest = {}

    def record(name, table, columns, errors=None, **kw):
        write(name, table, **kw)
        exp = {}
        entry = {"file": name + ".parquet", "columns": {}, "writer": {k: str(v) for k, v in kw.items()}}
        for leaf, (colname, kind) in enumerate(columns):
            key = "c%d" % leaf
            if errors and leaf in errors:
                entry["columns"][key] = {"leaf": leaf, "error": errors[leaf][0], "why": errors[leaf][1]}
                continue
            arr = table.column(colname)
            d = canon_list(arr) if kind == "list" else canon_flat(arr)
            for k, v in d.items():
                exp["%s_%s" % (key, k)] = np.asarray(v)
            entry["columns"][key] = {"leaf": leaf, "kind": kind}
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **exp)
        manifest[name] = entry

    rng = np.random.default_rng(1)
    # C1 shape: required INT64, PLAIN, uncompressed, V1 (multi row group, multi page)
    t = pa.table({"a": pa.array(rng.integers(-2**63, 2**63 - 1, 50000, dtype=np.int64))},
                 schema=pa.schema([pa.field("a", pa.int64(), nullable=False)]))
    record("c1_int64_plain", t, [("a", "flat")], use_dictionary=False, compression="none",
           data_page_version="1.0", row_group_size=20000, max_rows_per_page=5000)

    # C2 shape: required INT32 dictionary, Snappy, V1, several bit widths
    rng = np.random.default_rng(2)
    for bw, rows in ((1, 30000), (2, 30000), (4, 30000), (8, 30000), (12, 40000), (16, 70000)):
        K = 1 << bw
        dvals = rng.permutation(np.arange(-(2**31), 2**31 - 1, max(1, (2**32) // (K + 7)), dtype=np.int64)[:K]).astype(np.int32)
        idx = rng.integers(0, K, rows)
        t = pa.table({"v": pa.array(dvals[idx])}, schema=pa.schema([pa.field("v", pa.int32(), nullable=False)]))
        record("c2_dict_bw%d" % bw, t, [("v", "flat")], compression="snappy", data_page_version="1.0",
               dictionary_pagesize_limit=1 << 30, row_group_size=16384)
    # run-heavy index stream (geometric runs, mean 16) exercises RLE runs
    K = 256
    runs = rng.geometric(1 / 16, 4000)
    idx = np.repeat(rng.integers(0, K, len(runs)), runs)[:40000]
    dvals = rng.permutation(K).astype(np.int32) * 7919
    t = pa.table({"v": pa.array(dvals[idx])}, schema=pa.schema([pa.field("v", pa.int32(), nullable=False)]))
    record("c2_dict_runs", t, [("v", "flat")], compression="snappy", data_page_version="1.0",
           dictionary_pagesize_limit=1 << 30, row_group_size=16384)

    # C3 shape: DELTA_BINARY_PACKED INT64 ts + optional DOUBLE, V2, Snappy
    rng = np.random.default_rng(3)
    n = 50000
    step = np.where(rng.random(n) < 0.95, 1000, rng.integers(0, 4096, n))
    ts = (1_600_000_000_000_000 + np.cumsum(step)).astype(np.int64)
    x = np.round(rng.standard_normal(n), 2)
    xm = rng.random(n) < 0.1
    t = pa.table({"ts": pa.array(ts), "x": pa.array(x, mask=xm)},
                 schema=pa.schema([pa.field("ts", pa.int64(), nullable=False), pa.field("x", pa.float64())]))
    record("c3_delta_v2", t, [("ts", "flat"), ("x", "flat")], compression="snappy", data_page_version="2.0",
           use_dictionary=False, column_encoding={"ts": "DELTA_BINARY_PACKED", "x": "PLAIN"}, row_group_size=20000)

    # C4 shape: LIST<INT32> + dictionary STRING, rep/def levels, V1, Snappy
    rng = np.random.default_rng(4)
    n = 30000
    lens = rng.poisson(4, n)
    lists = []
    for i in range(n):
        u = rng.random()
        if u < 0.05:
            lists.append(None)
        elif u < 0.10:
            lists.append([])
        else:
            lists.append([None if rng.random() < 0.05 else int(v) for v in rng.integers(-1000, 1000, lens[i])])
    vocab = ["".join(chr(97 + c) for c in rng.integers(0, 26, rng.integers(4, 17))) for _ in range(1000)]
    s = [None if rng.random() < 0.1 else vocab[j] for j in rng.integers(0, 1000, n)]
    t = pa.table({"l": pa.array(lists, pa.list_(pa.int32())), "s": pa.array(s, pa.string())})
    record("c4_list_str", t, [("l", "list"), ("s", "flat")], compression="snappy", data_page_version="1.0",
           row_group_size=12000)

    # PLAIN BYTE_ARRAY (no dictionary), optional, Snappy
    rng = np.random.default_rng(6)
    n = 20000
    s = [None if rng.random() < 0.2 else "".join(chr(33 + c) for c in rng.integers(0, 90, rng.integers(0, 40)))
         for _ in range(n)]
    t = pa.table({"s": pa.array(s, pa.string())})
    record("plain_strings", t, [("s", "flat")], compression="snappy", use_dictionary=False, row_group_size=8000)

    # mixed: FLOAT, INT32 DELTA with nulls, uncompressed V2
    rng = np.random.default_rng(7)
    n = 25000
    f32 = rng.standard_normal(n).astype(np.float32)
    i32 = np.cumsum(rng.integers(-3, 50, n)).astype(np.int32)
    t = pa.table({"f": pa.array(f32), "d": pa.array(i32, mask=rng.random(n) < 0.3)},
                 schema=pa.schema([pa.field("f", pa.float32(), nullable=False), pa.field("d", pa.int32())]))
    record("mixed_v2_none", t, [("f", "flat"), ("d", "flat")], compression="none", data_page_version="2.0",
           use_dictionary=False, column_encoding={"f": "PLAIN", "d": "DELTA_BINARY_PACKED"}, row_group_size=10000)

    # GZIP pages (host inflate path)
    rng = np.random.default_rng(8)
    t = pa.table({"g": pa.array(rng.integers(0, 100, 10000).astype(np.int64), mask=rng.random(10000) < 0.05)})
    record("gzip_int64", t, [("g", "flat")], compression="gzip", row_group_size=4000)

    # dictionary with a single entry -> index bit width 0
    t = pa.table({"z": pa.array(np.full(5000, 42, np.int32))}, schema=pa.schema([pa.field("z", pa.int32(), nullable=False)]))
    record("dict_bw0", t, [("z", "flat")], compression="snappy")

    # all-null optional columns (PLAIN int32 and dictionary string)
    t = pa.table({"n": pa.array([None] * 3000, pa.int32()), "s": pa.array([None] * 3000, pa.string())})
    record("all_null", t, [("n", "flat"), ("s", "flat")], compression="snappy", use_dictionary=["s"])

    # FIXED_LEN_BYTE_ARRAY (decimal128 stored as FLBA(16))
    import decimal
    rng = np.random.default_rng(9)
    dec = [None if rng.random() < 0.1 else decimal.Decimal(int(v)) / 100 for v in rng.integers(-10**12, 10**12, 6000)]
    t = pa.table({"m": pa.array(dec, pa.decimal128(38, 2))})
    # canonical expected: the FLBA big-endian bytes as stored (decimal128 -> 16 bytes BE)
    write("flba_decimal", t, compression="snappy", use_dictionary=False, row_group_size=2500, store_decimal_as_integer=False)
    vals = np.zeros((len(dec), 16), np.uint8)
    for i, d in enumerate(dec):
        if d is not None:
            iv = int(d.scaleb(2))
            vals[i] = np.frombuffer(iv.to_bytes(16, "big", signed=True), np.uint8)
    valid = np.array([d is not None for d in dec])
    np.savez_compressed(os.path.join(HERE, "flba_decimal.npz"), c0_values=vals.ravel(), c0_validity=_bits(valid),
                        c0_slots=np.int64(len(dec)))
    manifest["flba_decimal"] = {"file": "flba_decimal.parquet", "columns": {"c0": {"leaf": 0, "kind": "flat"}}}

    # BOOLEAN: PLAIN bit-packed (V1) and RLE (V2)
    rng = np.random.default_rng(13)
    n = 30000
    t = pa.table({"b": pa.array(rng.random(n) < 0.3, mask=rng.random(n) < 0.1),
                  "r": pa.array(rng.random(n) < 0.5)},
                 schema=pa.schema([pa.field("b", pa.bool_()), pa.field("r", pa.bool_(), nullable=False)]))
    record("bool_v1_plain", t, [("b", "flat"), ("r", "flat")], compression="snappy", data_page_version="1.0",
           use_dictionary=False, row_group_size=16384)
    runs = np.repeat(rng.random(n // 12) < 0.4, rng.integers(1, 24, n // 12))[:n]
    t = pa.table({"b": pa.array(runs[:n], mask=rng.random(len(runs[:n])) < 0.2),
                  "r": pa.array(rng.random(len(runs[:n])) < 0.5)},
                 schema=pa.schema([pa.field("b", pa.bool_()), pa.field("r", pa.bool_(), nullable=False)]))
    record("bool_v2_rle", t, [("b", "flat"), ("r", "flat")], compression="none", data_page_version="2.0",
           use_dictionary=False, column_encoding={"b": "RLE", "r": "RLE"}, row_group_size=16384)

    # DELTA_LENGTH_BYTE_ARRAY / DELTA_BYTE_ARRAY strings:
    # sorted words (shared prefixes), nulls, several pages and row groups
    rng = np.random.default_rng(14)
    n = 45000
    words = sorted("k%05d/%s" % (rng.integers(0, 4000), "ab" * int(rng.integers(0, 9))) for _ in range(n))
    t = pa.table({"l": pa.array(words, type=pa.string(), mask=rng.random(n) < 0.1),
                  "d": pa.array(words, type=pa.string(), mask=rng.random(n) < 0.05)})
    record("delta_strings", t, [("l", "flat"), ("d", "flat")], compression="snappy", data_page_version="1.0",
           use_dictionary=False, column_encoding={"l": "DELTA_LENGTH_BYTE_ARRAY", "d": "DELTA_BYTE_ARRAY"},
           row_group_size=20000)

    # ---- reference-rejected files (defects D3 / D4 in SURVEY.md Appendix) ----
    # D3: DELTA page whose value count is 1 + 256k -> lookahead reads a missing block header
    t = pa.table({"ts": pa.array(np.arange(257, dtype=np.int64) * 3)},
                 schema=pa.schema([pa.field("ts", pa.int64(), nullable=False)]))
    record("err_delta_257", t, [("ts", "flat")], errors={0: (10, "D3: deltabp_decoder.go:329-332 lookahead past last block")},
           compression="none", use_dictionary=False, column_encoding={"ts": "DELTA_BINARY_PACKED"})
    # D3: single-value DELTA page: init reads a miniblock header that pyarrow never writes
    t = pa.table({"ts": pa.array(np.array([12345], dtype=np.int64))},
                 schema=pa.schema([pa.field("ts", pa.int64(), nullable=False)]))
    record("err_delta_1", t, [("ts", "flat")], errors={0: (10, "D3: deltabp_decoder.go:197-209 init needs a block")},
           compression="none", use_dictionary=False, column_encoding={"ts": "DELTA_BINARY_PACKED"})
    # D4: V2 page with is_compressed=false (incompressible doubles) is still fed to snappy
    rng = np.random.default_rng(10)
    t = pa.table({"x": pa.array(rng.standard_normal(4000))},
                 schema=pa.schema([pa.field("x", pa.float64(), nullable=False)]))
    record("err_v2_uncompressed_flag", t, [("x", "flat")],
           errors={0: (7, "D4: page_v2.go:123 ignores is_compressed; snappy rejects the raw bytes")},
           compression="snappy", data_page_version="2.0", use_dictionary=False)

    # D3 on a length stream: 129 strings -> the lookahead of the 129th length
    # reads a block header out of the string bytes (widths > 32 here)
    t = pa.table({"s": pa.array(["w%03d" % i for i in range(129)], type=pa.string())},
                 schema=pa.schema([pa.field("s", pa.string(), nullable=False)]))
    record("err_delta_strings_129", t, [("s", "flat")],
           errors={0: (15, "D3: deltabp_decoder.go:115-127 lookahead reads a block header from the string bytes")},
           compression="none", use_dictionary=False, column_encoding={"s": "DELTA_LENGTH_BYTE_ARRAY"})

    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("fixtures:", ", ".join(sorted(manifest)))


if __name__ == "__main__":
    what = sys.argv[1:] or ["kat", "fixtures"]
    if "kat" in what:
        make_kat()
    if "fixtures" in what:
        fixtures()
