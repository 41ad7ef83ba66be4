"""Synthetic Parquet files for the BASELINE.json configs.

Written with pyarrow on the machine that runs the bench (seeded, row group by
row group so host memory stays at one row group).  Only the bench and the
analysis tools import this; the decoder never does.

  c1  required INT64, PLAIN, uncompressed, V1                      (configs[0])
  c2  required INT32 dictionary, index bit width 1..20, Snappy, V1  (configs[1])
  c2runs  the same with run-heavy keys: runs of one key, geometric
          length with mean 16 (SURVEY.md §8(d) C2's run-heavy variant)
  c3  DELTA_BINARY_PACKED INT64 ts + optional DOUBLE, V2, Snappy    (configs[2])
  c4  LIST<INT32> + dictionary STRING with rep/def levels, V1       (configs[3])
  c5  TPC-H lineitem-shaped, 16 columns, Snappy, V1                 (configs[4])
  c5gz    C5's columns under GZIP (the k_inflate measurement, tools/gzip_ab.py)
"""
import os
import sys

import numpy as np

# rows per GPU and rows per row group of each config (c5: one GPU's share of the
# 256 row groups x ~1.41M rows of configs[4] at 8 GPUs = 32 row groups)
DEFAULTS = {
    "c1": (10_000_000, 1 << 20),
    "c2": (100_000_000, 1 << 20),
    "c2runs": (100_000_000, 1 << 20),
    "c3": (100_000_000, 1 << 20),
    "c4": (20_000_000, 1 << 20),
    "c5": (45_300_000, 1_415_625),
    "c5gz": (5_662_500, 707_813),
}

DESCR = {
    "c1": "C1: INT64 PLAIN, uncompressed, V1, %d rows, %d-row row groups",
    "c2": "C2: INT32 RLE_DICTIONARY bw 1-20, Snappy, V1, %d rows, %d-row row groups",
    "c2runs": "C2 run-heavy: INT32 RLE_DICTIONARY bw 1-20, keys in runs of geometric length (mean 16), Snappy, V1, "
              "%d rows, %d-row row groups",
    "c3": "C3: DELTA_BINARY_PACKED INT64 ts + optional DOUBLE (10%% nulls), V2, Snappy, %d rows, %d-row row groups",
    "c4": "C4: LIST<INT32> (maxD 3, maxR 1) + dictionary STRING (10%% nulls), V1, Snappy, %d rows, %d-row row groups",
    "c5": "C5: TPC-H lineitem-shaped 16 columns, Snappy, V1, %d rows, %d-row row groups (one GPU's 32 of 256 RGs)",
    "c5gz": "C5 under GZIP (level 6): TPC-H lineitem-shaped 16 columns, V1, %d rows, %d-row row groups",
}

DTYPE = {"c1": "int64", "c2": "int32", "c2runs": "int32", "c3": "int64+f64 bits", "c4": "int32+bytes", "c5": "int64/int32/f64 bits/bytes",
         "c5gz": "int64/int32/f64 bits/bytes"}


def _write(path, schema, gen, rows, rg_rows, **kw):
    import pyarrow.parquet as pq
    tmp = path + ".tmp%d" % os.getpid()
    with pq.ParquetWriter(tmp, schema, **kw) as w:
        done, i = 0, 0
        while done < rows:
            n = min(rg_rows, rows - done)
            w.write_table(gen(i, done, n), row_group_size=n)
            if i % 8 == 7:
                print("synth: %s row group %d (%d rows)" % (os.path.basename(path), i + 1, done + n),
                      file=sys.stderr, flush=True)
            done += n
            i += 1
    os.replace(tmp, path)


def make(cfg, path, rows, rg_rows, fixed_bw=0, **writer_kw):
    """Write config `cfg` to `path`.  `writer_kw` overrides pyarrow writer
    options (tests use a small dictionary_pagesize_limit to force the PLAIN
    fallback of l_comment inside a small file)."""
    import pyarrow as pa
    import pyarrow.compute as pc

    if cfg == "c1":
        rng = np.random.default_rng(1)
        schema = pa.schema([pa.field("a", pa.int64(), nullable=False)])
        gen = lambda i, d, n: pa.table({"a": pa.array(rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64))},
                                       schema=schema)
        _write(path, schema, gen, rows, rg_rows, use_dictionary=False, compression="none", data_page_version="1.0")

    elif cfg == "c2":
        rng = np.random.default_rng(2)
        schema = pa.schema([pa.field("v", pa.int32(), nullable=False)])

        def gen(i, d, n):
            bw = fixed_bw if fixed_bw else 1 + (i % 20)
            K = 1 << bw
            dvals = (rng.permutation(K).astype(np.int64) * 2654435761 % (1 << 32) - (1 << 31)).astype(np.int32)
            return pa.table({"v": pa.array(dvals[rng.integers(0, K, n)])}, schema=schema)
        _write(path, schema, gen, rows, rg_rows, compression="snappy", use_dictionary=True,
               data_page_version="1.0", dictionary_pagesize_limit=1 << 30)

    elif cfg == "c2runs":
        # every row group: runs of one dictionary key, run lengths geometric
        # with mean 16 (pyarrow's hybrid encoder makes RLE runs of the runs of
        # 8 or more, bit-packed groups of the rest), so the pages take the
        # run-table path of the expand and compress under Snappy
        rng = np.random.default_rng(22)
        schema = pa.schema([pa.field("v", pa.int32(), nullable=False)])

        def gen(i, d, n):
            bw = fixed_bw if fixed_bw else 1 + (i % 20)
            K = 1 << bw
            dvals = (rng.permutation(K).astype(np.int64) * 2654435761 % (1 << 32) - (1 << 31)).astype(np.int32)
            lens = rng.geometric(1.0 / 16, n // 8 + 64)
            while lens.sum() < n:
                lens = np.concatenate([lens, rng.geometric(1.0 / 16, n // 8 + 64)])
            keys = np.repeat(rng.integers(0, K, len(lens)), lens)[:n]
            return pa.table({"v": pa.array(dvals[keys])}, schema=schema)
        _write(path, schema, gen, rows, rg_rows, compression="snappy", use_dictionary=True,
               data_page_version="1.0", dictionary_pagesize_limit=1 << 30)

    elif cfg == "c3":
        # this distribution keeps every V2 page compressible, so
        # is_compressed is true on every page (D4 not triggered)
        rng = np.random.default_rng(3)
        schema = pa.schema([pa.field("ts", pa.int64(), nullable=False), pa.field("x", pa.float64())])
        last = [1_600_000_000_000_000]

        def gen(i, d, n):
            step = np.where(rng.random(n) < 0.95, 1000, rng.integers(0, 4096, n))
            ts = last[0] + np.cumsum(step)
            last[0] = int(ts[-1])
            x = np.round(rng.standard_normal(n), 2)
            return pa.table({"ts": pa.array(ts.astype(np.int64)), "x": pa.array(x, mask=rng.random(n) < 0.1)},
                            schema=schema)
        _write(path, schema, gen, rows, rg_rows, compression="snappy", data_page_version="2.0", use_dictionary=False,
               column_encoding={"ts": "DELTA_BINARY_PACKED", "x": "PLAIN"})

    elif cfg == "c4":
        rng = np.random.default_rng(4)
        vocab = pa.array(["".join(chr(97 + c) for c in rng.integers(0, 26, rng.integers(4, 17))) for _ in range(1000)])
        schema = pa.schema([pa.field("l", pa.list_(pa.int32())), pa.field("s", pa.string())])

        def gen(i, d, n):
            u = rng.random(n)
            null_list, empty = u < 0.05, (u >= 0.05) & (u < 0.10)
            lens = np.where(null_list | empty, 0, rng.poisson(4, n))
            offs = np.zeros(n + 1, np.int32)
            offs[1:] = np.cumsum(lens)
            m = int(offs[-1])
            vals = pa.array(rng.integers(-1000, 1000, m).astype(np.int32), mask=rng.random(m) < 0.05)
            lst = pa.ListArray.from_arrays(pa.array(offs), vals, mask=pa.array(null_list))
            s = pc.take(vocab, pa.array(rng.integers(0, 1000, n), mask=rng.random(n) < 0.1))
            return pa.table({"l": lst, "s": s}, schema=schema)
        _write(path, schema, gen, rows, rg_rows, compression="snappy", data_page_version="1.0")

    elif cfg == "c5":
        rng = np.random.default_rng(5)
        i64, i32, f64, st = pa.int64(), pa.int32(), pa.float64(), pa.string()
        cols = [("l_orderkey", i64), ("l_partkey", i64), ("l_suppkey", i64), ("l_linenumber", i32),
                ("l_quantity", f64), ("l_extendedprice", f64), ("l_discount", f64), ("l_tax", f64),
                ("l_returnflag", st), ("l_linestatus", st), ("l_shipdate", i32), ("l_commitdate", i32),
                ("l_receiptdate", i32), ("l_shipinstruct", st), ("l_shipmode", st), ("l_comment", st)]
        schema = pa.schema([pa.field(c, t, nullable=False) for c, t in cols])
        sf = 60
        flags, status = pa.array(["A", "N", "R"]), pa.array(["O", "F"])
        instr = pa.array(["DELIVER IN PERSON", "COLLECT COD", "NONE", "TAKE BACK RETURN"])
        modes = pa.array(["REG AIR", "AIR", "RAIL", "SHIP", "TRUCK", "MAIL", "FOB"])
        letters = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz     ", np.uint8)

        def gen(i, d, n):
            row = d + np.arange(n, dtype=np.int64)
            qty = rng.integers(1, 51, n).astype(np.float64)
            ship = rng.integers(8035, 10561, n).astype(np.int32)  # 1992-01-02 .. 1998-12-01
            clen = rng.integers(10, 44, n)
            coff = np.zeros(n + 1, np.int32)
            coff[1:] = np.cumsum(clen)
            cdat = letters[rng.integers(0, len(letters), int(coff[-1]))]
            comment = pa.StringArray.from_buffers(n, pa.py_buffer(coff.tobytes()), pa.py_buffer(cdat.tobytes()))
            t = {
                "l_orderkey": pa.array(row // 4 * 4 + 1),
                "l_partkey": pa.array(rng.integers(1, 200_000 * sf + 1, n)),
                "l_suppkey": pa.array(rng.integers(1, 10_000 * sf + 1, n)),
                "l_linenumber": pa.array((row % 7 + 1).astype(np.int32)),
                "l_quantity": pa.array(qty),
                "l_extendedprice": pa.array(np.round(qty * rng.uniform(900, 2100, n), 2)),
                "l_discount": pa.array(rng.integers(0, 11, n) / 100.0),
                "l_tax": pa.array(rng.integers(0, 9, n) / 100.0),
                "l_returnflag": pc.take(flags, pa.array(rng.integers(0, 3, n))),
                "l_linestatus": pc.take(status, pa.array(rng.integers(0, 2, n))),
                "l_shipdate": pa.array(ship),
                "l_commitdate": pa.array(ship + rng.integers(-60, 61, n).astype(np.int32)),
                "l_receiptdate": pa.array(ship + rng.integers(1, 31, n).astype(np.int32)),
                "l_shipinstruct": pc.take(instr, pa.array(rng.integers(0, 4, n))),
                "l_shipmode": pc.take(modes, pa.array(rng.integers(0, 7, n))),
                "l_comment": comment,
            }
            return pa.table(t, schema=schema)
        kw = dict(compression="snappy", data_page_version="1.0")
        kw.update(writer_kw)
        _write(path, schema, gen, rows, rg_rows, **kw)
    elif cfg == "c5gz":
        kw = dict(compression="gzip", compression_level=6)
        kw.update(writer_kw)
        make("c5", path, rows, rg_rows, **kw)
    else:
        raise ValueError("unknown config %r" % cfg)
