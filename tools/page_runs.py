"""Analysis aid: RLE/bit-packed run statistics of dictionary-index pages as
pyarrow writes them (uncompressed file, one row group per bit width).

usage: python tools/page_runs.py [rows_per_rg]
"""
import os
import sys

import numpy as np


def uvarint(b, i):
    x = s = 0
    while True:
        c = b[i]
        i += 1
        x |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return x, i


def skip_struct(b, i):
    """compact-thrift struct: returns {field_id: value-or-substruct} for ints/structs we need"""
    out = {}
    fid = 0
    while True:
        h = b[i]
        i += 1
        if h == 0:
            return out, i
        t = h & 0x0F
        d = h >> 4
        if d:
            fid += d
        else:
            z, i = uvarint(b, i)
            fid = (z >> 1) ^ -(z & 1)
        if t in (5, 6, 4):  # i32 / i64 / i16 zigzag
            z, i = uvarint(b, i)
            out[fid] = (z >> 1) ^ -(z & 1)
        elif t in (1, 2):
            out[fid] = t == 1
        elif t == 3:
            i += 1
        elif t == 7:
            i += 8
        elif t == 8:
            n, i = uvarint(b, i)
            i += n
        elif t == 12:
            out[fid], i = skip_struct(b, i)
        elif t in (9, 10):
            h2 = b[i]
            i += 1
            n = h2 >> 4
            et = h2 & 0x0F
            if n == 15:
                n, i = uvarint(b, i)
            for _ in range(n):
                if et == 12:
                    _, i = skip_struct(b, i)
                elif et in (5, 6, 4):
                    _, i = uvarint(b, i)
                elif et == 8:
                    m, i = uvarint(b, i)
                    i += m
                else:
                    raise ValueError("list elem type %d" % et)
        else:
            raise ValueError("type %d" % t)


def runs(stream, bw, n):
    i = 0
    got = 0
    nr_rle = nr_bp = 0
    lens = []
    while got < n and i < len(stream):
        h, i = uvarint(stream, i)
        if h & 1:
            g = h >> 1
            i += g * bw
            got += g * 8
            nr_bp += 1
            lens.append(g * 8)
        else:
            c = h >> 1
            i += (bw + 7) // 8
            got += c
            nr_rle += 1
            lens.append(c)
    return nr_rle, nr_bp, lens


def main():
    import pyarrow as pa
    import pyarrow.parquet as pq
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    path = "/tmp/page_runs.parquet"
    rng = np.random.default_rng(2)
    schema = pa.schema([pa.field("v", pa.int32(), nullable=False)])
    bws = list(range(1, 21))
    with pq.ParquetWriter(path, schema, compression="none", use_dictionary=True, data_page_version="1.0",
                          dictionary_pagesize_limit=1 << 30) as w:
        for bw in bws:
            K = 1 << bw
            dvals = rng.permutation(K).astype(np.int32)
            idx = rng.integers(0, K, rows)
            w.write_table(pa.table({"v": pa.array(dvals[idx])}, schema=schema), row_group_size=rows)
    b = open(path, "rb").read()
    md = pq.ParquetFile(path).metadata
    for rg in range(md.num_row_groups):
        cc = md.row_group(rg).column(0)
        i = cc.dictionary_page_offset if cc.has_dictionary_page else cc.data_page_offset
        end = i + cc.total_compressed_size
        stats = []
        while i < end:
            ph, j = skip_struct(b, i)
            size = ph[3]
            if ph[1] == 0:  # DATA_PAGE
                n = ph[5][1]
                body = b[j:j + size]
                pbw = body[0]
                r, p, lens = runs(body[1:], pbw, n)
                stats.append((n, len(body), pbw, r, p, np.mean(lens)))
            i = j + size
        s = np.array(stats, dtype=float)
        print("bw %2d pages %3d  bytes/page %7.0f  runs/page rle %7.1f bp %6.1f  mean run len %7.1f" %
              (bws[rg], len(s), s[:, 1].mean(), s[:, 3].mean(), s[:, 4].mean(), s[:, 5].mean()))


if __name__ == "__main__":
    main()
