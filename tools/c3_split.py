"""Analysis: C3's decode phase per column — files holding only the DELTA
timestamp column or only the nullable DOUBLE column (tools/synth.py c3's
distributions), decode-phase time and kernel timeline of each."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-go_amd"), os.path.join(ROOT, "tools")]
import pyarrow as pa  # noqa: E402
import pyarrow.parquet as pq  # noqa: E402

import pqgpu  # noqa: E402

rows, rgr = 50_000_000, 1 << 20
rng = np.random.default_rng(3)
for col in ("ts", "x"):
    path = "/tmp/c3_%s.parquet" % col
    if not os.path.exists(path):
        if col == "ts":
            schema = pa.schema([pa.field("ts", pa.int64(), nullable=False)])
            kw = dict(column_encoding={"ts": "DELTA_BINARY_PACKED"})
        else:
            schema = pa.schema([pa.field("x", pa.float64())])
            kw = dict(column_encoding={"x": "PLAIN"})
        last = 1_600_000_000_000_000
        with pq.ParquetWriter(path, schema, compression="snappy", data_page_version="2.0", use_dictionary=False,
                              **kw) as w:
            for i in range(0, rows, rgr):
                n = min(rgr, rows - i)
                if col == "ts":
                    step = np.where(rng.random(n) < 0.95, 1000, rng.integers(0, 4096, n))
                    ts = last + np.cumsum(step)
                    last = int(ts[-1])
                    t = pa.table({"ts": pa.array(ts.astype(np.int64))}, schema=schema)
                else:
                    t = pa.table({"x": pa.array(np.round(rng.standard_normal(n), 2), mask=rng.random(n) < 0.1)},
                                 schema=schema)
                w.write_table(t, row_group_size=n)
    os.environ["PQG_SEGMENT_TIMES"] = "1"
    r = pqgpu.FileReader(path)
    b = r.batch()
    del os.environ["PQG_SEGMENT_TIMES"]
    for _ in range(3):
        b.decode()
    b.sync()
    b.kernel_times()
    for _ in range(5):
        b.decode()
    b.sync()
    print(col, {k: round(v, 3) for k, v in b.kernel_times().items()}, flush=True)
    b.close()
