import sys, io, numpy as np
sys.path.insert(0,'parquet-go_amd'); sys.path.insert(0,'oracle')
import pyarrow as pa, pyarrow.parquet as pq, pqgpu, oracle
rng = np.random.default_rng(11)
n = 120000
ts = (1_600_000_000_000_000 + np.cumsum(np.where(rng.random(n) < 0.95, 1000, rng.integers(0, 4096, n)))).astype(np.int64)
t = pa.table({"ts": pa.array(ts), "x": pa.array(np.round(rng.standard_normal(n), 2), mask=rng.random(n) < 0.1),
    "i": pa.array(rng.integers(-5, 5, n).astype(np.int32), mask=rng.random(n) < 0.5),
    "s": pa.array(["k%d" % v if v % 7 else None for v in rng.integers(0, 500, n)])})
for ver in ("1.0", "2.0"):
    buf = io.BytesIO(); pq.write_table(t, buf, compression="snappy", data_page_version=ver, use_dictionary=["s", "i"], column_encoding={"ts": "DELTA_BINARY_PACKED", "x": "PLAIN"}, row_group_size=50000)
    data = buf.getvalue()
    o = oracle.File(data)
    for leaf in range(4):
        try: o.decode(leaf); print(ver, leaf, 'oracle ok')
        except oracle.OracleError as e: print(ver, leaf, 'oracle err', e)
        r = pqgpu.FileReader(data)
        try:
            b = r.batch(0, None, [leaf]); b.decode(); rc = b.sync(raise_on_error=False)
            print(ver, leaf, 'gpu rc', rc, pqgpu.last_error())
        except Exception as e: print(ver, leaf, 'gpu exc', e)
