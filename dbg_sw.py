import sys, os, io
sys.path[:0] = ["tests", "oracle", "parquet-go_amd"]
import numpy as np
import conftest, oracle, pqgpu
import test_gpu_parity as T
rng = np.random.default_rng(61)
t = T._plain_string_cases(rng)["blob_nullable"]
data = T._pq_bytes(t, compression="none", use_dictionary=False, data_page_size=1 << 20, data_page_version="1.0", row_group_size=40000)
o = oracle.File(data)
exp = o.decode(0)
for levels in (True, False):
    rc, got, cols = T.gpu_decode_all(data, levels)
    g = got[0]
    for k in ("values", "str_offsets", "validity", "def"):
        a, b = g[k], exp[k]
        if a.size != b.size or not np.array_equal(a, b):
            bad = np.nonzero(a[:min(a.size,b.size)] != b[:min(a.size,b.size)])[0]
            print(levels, k, a.size, b.size, "first bad", bad[:5], a[bad[:5]] if bad.size else None, b[bad[:5]] if bad.size else None)
        else:
            print(levels, k, "ok", a.size)
    so = g["str_offsets"]; eo = exp["str_offsets"]
    print("offs", so[:12], eo[:12])
