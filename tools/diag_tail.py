"""Diagnostic: k_expand_mix block timeline (libpqgpu_diag.so): when LDS-group and
L1/L2 blocks run and end.  usage: python tools/diag_tail.py [BW] [ROWS]"""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-go_amd"), ROOT]
import pqgpu  # noqa: E402
pqgpu._LIB_PATH = os.path.join(ROOT, "parquet-go_amd", "libpqgpu_diag.so")
import bench  # noqa: E402
bw = int(sys.argv[1]) if len(sys.argv) > 1 else 0
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000_000
path = "/tmp/diag_bw%d_%d.parquet" % (bw, rows)
if not os.path.exists(path):
    bench.make_file(path, rows, 1 << 20, fixed_bw=bw)
b = pqgpu.FileReader(path).batch()
for _ in range(3):
    b.decode()
b.sync()
L = pqgpu.lib()
L.pqg_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
n = 8 * 4 * 400000
out = np.zeros(n, np.uint64)
got = L.pqg_diag_stamps(b._h, out.ctypes.data, n)
s = out[:got].reshape(-1, 8).astype(np.int64)
s = s[(s[:, 0] > 0) & (s[:, 7] > 0)]
t0 = s[:, 0].min()
st, en, kind = (s[:, 0] - t0) / 100.0, (s[:, 7] - t0) / 100.0, s[:, 6]
print("waves", len(s), "span us %.1f" % en.max())
for k, nm in ((1, "LDS-group"), (2, "L1/L2")):
    m = kind == k
    if m.sum():
        life = en[m] - st[m]
        print("%-9s waves %6d  start med %6.1f  end med %6.1f  end max %6.1f  life med %6.1f p90 %6.1f" % (
            nm, m.sum(), np.median(st[m]), np.median(en[m]), en[m].max(), np.median(life), np.percentile(life, 90)))
edges = np.linspace(0, en.max(), 21)
for k, nm in ((1, "LDS"), (2, "L2 ")):
    m = kind == k
    act = [int(((st[m] <= e) & (en[m] > e)).sum()) for e in edges]
    print(nm, "resident waves over time:", " ".join("%d" % x for x in act))
names = ["desc", "win+span", "stage", "keys+gath", "stores"]
for k, nm in ((1, "LDS-group"), (2, "L1/L2")):
    m = (kind == k) & (s[:, 5] > 0)
    row = []
    for i, n_ in enumerate(names):
        d = (s[m, i + 1] - s[m, i]) / 100.0
        d = d[(s[m, i + 1] > 0) & (s[m, i] > 0)]
        row.append("%s %.2f" % (n_, np.median(d) if len(d) else -1))
    print(nm, "last job phases (median us):", ", ".join(row))
