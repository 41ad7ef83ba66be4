"""Diagnostic: per-wave phase times of k_expand from s_memrealtime stamps
(libpqgpu_diag.so built with `make -C parquet-go_amd/csrc diag`).
usage: python tools/diag_stamps.py BW [ROWS]   (BW 0 = the bench's 1..20 sweep)"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parquet-go_amd"))
sys.path.insert(0, ROOT)
import pqgpu  # noqa: E402

pqgpu._LIB_PATH = os.path.join(ROOT, "parquet-go_amd", "libpqgpu_diag.so")
import bench  # noqa: E402

bw = int(sys.argv[1])
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 20_000_000
path = "/tmp/diag_bw%d_%d.parquet" % (bw, rows)
if not os.path.exists(path):
    bench.make_file(path, rows, 1 << 20, fixed_bw=bw)
r = pqgpu.FileReader(path)
b = r.batch()
for _ in range(3):
    b.decode()
b.sync()
print(b.kernel_times())
L = pqgpu.lib()
L.pqg_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
n = 8 * 4 * 200000
out = np.zeros(n, np.uint64)
got = L.pqg_diag_stamps(b._h, out.ctypes.data, n)
s = out[:got].reshape(-1, 8).astype(np.int64)
s = s[s[:, 0] > 0]
t0 = s[:, 0].min()
print("waves", len(s), "kernel span us %.1f" % ((s[:, 5].max() - t0) / 100.0))
names = ["desc", "win+span", "stage", "half0", "rest"]
for k, nm in enumerate(names):
    d = s[:, k + 1] - s[:, k]
    d = d[(s[:, k + 1] > 0) & (s[:, k] > 0)]
    if len(d):
        print("%-9s n %6d  median %7.2f us  p90 %7.2f  max %7.2f" % (nm, len(d), np.median(d) / 100, np.percentile(d, 90) / 100, d.max() / 100))
full = s[s[:, 5] > 0]
life = (full[:, 5] - full[:, 0]) / 100.0
print("lifetime median %.2f us p90 %.2f" % (np.median(life), np.percentile(life, 90)))
st = (s[:, 0] - t0) / 100.0
h, e = np.histogram(st, bins=20)
print("wave starts over time (us):", " ".join("%d" % x for x in h), "edges", "%.1f..%.1f" % (e[0], e[-1]))
en = (full[:, 5] - t0) / 100.0
h, e = np.histogram(en, bins=20)
print("wave ends over time (us):  ", " ".join("%d" % x for x in h))
