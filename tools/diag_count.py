"""Diagnostic: where k_prepare's count path (lists / strings) spends its time,
per column, from the s_memrealtime stamps of libpqgpu_diag.so
(make -C parquet-go_amd/csrc diag).

usage: python tools/diag_count.py CONFIG [ROWS] [RG_ROWS]
Per page: start -> levels (layout, value init), rep-level pass, def-level
pass, strings (length walk / dictionary lengths); us, 100 MHz stamps."""
import ctypes
import os
import sys

os.environ["PQGPU_LIB"] = "libpqgpu_diag.so"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-go_amd"), os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402

import pqgpu  # noqa: E402
import synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
rows = int(sys.argv[2]) if len(sys.argv) > 2 else synth.DEFAULTS[cfg][0]
rgr = int(sys.argv[3]) if len(sys.argv) > 3 else synth.DEFAULTS[cfg][1]
path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "pqgpu_bench_%s_%d_%d_0.parquet" % (cfg, rows, rgr))
if not os.path.exists(path):
    synth.make(cfg, path, rows, rgr)
r = pqgpu.FileReader(path)
b = r.batch()
for _ in range(2):
    b.decode()
b.sync()
L = pqgpu.lib()
L.pqg_diag_reset.argtypes = [ctypes.c_void_p]
L.pqg_diag_reset(b._h)
b.decode()
b.sync()
L.pqg_diag_stamps2.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
L.pqg_diag_page_cols.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
npg = b.stats()["pages"]
pc = np.zeros(npg, np.int32)
L.pqg_diag_page_cols(b._h, pc.ctypes.data, npg)
st = np.zeros(16 * (npg + 1) + 256, np.uint64)
L.pqg_diag_stamps2(b._h, st.ctypes.data, st.size)
s = st[:8 * npg].reshape(npg, 8).astype(np.int64)
names = [c["name"] for c in r.Columns()]
m = (s[:, 4] >= 100) & (s[:, 0] > 0) & (s[:, 7] > 0)
t0 = s[m, 0].min() if m.any() else 0
print("%s: %d pages on the count path" % (cfg, m.sum()))
print("%-12s %5s %7s | %8s %8s %8s %8s | %8s %8s" % ("column", "pages", "values", "init", "rep", "def", "strings", "start", "end"))
for ci in sorted(set((pc[m] >> 8).tolist())):
    k = m & ((pc >> 8) == ci)
    q = s[k]
    parts = [(q[:, 1] - q[:, 0]), (q[:, 2] - q[:, 1]), (q[:, 6] - q[:, 2]), (q[:, 7] - q[:, 6])]
    print("%-12s %5d %7d | %s | %8.1f %8.1f   (median us; enc %s)" % (
        names[ci][:12], k.sum(), np.median(q[:, 3]), " ".join("%8.1f" % (np.median(x) / 100) for x in parts),
        np.median(q[:, 0] - t0) / 100, np.max(q[:, 7] - t0) / 100, sorted(set((q[:, 4] - 100).tolist()))))
