"""Diagnostic: where k_decode<2>'s steps spend their cycles, per column, from
the phase stamps of the libpqgpu_decdiag.so build (make -C
parquet-go_amd/csrc decdiag): per page the shader cycles of each step phase
(levels / counts / scans, the key stream, key checks + dictionary entries,
string outputs, validity bitmaps), summed over the page's steps.

usage: python tools/diag_decode.py CONFIG [ROWS] [RG_ROWS]"""
import ctypes
import os
import sys

os.environ["PQGPU_LIB"] = "libpqgpu_decdiag.so"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-go_amd"), os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402

import pqgpu  # noqa: E402
import synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
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
for fn in ("pqg_diag_stamps", "pqg_diag_stamps2"):
    getattr(L, fn).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
L.pqg_diag_page_cols.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
npg = b.stats()["pages"]
pc = np.zeros(npg, np.int32)
L.pqg_diag_page_cols(b._h, pc.ctypes.data, npg)
ph = np.zeros(8 * (npg + 1) + 256, np.uint64)
L.pqg_diag_stamps2(b._h, ph.ctypes.data, ph.size)
pg = np.zeros(4 * (npg + 1), np.uint64)
L.pqg_diag_stamps(b._h, pg.ctypes.data, pg.size)
ph = ph[:8 * npg].reshape(npg, 8).astype(np.float64)
pg = pg[:4 * npg].reshape(npg, 4).astype(np.float64)
names = [c["name"] for c in r.Columns()]
steps = ["levels", "keys", "dict", "outputs", "bitmaps"]
m_all = ph[:, 7] > 0
print("%s: %d k_decode<1>/<2>/<4>/<5> pages; longest wave %.0f kcycles" % (cfg, m_all.sum(), pg[:, 1].max() / 1e3))
print("%-16s %6s %9s %9s | %s | %s" % ("column", "pages", "values", "kcyc/pg", " ".join("%8s" % s for s in steps), "cyc/256"))
for ci in sorted(set((pc >> 8).tolist())):
    m = ((pc >> 8) == ci) & m_all
    if not m.any():
        continue
    tot = ph[m, :5].sum(0)
    nvals = pg[m, 2].sum()
    print("%-16s %6d %9d %9.0f | %s | %6.0f" % (names[ci][:16], m.sum(), nvals, pg[m, 0].mean() / 1e3,
                                               " ".join("%7.1f%%" % (100 * x / max(tot.sum(), 1)) for x in tot),
                                               tot.sum() / max(nvals / 256, 1)))
