"""Diagnostic: where k_snappy's time goes, per column, from the phase stamps
of the libpqgpu_snapdiag.so build (make -C parquet-go_amd/csrc snapdiag).

usage: python tools/diag_snappy.py CONFIG [ROWS] [RG_ROWS]
Per page the build accumulates shader cycles (s_memtime) of each step of a
short-token batch (window, chain, decode, far copies, tables, byte passes,
flush) and counts batches; per column this prints the sums and per-batch
means, plus page start / end spread."""
import ctypes
import os
import sys

os.environ["PQGPU_LIB"] = "libpqgpu_snapdiag.so"
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
L.pqg_diag_reset(b._h)  # the stamps below are of exactly one decode
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
pg = pg[:4 * npg].reshape(npg, 4).astype(np.float64)  # per page: wave-cycles (all segments), longest wave, bytes out, in
names = [c["name"] for c in r.Columns()]
print("%s: %d pages; longest wave %.0f kcycles" % (cfg, npg, pg[:, 1].max() / 1e3))
# k_snappy's batch steps (PQ_SNAP_STAMPS marks -1..6); k_snappy_wg's with PQG_SNAPPY_WG=1
steps = (["window", "chain", "decode", "table", "longlit", "bytes", "flush"] if os.environ.get("PQG_SNAPPY_WG") == "1"
         else ["tables", "chain", "check", "far", "short", "dep", "flush"])
print("%-16s %6s %8s %8s %9s | %s | %s" % ("column", "pages", "batches", "MB out", "kcyc/pg", " ".join("%7s" % s for s in steps),
                                           "cyc/batch"))
for ci in sorted(set((pc >> 8).tolist())):
    m = (pc >> 8) == ci
    m &= pg[:, 2] > 0
    if not m.any():
        continue
    nb = ph[m, 7].sum()
    tot = ph[m, :7].sum(0)
    life = pg[m, 1]
    print("%-16s %6d %8d %8.1f %9.0f | %s | %6.0f" % (
        names[ci][:16], m.sum(), nb, pg[m, 2].sum() / 1e6, pg[m, 0].mean() / 1e3,
        " ".join("%6.1f%%" % (100 * x / max(tot.sum(), 1)) for x in tot), tot.sum() / max(nb, 1)))
    print("%16s longest wave kcyc: median %.0f p90 %.0f max %.0f; batches/page max %d" % (
        "", np.median(life) / 1e3, np.percentile(life, 90) / 1e3, life.max() / 1e3, ph[m, 7].max()))

# k_snappy_walk (pages longer than one segment): per page, cycles of the walk
# and its parts, chunks, path rounds and pass-1 steps (after the k_snappy
# stamps and 256 run-walk stamps in the same buffer)
full = np.zeros(16 * (npg + 1) + 256, np.uint64)
L.pqg_diag_stamps2(b._h, full.ctypes.data, full.size)
w = full[8 * (npg + 1) + 256:][:8 * npg].reshape(npg, 8).astype(np.float64)
walked = np.nonzero(w[:, 0] > 0)[0]
print("\nk_snappy_walk: %d pages" % walked.size)
print("%-16s %4s %7s %7s %6s | %7s %7s %7s %7s | %6s %7s" % ("column", "kind", "KB in", "kcyc", "GHz", "pass1", "pass3", "bound", "hops",
                                                           "rounds", "p1steps"))
for p in walked[np.argsort(-w[walked, 0])][:40]:
    print("%-16s %4d %7.0f %7.0f %6.2f | %6.1f%% %6.1f%% %6.1f%% %6.1f%% | %6d %7d" % (
        names[pc[p] >> 8][:16], pc[p] & 255, pg[p, 3] / 1e3 if pg[p, 3] else 0, w[p, 0] / 1e3, w[p, 0] / max(w[p, 1], 1) / 10,
        100 * w[p, 2] / w[p, 0], 100 * w[p, 3] / w[p, 0], 100 * w[p, 4] / w[p, 0], 100 * w[p, 7] / w[p, 0], w[p, 5], w[p, 6]))
