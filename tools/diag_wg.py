"""Diagnostic: per-job phase times of k_expand_wg from s_memrealtime stamps
(libpqgpu_diag.so built with `make -C parquet-go_amd/csrc diag`), on a
single-bit-width C2-like file whose chunks all take k_expand_wg.

Per wave the stamps accumulate, over its jobs (pq_kernels.hip WSTAMP):
'prologue' = the group descriptor, first descriptors, dictionary copy and
barrier (once a wave), 'desc' = the next job's descriptor / window issue and
this job's descriptor unpack, 'keys' = key loads landed and extracted,
'gather' = LDS gathers (sliced: every slice's copy, barriers and gathers),
'store' = stores issued.

usage: python tools/diag_wg.py BW [ROWS]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parquet-go_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
os.environ["PQGPU_LIB"] = "libpqgpu_diag.so"
import pqgpu  # noqa: E402
import synth  # noqa: E402

bw = int(sys.argv[1])
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 25165824
path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "diag_bw%d_%d.parquet" % (bw, rows))
if not os.path.exists(path):
    synth.make("c2", path, rows, 1 << 20, fixed_bw=bw)
r = pqgpu.FileReader(path)
b = r.batch()
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
if not len(s):
    print("bw %d: no k_expand_wg stamps (no chunk took it?)" % bw)
    sys.exit(0)
t0 = s[:, 0].min()
jobs = s[:, 7]
print("bw %d: waves with jobs %d, jobs %d (median %d a wave), kernel span %.1f us" %
      (bw, len(s), jobs.sum(), np.median(jobs), (s[:, 6].max() - t0) / 100.0))
print("prologue per wave median %.2f us p90 %.2f" % (np.median(s[:, 1]) / 100.0, np.percentile(s[:, 1], 90) / 100.0))
names = ["desc", "keys", "gather", "store"]
tot = s[:, 2:6].sum(axis=1)
for k, nm in enumerate(names):
    per = s[:, k + 2] / jobs / 100.0
    print("%-8s per job median %7.2f us  p90 %7.2f   share %5.1f%%" %
          (nm, np.median(per), np.percentile(per, 90), 100.0 * s[:, k + 2].sum() / max(1, tot.sum())))
life = (s[:, 6] - s[:, 0]) / 100.0
start = (s[:, 0] - t0) / 100.0
print("wave start median %.1f us p90 %.1f max %.1f; life median %.1f us p90 %.1f; per job median %.2f us" %
      (np.median(start), np.percentile(start, 90), start.max(), np.median(life), np.percentile(life, 90),
       np.median(tot / jobs / 100.0)))
