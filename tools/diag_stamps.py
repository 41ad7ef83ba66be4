"""Diagnostic: per-job phase times of k_expand_mix from s_memrealtime stamps
(libpqgpu_diag.so built with `make -C parquet-go_amd/csrc diag`).

Per wave the stamps accumulate, over the jobs it ran, the time from one
stamp to the next (pq_kernels.hip STAMP): 'rec' = to the job's start (the
record load, the gap after the previous job; for a wave's first job also
the dictionary copy), 'issue' = run window + key staging issued, 'wait' =
those loads landed, 'keys+gath' = key extraction and the gathers, 'store'.

usage: python tools/diag_stamps.py BW [ROWS]   (BW 0 = the bench's 1..20 sweep)"""
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
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 20_000_000
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
t0 = s[:, 0].min()
jobs = s[:, 7]
print("bw %d: waves with jobs %d, jobs %d (median %d a wave), kernel span %.1f us" %
      (bw, len(s), jobs.sum(), np.median(jobs), (s[:, 6].max() - t0) / 100.0))
names = ["rec", "issue", "wait", "keys+gath", "store"]
tot = s[:, 1:6].sum(axis=1)
for k, nm in enumerate(names):
    per = s[:, k + 1] / jobs / 100.0
    print("%-10s per job median %7.2f us  p90 %7.2f   share %5.1f%%" %
          (nm, np.median(per), np.percentile(per, 90), 100.0 * s[:, k + 1].sum() / max(1, tot.sum())))
life = (s[:, 6] - s[:, 0]) / 100.0
print("wave life median %.1f us p90 %.1f; per job median %.2f us" %
      (np.median(life), np.percentile(life, 90), np.median(tot / jobs / 100.0)))
