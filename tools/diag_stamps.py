"""Diagnostic: per-workgroup phase times of k_decode_dict_wg from s_memtime stamps
(libpqgpu_diag.so built with `make -C parquet-go_amd/csrc diag`)."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parquet-go_amd")); sys.path.insert(0, ROOT)
import pqgpu
pqgpu._LIB_PATH = os.path.join(ROOT, "parquet-go_amd", "libpqgpu_diag.so")
import bench
path = "/tmp/diag_bw%s.parquet" % sys.argv[1]
if not os.path.exists(path):
    bench.make_file(path, 20_000_000, 1 << 20, fixed_bw=int(sys.argv[1]))
r = pqgpu.FileReader(path)
b = r.batch()
for _ in range(3):
    b.decode()
b.sync()
print(b.kernel_times())
L = pqgpu.lib()
L.pqg_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
n = 8 * 1100
out = np.zeros(n, np.uint64)
got = L.pqg_diag_stamps(b._h, out.ctypes.data, n)
s = out[:got].reshape(-1, 8).astype(np.int64)
s = s[s[:, 0] > 0]
t0 = s[:, 0].min()
print("workgroups", len(s))
for name, i, j in (("stage", 0, 1), ("walk", 1, 2), ("steps", 2, 3), ("total", 0, 3)):
    d = s[:, j] - s[:, i]
    print("%-6s median %8.0f  p90 %8.0f  max %8.0f cycles(100MHz ticks?)" % (name, np.median(d), np.percentile(d, 90), d.max()))
print("span start->last end", (s[:, 3].max() - t0), "first start spread", np.percentile(s[:, 0] - t0, [50, 90, 100]))
