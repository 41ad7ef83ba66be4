import sys, time, os
sys.path[:0]=['parquet-go_amd','.']
import pqgpu, bench
path="/tmp/pqgpu_bench_c2_100000000_1048576_0.parquet"
if not os.path.exists(path): bench.make_file(path, 100000000, 1<<20)
t=time.perf_counter(); r=pqgpu.FileReader(path); print("open ms", (time.perf_counter()-t)*1e3, flush=True)
for k in range(2):
    t=time.perf_counter(); b=r.batch(); print("create ms", (time.perf_counter()-t)*1e3, flush=True); b.close()
