"""Diagnostic: the kernel timeline of one decode step (rocprofv3 kernel trace
of a short `bench.py --child` run): per launch, its stream queue, start and
end relative to the step's first launch, and duration.

usage: python tools/timeline.py CONFIG [extra bench args]   (on the GPU box)
       python tools/timeline.py --csv KERNEL_TRACE.csv [NAME]  (a kept trace, e.g.
       profiles/r03/*/rocprof_kernel_trace_c5.csv from bench.py's own child run)
"""
import csv
import glob
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
if cfg == "--csv":
    rows = list(csv.DictReader(open(sys.argv[2])))
    cfg = sys.argv[3] if len(sys.argv) > 3 else os.path.basename(sys.argv[2])
else:
  with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
    cmd = ["timeout", "-s", "KILL", "150", "rocprofv3", "--kernel-trace", "--output-format", "csv", "-d", td, "-o", "run",
           "--", sys.executable, os.path.join(ROOT, "bench.py"), "--child", "--steps", "3", "--warmup", "1",
           "--config", cfg] + sys.argv[2:]
    subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, check=True, timeout=180)
    rows = []
    for f in glob.glob(os.path.join(td, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
name = lambda r: r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pq::", "").strip()
# a decode step ends with k_level_check (k_reset runs only when a step has
# bitmaps to zero or its statuses were not planned by the previous step)
ends = [i for i, r in enumerate(rows) if name(r) == "k_level_check"]
if len(ends) < 2:
    sys.exit("fewer than two decode steps in the trace")
step = rows[ends[-2] + 1:ends[-1] + 1]  # the last complete step
t0 = int(step[0]["Start_Timestamp"])
end = max(int(r["End_Timestamp"]) for r in step)
print("%s: step %.3f ms (first launch to last end), %d launches" % (cfg, (end - t0) / 1e6, len(step)))
print("%-22s %6s %9s %9s %9s %7s" % ("kernel", "queue", "start us", "end us", "dur us", "grid"))
for r in step:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print("%-22s %6s %9.1f %9.1f %9.1f %7s" % (name(r)[:22], r.get("Queue_Id", r.get("Stream_Id", "")), s / 1e3, e / 1e3,
                                             (e - s) / 1e3, r.get("Grid_Size", r.get("Grid_Size_X", ""))))
