"""Per-kernel dispatch durations of the last decode in a rocprofv3 kernel trace."""
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# last decode: from the last k_snappy dispatch on
last = max(i for i, r in enumerate(rows) if "k_snappy" in r["Kernel_Name"])
t0 = int(rows[last]["Start_Timestamp"])
for r in rows[last:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    print("%-34s start %8.1f us  dur %8.1f us  grid %s lds %s" % (name[:34], (s - t0) / 1e3, (e - s) / 1e3,
          r.get("Grid_Size", r.get("Grid_Size_X", "?")), r.get("LDS_Block_Size", r.get("Lds_Size", "?"))))
