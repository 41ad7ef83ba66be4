"""Summarise rocprofv3 --pmc passes (tools/pmc.sh output): per kernel, mean counter value per dispatch."""
import collections
import csv
import glob
import sys

tag = sys.argv[1]
want = sys.argv[2:] or None
acc = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in sorted(glob.glob("%s_pmc*/**/*counter_collection.csv" % tag, recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, cs in acc.items():
    if want and not any(w in k for w in want):
        continue
    print("== %s  (median dispatch %.1f us)" % (k, sorted(dur[k])[len(dur[k]) // 2]))
    for c, v in sorted(cs.items()):
        print("   %-22s %16.0f" % (c, sum(v) / len(v)))
