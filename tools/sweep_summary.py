"""Summarise bench JSON lines of an analysis sweep: decode-phase time and rate.
usage: python tools/sweep_summary.py gpurun_out/TAG_*.json"""
import json
import sys

for f in sys.argv[1:]:
    try:
        line = [l for l in open(f) if l.startswith("{")][-1]
        d = json.loads(line)
    except Exception:
        print("%-40s (no bench line)" % f)
        continue
    p = d["config"].get("phase_ms", {})
    r = d["config"]["rows_per_gpu"]
    dec = p.get("k_decode+k_expand") or 0
    print("%-40s step %.4f ms  prepare %.4f  decode %.4f  %s Gval/s" %
          (f, d["ms_per_step"], p.get("k_prepare", 0), dec, "%.0f" % (r / dec / 1e6) if dec else "-"))
