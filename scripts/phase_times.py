#!/usr/bin/env python3
"""Per-phase GPU BVH build times from a rocprofv3 kernel trace of
scripts/prof_bvh_build.py (last build's 17 vx_main dispatches)."""
import csv
import sys

PH = ["bounds", "morton"] + [f"{p}{i}" for i in range(4) for p in ("hist", "scan", "scatter")] + \
     ["tree", "boxes", "emit"]
rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Kernel_Name"] == "vx_main_bvh_build"]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = rows[-17:]
for name, r in zip(PH, last):
    print(f"{name:10s} {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000:9.1f} us")
