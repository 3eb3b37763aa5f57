#!/usr/bin/env python3
"""Reduce two rocprofv3 --pmc passes (FETCH_SIZE; WRITE_SIZE, run separately:
FETCH_SIZE takes 3 of the 4 TCC slots, WRITE_SIZE 2) over scripts/prof_rt.py
to HBM bytes per launch of vx_main, and write the JSON bench.py reports as
roofline.traffic.

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE counts
64 B per 128-B memory-side read request, i.e. exactly half of the bytes of a
wide coalesced read, so the read side is doubled; WRITE_SIZE is taken as is.
Both are in KB.  Usage: pmc_traffic.py <fetch_dir> <write_dir> <out.json>
<width> <height> <shadows 0|1> <kernel .co> [mode: shadow|path|flat]"""
import csv
import glob
import hashlib
import json
import os
import sys


def per_dispatch(d, counter):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Kernel_Name"] != "vx_main" or row["Counter_Name"] != counter:
                    continue
                vals[row["Dispatch_Id"]] = vals.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    fdir, wdir, out, w, h, sh, co = sys.argv[1:8]
    mode = sys.argv[8] if len(sys.argv) > 8 else "shadow"
    f = per_dispatch(fdir, "FETCH_SIZE")
    wr = per_dispatch(wdir, "WRITE_SIZE")
    if not f or not wr:
        sys.exit("no vx_main dispatches with FETCH_SIZE / WRITE_SIZE")
    f_kb, w_kb = sum(f) / len(f), sum(wr) / len(wr)
    res = {
        "kernel": "vx_main", "mode": mode, "width": int(w), "height": int(h),
        "shadows": bool(int(sh)),
        "kernel_md5": hashlib.md5(open(co, "rb").read()).hexdigest(),
        "dispatches": [len(f), len(wr)],
        "fetch_size_kb": round(f_kb, 1), "write_size_kb": round(w_kb, 1),
        "correction": "read bytes = 2 x FETCH_SIZE x 1024 (gfx950 half-count), write = WRITE_SIZE x 1024",
        "traffic_bytes": int(2 * f_kb * 1024 + w_kb * 1024),
    }
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
