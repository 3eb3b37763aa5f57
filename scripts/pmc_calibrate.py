#!/usr/bin/env python3
"""Reduce scripts/pmc_calibrate.sh: per probe kernel and size, the mean
FETCH_SIZE / WRITE_SIZE per dispatch (KB, first dispatch of each kernel
skipped: cold caches) against the bytes it touched -> bytes per counted KB.
pmc_profile.py applies the factors of the access forms each RT kernel uses.
Usage: pmc_calibrate.py <tag_dir> <out.json>"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

PROBES = {"probe_store4": ("WRITE_SIZE", "4-B/lane buffer_store_dword (framebuffer store)"),
          "probe_store16": ("WRITE_SIZE", "16-B/lane buffer_store_dwordx4"),
          "probe_load16": ("FETCH_SIZE", "16-B/lane buffer_load_dwordx4"),
          "probe_sload64": ("FETCH_SIZE", "64-B s_load_dwordx16 records")}


def main():
    tag, out = sys.argv[1:3]
    res = {"source": "scripts/pmc_calibrate.sh (skybox_rt_amd/csrc/tools/pmc_probe.hip)", "probes": {}}
    for d in sorted(glob.glob(os.path.join(tag, "cal_*"))):
        if not os.path.isdir(d):
            continue
        _, mib, ctr = os.path.basename(d).split("_", 2)
        known = int(mib) << 20
        per = defaultdict(lambda: defaultdict(float))
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if row["Counter_Name"] == ctr:
                        per[row["Kernel_Name"]][int(row["Dispatch_Id"])] += float(row["Counter_Value"])
        for k, (c, what) in PROBES.items():
            if c != ctr or k not in per:
                continue
            vals = [v for _, v in sorted(per[k].items())][1:]
            kb = sum(vals) / len(vals)
            res["probes"][f"{k}_{mib}MiB"] = {
                "counter": ctr, "form": what, "bytes": known, "counter_kb_per_dispatch": round(kb, 1),
                "bytes_per_counted_byte": round(known / (kb * 1024), 4) if kb else None,
                "dispatches": len(vals)}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
