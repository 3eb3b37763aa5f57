#!/usr/bin/env python3
"""Reduce scripts/pmc_busy.sh's passes: per-launch averages of every counter
over the workload image's own dispatches (vx_main_<image>), and busy
fractions against the GPU's active cycles (GRBM_GUI_ACTIVE) per instance.
Usage: pmc_busy.py <dir> <mode>"""
import csv
import glob
import json
import os
import sys

IMAGE = {"shadow": "vx_main_rt_kernel", "path": "vx_main_pt_kernel", "flat": "vx_main_rt_flat",
         "bvh": "vx_main_rt_bvh"}


def main():
    d, mode = sys.argv[1], sys.argv[2]
    k = IMAGE[mode]
    sums, disp = {}, {}
    for f in glob.glob(os.path.join(d, f"{mode}_*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"] != k:
                continue
            c = r["Counter_Name"]
            sums[c] = sums.get(c, 0.0) + float(r["Counter_Value"])
            disp.setdefault(c, set()).add((f, r["Dispatch_Id"]))
    avg = {c: sums[c] / len(disp[c]) for c in sums}
    out = {"kernel": k, "per_launch": {c: round(v, 1) for c, v in sorted(avg.items())}}
    # the launch's length in shader-engine cycles: SQ_BUSY_CYCLES is summed
    # over the 32 shader engines (8 XCDs x 4); the TA / TD / TCP counters
    # over the 256 CUs' instances
    sq = avg.get("SQ_BUSY_CYCLES")
    if sq:
        ses, cus = 32, 256
        cyc = sq / ses
        out["launch_cycles_per_se"] = round(cyc, 1)
        fr = {}
        for c in ("TA_TA_BUSY_sum", "TD_TD_BUSY_sum", "TCP_TCP_TA_DATA_STALL_CYCLES_sum",
                  "TCP_PENDING_STALL_CYCLES_sum", "TCP_TCR_TCP_STALL_CYCLES_sum"):
            if c in avg:
                fr[c] = round(avg[c] / (cyc * cus), 4)
        out["busy_frac_per_instance"] = fr
    if avg.get("SQC_DCACHE_REQ"):
        out["sqc_dcache_hit_rate"] = round(avg.get("SQC_DCACHE_HITS", 0.0) / avg["SQC_DCACHE_REQ"], 4)
    if avg.get("SQ_WAVE_CYCLES"):
        out["sq_frac_of_wave_cycles"] = {c: round(avg[c] / avg["SQ_WAVE_CYCLES"], 4) for c in avg
                                         if c.startswith("SQ_ACTIVE_INST") or c.startswith("SQ_WAIT")
                                         or c.startswith("SQ_INST_CYCLES")}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
