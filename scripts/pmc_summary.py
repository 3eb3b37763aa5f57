#!/usr/bin/env python3
"""Summarize rocprofv3 --pmc passes (scripts/pmc_profile.sh layout) for one kernel:
mean value of every counter over that kernel's dispatches, plus derived
ratios.  Usage: pmc_summary.py gpurun_out/<TAG> [kernel_name]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    kname = sys.argv[2] if len(sys.argv) > 2 else "vx_main_rt_kernel"
    vals = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "*", "*counter_collection.csv"))):
        per = defaultdict(float)
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Kernel_Name"] != kname:
                    continue
                per[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
        for (_, c), v in per.items():
            vals[c].append(v)
    m = {c: sum(v) / len(v) for c, v in vals.items() if v}
    for c in sorted(m):
        print(f"{c:32s} {m[c]:18.1f}")
    g = m.get
    print("--- derived")
    if g("SQ_WAVE_CYCLES"):
        wc = m["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
            if g(k) is not None:
                print(f"{k + ' / WAVE_CYCLES':44s} {m[k] / wc:8.3f}")
    if g("SQ_WAVES") and g("SQ_INSTS_VALU"):
        print(f"{'VALU insts per wave':44s} {m['SQ_INSTS_VALU'] / m['SQ_WAVES']:8.0f}")
        for k in ("SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_FLAT"):
            if g(k) is not None:
                print(f"{k + ' per wave':44s} {m[k] / m['SQ_WAVES']:8.0f}")
    if g("SQ_THREAD_CYCLES_VALU") and g("SQ_ACTIVE_INST_VALU"):
        print(f"{'VALU lane utilisation':44s} {m['SQ_THREAD_CYCLES_VALU'] / (64 * m['SQ_ACTIVE_INST_VALU']):8.3f}")
    if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum") is not None:
        t = m["TCC_HIT_sum"] + m["TCC_MISS_sum"]
        print(f"{'L2 hit rate':44s} {m['TCC_HIT_sum'] / t if t else 0:8.3f}")
    if g("TCP_TOTAL_CACHE_ACCESSES_sum") and g("TCP_TCC_READ_REQ_sum") is not None:
        print(f"{'L1 -> L2 read req / L1 access':44s} "
              f"{m['TCP_TCC_READ_REQ_sum'] / m['TCP_TOTAL_CACHE_ACCESSES_sum']:8.4f}")
    if g("FETCH_SIZE") is not None:
        print(f"{'FETCH_SIZE (KB) per dispatch':44s} {m['FETCH_SIZE']:8.0f}")
    if g("WRITE_SIZE") is not None:
        print(f"{'WRITE_SIZE (KB) per dispatch':44s} {m['WRITE_SIZE']:8.0f}")


if __name__ == "__main__":
    main()
