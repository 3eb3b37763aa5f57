#!/usr/bin/env python3
"""Reduce the rocprofv3 --pmc passes of scripts/pmc_profile.sh for one mode to
the record bench.py reports (profiles/pmc_<mode>.json): per-launch means over
the dispatches of the timed image's own entry (vx_main_<image>: the setup
and instrumented launches of the same process are other kernels) of every
counter, HBM traffic and derived ratios.

HBM bytes, calibrated on known-byte probes (scripts/pmc_calibrate.sh ->
profiles/r03/pmc_calibration.json): FETCH_SIZE counts a 16-B/lane vector read
at half its bytes (x2, as MI355X_MICROARCH.md says) but a 64-B s_load_dwordx16
record read at its bytes (x1); WRITE_SIZE counts the 4-B/lane framebuffer
stores at their bytes (x1).  The RT kernels read through both paths and the
memory-side counter cannot tell them apart, so the read side is reported as
bounds [FETCH x1, FETCH x2] and `traffic_bytes` is the upper bound.  SQ_WAVE_CYCLES
/ SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles (summed over waves), so their
ratios are what is meaningful.
A workload of several kernels per frame (config 4: pt_primary + pt_queue)
passes its images comma-separated: every counter is the sum over the images
of their per-dispatch means (one dispatch of each per frame), the record
carries each image's MD5 and `kernel_md5` = the MD5 of the images' bytes
concatenated in that order.
Usage: pmc_profile.py <tag_dir> <mode> <side> <kernel .co[,.co]> <out.json>"""
import csv
import glob
import hashlib
import json
import os
import sys
from collections import defaultdict


def means(d, kname):
    """counter -> mean over dispatches of kernel `kname` (values summed per dispatch)."""
    per = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Kernel_Name"] != kname:
                    continue
                per[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    return {c: sum(v.values()) / len(v) for c, v in per.items() if v}, \
        {c: len(v) for c, v in per.items()}


def images_md5(cos):
    """MD5 of the images' bytes concatenated in order (one image: its MD5)."""
    h = hashlib.md5()
    for co in cos:
        h.update(open(co, "rb").read())
    return h.hexdigest()


def main():
    tag, mode, side, co_arg, out = sys.argv[1:6]
    cos = co_arg.split(",")
    knames = [f"vx_main_{os.path.splitext(os.path.basename(co))[0]}" for co in cos]
    side = int(side)
    m, nd = defaultdict(float), {}
    for kname in knames:
        for d in sorted(glob.glob(os.path.join(tag, f"{mode}_*"))):
            if os.path.isdir(d):
                a, b = means(d, kname)
                for c, v in a.items():
                    m[c] += v
                for c, v in b.items():
                    nd[f"{kname}:{c}"] = v
    m = dict(m)
    if "FETCH_SIZE" not in m or "WRITE_SIZE" not in m:
        sys.exit(f"no {knames} dispatches with FETCH_SIZE / WRITE_SIZE")
    kname = "+".join(knames)
    g = m.get
    der = {}
    wc = g("SQ_WAVE_CYCLES")
    if wc:
        for k, n in (("SQ_WAIT_ANY", "wait_any_frac"), ("SQ_WAIT_INST_ANY", "wait_inst_any_frac"),
                     ("SQ_ACTIVE_INST_ANY", "active_inst_any_frac"),
                     ("SQ_ACTIVE_INST_VALU", "active_inst_valu_frac"),
                     ("SQ_ACTIVE_INST_LDS", "active_inst_lds_frac"),
                     ("SQ_WAIT_INST_LDS", "wait_inst_lds_frac")):
            if g(k) is not None:
                der[n] = round(m[k] / wc, 4)
    if g("SQ_WAVES"):
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS",
                  "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_WR"):
            if g(k) is not None:
                der[k.lower().replace("sq_insts_", "") + "_insts_per_wave"] = round(m[k] / m["SQ_WAVES"], 1)
    if g("SQ_THREAD_CYCLES_VALU") and g("SQ_ACTIVE_INST_VALU"):
        der["valu_lane_utilisation"] = round(m["SQ_THREAD_CYCLES_VALU"] / (64 * m["SQ_ACTIVE_INST_VALU"]), 4)
    if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum") is not None and m["TCC_HIT_sum"] + m["TCC_MISS_sum"]:
        der["l2_hit_rate"] = round(m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"]), 4)
    if g("TCP_TOTAL_CACHE_ACCESSES_sum") and g("TCP_TCC_READ_REQ_sum") is not None:
        der["l1_hit_rate"] = round(1.0 - m["TCP_TCC_READ_REQ_sum"] / m["TCP_TOTAL_CACHE_ACCESSES_sum"], 4)
    f_kb, w_kb = m["FETCH_SIZE"], m["WRITE_SIZE"]
    lo, hi = int(f_kb * 1024 + w_kb * 1024), int(2 * f_kb * 1024 + w_kb * 1024)
    res = {
        "kernel": kname, "mode": mode, "width": side, "height": side,
        "kernel_image": "+".join(os.path.basename(co) for co in cos),
        "kernel_md5": images_md5(cos),
        "kernel_md5s": {os.path.basename(co): images_md5([co]) for co in cos},
        "dispatches": nd,
        "fetch_size_kb": round(f_kb, 1), "write_size_kb": round(w_kb, 1),
        "correction": ("calibrated (profiles/r03/pmc_calibration.json): reads FETCH_SIZE x1024 x1 "
                       "(s_load records) .. x2 (16-B/lane vector loads), writes WRITE_SIZE x1024 x1 "
                       "(4-B/lane stores)"),
        "traffic_calibrated": True,
        "traffic_bounds": [lo, hi],
        "traffic_bytes": hi,
        "sq": {k: round(v, 1) for k, v in sorted(m.items()) if k not in ("FETCH_SIZE", "WRITE_SIZE")},
        "derived": der,
        "source": "scripts/pmc_profile.sh (rocprofv3 --pmc, one pass per counter group)",
    }
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
