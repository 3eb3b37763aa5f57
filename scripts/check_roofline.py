#!/usr/bin/env python3
"""Recompute a bench line's roofline numbers from the committed profiles
(the headline must be reproducible from profiles/ for the
image actually timed).

Inputs: the bench JSON line (bench.py's stdout, or the driver's BENCH_rNN.json
whose `parsed` holds it), the rocprofv3 --kernel-trace --stats summary of the
same command (<prefix>_kernel_stats.csv: one row per kernel name; every
image's entry is vx_main_<image>, so the timed kernel is its own row), and
the PMC record the line cites (profiles/pmc_<mode>.json).

Recomputed:
  roofline.frac            algorithmic bytes per launch / rocprof average
                           duration of the timed image / 8 TB/s
  roofline.measured_hbm_frac  PMC traffic per launch / the same duration / 8 TB/s
  roofline_issue.frac      PMC VALU wave-instructions per launch / duration /
                           1228.8 G/s
and compared with the line (which uses the HIP-event average of its own timed
launches): each must agree within --tol (default 5 %).

The line's series entries (bvh_walk: config 3 by BVH traversal, image
rt_bvh; path: config 4; flat: config 2; strong_4096: config 5's frame on one
GPU) are checked the same way against their own images' dispatches and the
PMC records they cite.

Usage: check_roofline.py <bench.json> <kernel_stats.csv> [--pmc profiles/pmc_shadow.json]
       [--trace <kernel_trace.csv[.gz]>]  (default: the stats path with kernel_stats -> kernel_trace)"""
import argparse
import csv
import gzip
import json
import os
import sys

HBM_PEAK_GBS = 8000.0
VALU_ISSUE_PEAK_GIPS = 1024 * 2.4 / 2.0
# the kernels of one frame (config 4: the one-kernel pt_kernel; under
# RT_PT_QUEUE=1 two launches, pt_primary + pt_queue)
IMAGE_OF = {"shadow": ("vx_main_rt_kernel",), "path": ("vx_main_pt_kernel",),
            "flat": ("vx_main_rt_flat",)}


def load_line(path):
    d = json.load(open(path))
    return d.get("parsed", d)


def mode_of(line):
    m = line["metric"]
    return "path" if "path trace" in m else ("flat" if "flat" in m else "shadow")


def timed_runs(path, kname, steps, max_gap_ns=100000):
    """Every run of >= `steps` consecutive `kname` dispatches with no other
    kernel between them and no idle gap of max_gap_ns or more (see
    timed_region): the average duration (s) of each run's first `steps`."""
    f = gzip.open(path, "rt") if path.endswith(".gz") else open(path)
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                 for r in csv.DictReader(f)), key=lambda t: t[0])
    runs, run = [], []
    for st, en, nm in ks + [(0, 0, "")]:
        if nm == kname and (not run or st - run[-1][1] < max_gap_ns):
            run.append((st, en))
            continue
        if len(run) >= steps:
            d = [e - b for b, e in run[:steps]]
            runs.append(sum(d) / len(d) * 1e-9)
        run = [(st, en)] if nm == kname else []
    return runs


def timed_region(path, kname, steps, max_gap_ns=100000):
    """Average duration (s) of the timed frames in a rocprofv3 kernel trace:
    the first run of >= `steps` consecutive `kname` dispatches with no other
    kernel between them and no idle gap of max_gap_ns or more (the timed
    region starts after the warmup's drain + synchronize, a gap of ~1 ms, and
    the kernel clock's frames after it follow another; the host's occasional
    few-10-us stalls inside the region do not split it); its first `steps`
    dispatches.  None when there is no such run."""
    f = gzip.open(path, "rt") if path.endswith(".gz") else open(path)
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                 for r in csv.DictReader(f)), key=lambda t: t[0])
    run = []
    for st, en, nm in ks:
        if nm == kname and (not run or st - run[-1][1] < max_gap_ns):
            run.append((st, en))
            continue
        if len(run) >= steps:
            break
        run = [(st, en)] if nm == kname else []
    if len(run) < steps:
        return None
    d = [en - st for st, en in run[:steps]]
    return sum(d) / len(d) * 1e-9


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("bench")
    ap.add_argument("stats")
    ap.add_argument("--pmc", default=None)
    ap.add_argument("--tol", type=float, default=0.05)
    ap.add_argument("--trace", default=None)
    a = ap.parse_args()
    line = load_line(a.bench)
    mode = mode_of(line)
    rows = {r["Name"]: r for r in csv.DictReader(open(a.stats))}
    knames = IMAGE_OF[mode]
    if mode == "path" and "vx_main_pt_queue" in rows and "vx_main_pt_kernel" not in rows:
        knames = ("vx_main_pt_primary", "vx_main_pt_queue")
    for k in knames:
        if k not in rows:
            sys.exit(f"{k} not in {a.stats} (names: {sorted(rows)})")
    # a frame's device time: the sum of its kernels' average durations
    dur_s = sum(float(rows[k]["AverageNs"]) for k in knames) * 1e-9
    pmc = json.load(open(a.pmc or f"profiles/pmc_{mode}.json"))
    rf = line["roofline"]
    out = {"kernel": "+".join(knames), "rocprof_calls": [int(rows[k]["Calls"]) for k in knames],
           "rocprof_avg_ms": round(dur_s * 1e3, 5),
           "line_kernel_ms": line["config"]["kernel_ms"], "checks": {}}
    # The summary averages every dispatch of the command -- also the
    # synchronous frames before the timed region and, at N = 1, the
    # moving-light series after it (the same kernel on frames whose light
    # moves).  With the per-dispatch trace beside it (--trace, default
    # <prefix>_kernel_trace.csv), the check uses the timed region itself
    # (timed_region).
    tpath = a.trace or a.stats.replace("kernel_stats", "kernel_trace")
    if not os.path.exists(tpath) and os.path.exists(tpath + ".gz"):
        tpath += ".gz"
    if len(knames) == 1 and tpath != a.stats and os.path.exists(tpath):
        tr = timed_region(tpath, knames[0], int(line["steps"]))
        if tr is not None:
            out["rocprof_summary_avg_ms"] = out["rocprof_avg_ms"]
            out["rocprof_avg_ms"] = round(tr * 1e3, 5)
            out["rocprof_avg_of"] = f"the {line['steps']} timed dispatches ({os.path.basename(tpath)})"
            dur_s = tr
    ok = True

    def check(name, mine, theirs):
        nonlocal ok
        rel = abs(mine - theirs) / theirs if theirs else float("inf")
        good = rel <= a.tol
        ok &= good
        out["checks"][name] = {"recomputed": round(mine, 4), "line": theirs, "rel_diff": round(rel, 4),
                               "ok": good}

    if mode != "flat":
        check("roofline.frac", rf["algorithmic_bytes_per_launch"] / dur_s / 1e9 / HBM_PEAK_GBS, rf["frac"])
    if rf.get("measured_hbm_frac") is not None:
        check("roofline.measured_hbm_frac", pmc["traffic_bytes"] / dur_s / 1e9 / HBM_PEAK_GBS,
              rf["measured_hbm_frac"])
    issue = line.get("roofline_issue") or (rf if rf.get("bound") == "valu_issue" else None)
    if issue is not None and issue.get("frac") is not None:
        check("roofline_issue.frac", pmc["sq"]["SQ_INSTS_VALU"] / dur_s / 1e9 / VALU_ISSUE_PEAK_GIPS,
              issue["frac"])
    # the N = 1 series entries (bvh_walk, path, flat, strong_4096), each
    # against its own image's dispatches: from the trace, the first run of
    # the entry's steps within a factor 1.5 of its kernel clock (strong_4096
    # shares rt_kernel with the headline: its 4096^2 frames are ~10x
    # longer); without a trace, the summary row of an image no other entry
    # uses
    users = {}
    for name, sb in line.get("series", {}).items():
        if isinstance(sb, dict) and "image" in sb:
            users.setdefault(sb["image"].split("entry ")[-1].rstrip(")"), []).append(name)
    for name, sb in line.get("series", {}).items():
        if not isinstance(sb, dict) or "roofline" not in sb or "image" not in sb:
            continue
        kn = sb["image"].split("entry ")[-1].rstrip(")")
        if kn not in rows:
            continue
        db = None
        if tpath != a.stats and os.path.exists(tpath):
            near = [d for d in timed_runs(tpath, kn, int(sb["steps"]))
                    if 1 / 1.5 < d * 1e3 / sb["kernel_ms"] < 1.5]
            db = near[0] if near else None
        if db is None and kn != knames[0] and len(users.get(kn, [])) == 1:
            db = float(rows[kn]["AverageNs"]) * 1e-9
        if db is None:
            continue
        out[name] = {"kernel": kn, "rocprof_avg_ms": round(db * 1e3, 5), "line_kernel_ms": sb["kernel_ms"]}
        br = sb["roofline"]
        src = br.get("pmc_source") or (sb.get("roofline_issue") or {}).get("source", "").split(" ")[0]
        try:
            pb = json.load(open(src)) if src else None
        except OSError:
            pb = None
        if br.get("bound") == "hbm":
            check(f"series.{name}.roofline.frac", br["algorithmic_bytes_per_launch"] / db / 1e9 / HBM_PEAK_GBS,
                  br["frac"])
            if pb is not None and br.get("measured_hbm_frac") is not None:
                check(f"series.{name}.roofline.measured_hbm_frac", pb["traffic_bytes"] / db / 1e9 / HBM_PEAK_GBS,
                      br["measured_hbm_frac"])
        bi = sb.get("roofline_issue") or (br if br.get("bound") == "valu_issue" else None)
        if pb is not None and bi and bi.get("frac") is not None:
            check(f"series.{name}.roofline_issue.frac", pb["sq"]["SQ_INSTS_VALU"] / db / 1e9 / VALU_ISSUE_PEAK_GIPS,
                  bi["frac"])
    out["ok"] = ok
    print(json.dumps(out, indent=1))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
