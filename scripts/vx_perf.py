#!/usr/bin/env python3
"""vx_dump_perf for MI355X: the reference's performance-counter classes
(VORTEX_PROFILING = VX_DCR_MPM_CLASS_CORE 1 / MEM 2 / TEX 3 / RASTER 4 /
OM 5; runtime/stub/utils.cpp:159-805) mapped to gfx950 hardware counters,
collected with rocprofv3 --pmc (one pass per counter group, within the
per-block limits) over any command that launches the `vx_main` kernels, and
printed as the reference's "PERF: ..." lines (per launch, averaged over the
command's launches of the kernel).

    python scripts/vx_perf.py --class 1 -- python3 scripts/prof_rt.py --frames 10

Mapping (reference line <- gfx950 counter):
  every class  instrs, cycles, IPC        <- SQ_INSTS, GRBM_GUI_ACTIVE / 8 (the counter sums
                                             the 8 XCDs' busy cycles)
  CORE   scheduler idle / stalls          <- SQ_WAIT_ANY, SQ_WAIT_INST_ANY (of SQ_WAVE_CYCLES)
         scoreboard stalls (alu/fpu/lsu)  <- SQ_ACTIVE_INST_{SALU,VALU,VMEM,LDS} shares
         ifetches, loads, stores          <- SQ_IFETCH, SQ_INSTS_VMEM_RD + SMEM, SQ_INSTS_VMEM_WR
         ifetch / load latency            <- InstrFetchLatency, VmemLatency
  MEM    lmem reads/writes/bank stalls    <- SQ_INSTS_LDS, SQ_LDS_BANK_CONFLICT
         dcache reads/read misses         <- TCP_TOTAL_CACHE_ACCESSES_sum, TCP_TCC_READ_REQ_sum
         l2cache reads/writes/misses      <- TCC_READ_sum, TCC_WRITE_sum, TCC_MISS_sum
         memory requests (reads, writes)  <- TCC_EA0_RDREQ_sum, TCC_EA0_WRREQ_sum
  TEX    tex memory reads / stalls        <- TA_BUFFER_READ_WAVEFRONTS_sum, TA_DATA_STALLED_BY_TC_CYCLES_sum
         tcache reads / read misses       <- TCP_TOTAL_CACHE_ACCESSES_sum, TCP_TCC_READ_REQ_sum
  RASTER raster memory reads / latency    <- SQ_INSTS_SMEM, SmemLatency (records via the scalar cache)
         rcache reads / read misses       <- SQC_DCACHE_REQ, SQC_DCACHE_MISSES
  OM     om memory writes / stalls        <- TA_BUFFER_WRITE_WAVEFRONTS_sum, TCP_PENDING_STALL_CYCLES_sum
         ocache writes / write requests   <- TCP_TOTAL_WRITE_sum, TCP_TCC_WRITE_REQ_sum
"""
import argparse
import csv
import glob
import os
import subprocess
import sys
from collections import defaultdict

XCDS = 8  # MI355X: GRBM_GUI_ACTIVE is reported per XCD and summed
BASE = [["SQ_INSTS", "SQ_WAVES", "GRBM_GUI_ACTIVE"]]
PASSES = {
    1: [["SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_SALU",
         "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS"],
        ["SQ_IFETCH", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_WR"],
        ["InstrFetchLatency"], ["VmemLatency"]],
    2: [["SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_LDS"],
        ["TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum"],
        ["TCC_READ_sum", "TCC_WRITE_sum"], ["TCC_MISS_sum", "TCC_HIT_sum"],
        ["TCC_EA0_RDREQ_sum", "TCC_EA0_WRREQ_sum"]],
    3: [["TA_BUFFER_READ_WAVEFRONTS_sum", "TA_DATA_STALLED_BY_TC_CYCLES_sum"],
        ["TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum"], ["VmemLatency"]],
    4: [["SQ_INSTS_SMEM"], ["SmemLatency"], ["SQC_DCACHE_REQ", "SQC_DCACHE_MISSES"]],
    5: [["TA_BUFFER_WRITE_WAVEFRONTS_sum", "TA_BUFFER_READ_WAVEFRONTS_sum"],
        ["TCP_TOTAL_WRITE_sum", "TCP_TCC_WRITE_REQ_sum"], ["TCP_PENDING_STALL_CYCLES_sum"]],
}


def collect(outdir, passes, cmd, kernel, timeout):
    vals = {}
    for i, counters in enumerate(passes):
        d = os.path.join(outdir, f"pass{i}")
        rc = subprocess.call(["timeout", "-s", "KILL", str(timeout), "rocprofv3", "--pmc", *counters,
                              "-d", d, "-o", "run", "--output-format", "csv", "--", *cmd],
                             stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        if rc != 0:
            raise SystemExit(f"rocprofv3 pass {counters} failed with {rc}")
        per = defaultdict(float)
        n = set()
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if not row["Kernel_Name"].startswith(kernel) or row["Kernel_Name"].endswith("_done"):
                        continue
                    per[row["Counter_Name"]] += float(row["Counter_Value"])
                    n.add(row["Dispatch_Id"])
        for c in counters:
            vals[c] = per.get(c, 0.0) / max(len(n), 1)
    return vals


def pct(a, b):
    return int(100.0 * a / b) if b else 0


def report(cls, v, out=sys.stdout):
    g = lambda k: int(v.get(k, 0))  # noqa: E731
    p = lambda s: print("PERF: " + s, file=out)  # noqa: E731
    if cls == 1:
        wc = v.get("SQ_WAVE_CYCLES", 0)
        p(f"scheduler idle={g('SQ_WAIT_ANY')} ({pct(v.get('SQ_WAIT_ANY', 0), wc)}%)")
        p(f"scheduler stalls={g('SQ_WAIT_INST_ANY')} ({pct(v.get('SQ_WAIT_INST_ANY', 0), wc)}%)")
        act = sum(v.get(k, 0) for k in ("SQ_ACTIVE_INST_SALU", "SQ_ACTIVE_INST_VALU",
                                        "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS"))
        p(f"scoreboard stalls={int(act)} ({pct(act, wc)}%) (alu={pct(v.get('SQ_ACTIVE_INST_SALU', 0), act)}%, "
          f"fpu={pct(v.get('SQ_ACTIVE_INST_VALU', 0), act)}%, lsu={pct(v.get('SQ_ACTIVE_INST_VMEM', 0), act)}%, "
          f"lmem={pct(v.get('SQ_ACTIVE_INST_LDS', 0), act)}%)")
        p(f"ifetches={g('SQ_IFETCH')}")
        p(f"loads={g('SQ_INSTS_VMEM_RD') + g('SQ_INSTS_SMEM')}")
        p(f"stores={g('SQ_INSTS_VMEM_WR')}")
        p(f"ifetch latency={g('InstrFetchLatency')} cycles")
        p(f"load latency={g('VmemLatency')} cycles")
    elif cls == 2:
        p(f"lmem reads={g('SQ_INSTS_LDS')}")
        p(f"lmem bank stalls={g('SQ_LDS_BANK_CONFLICT')} "
          f"(utilization={100 - pct(v.get('SQ_LDS_BANK_CONFLICT', 0), v.get('SQ_ACTIVE_INST_LDS', 0))}%)")
        acc, miss = v.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0), v.get("TCP_TCC_READ_REQ_sum", 0)
        p(f"dcache reads={int(acc)}")
        p(f"dcache read misses={int(miss)} (hit ratio={100 - pct(miss, acc)}%)")
        hit, mis = v.get("TCC_HIT_sum", 0), v.get("TCC_MISS_sum", 0)
        p(f"l2cache reads={g('TCC_READ_sum')}")
        p(f"l2cache writes={g('TCC_WRITE_sum')}")
        p(f"l2cache read misses={int(mis)} (hit ratio={pct(hit, hit + mis)}%)")
        r, w = g("TCC_EA0_RDREQ_sum"), g("TCC_EA0_WRREQ_sum")
        p(f"memory requests={r + w} (reads={r}, writes={w})")
    elif cls == 3:
        p(f"tex memory reads={g('TA_BUFFER_READ_WAVEFRONTS_sum')}")
        p(f"tex memory latency={g('VmemLatency')} cycles")
        p(f"tex stalls={g('TA_DATA_STALLED_BY_TC_CYCLES_sum')} "
          f"({pct(v.get('TA_DATA_STALLED_BY_TC_CYCLES_sum', 0), v.get('GRBM_GUI_ACTIVE', 0))}%)")
        acc, miss = v.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0), v.get("TCP_TCC_READ_REQ_sum", 0)
        p(f"tcache reads={int(acc)}")
        p(f"tcache read misses={int(miss)} (hit ratio={100 - pct(miss, acc)}%)")
    elif cls == 4:
        p(f"raster memory reads={g('SQ_INSTS_SMEM')}")
        p(f"raster memory latency={g('SmemLatency')} cycles")
        req, miss = v.get("SQC_DCACHE_REQ", 0), v.get("SQC_DCACHE_MISSES", 0)
        p(f"rcache reads={int(req)}")
        p(f"rcache read misses={int(miss)} (hit ratio={100 - pct(miss, req)}%)")
    elif cls == 5:
        p(f"om memory reads={g('TA_BUFFER_READ_WAVEFRONTS_sum')}")
        p(f"om memory writes={g('TA_BUFFER_WRITE_WAVEFRONTS_sum')}")
        p(f"om stalls={g('TCP_PENDING_STALL_CYCLES_sum')}")
        p(f"ocache writes={g('TCP_TOTAL_WRITE_sum')}")
        p(f"ocache write requests={g('TCP_TCC_WRITE_REQ_sum')}")
    instrs, cycles = g("SQ_INSTS"), g("GRBM_GUI_ACTIVE") // XCDS
    p(f"instrs={instrs}, cycles={cycles}, IPC={instrs / cycles if cycles else 0.0:f}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--class", dest="cls", type=int, default=int(os.environ.get("VORTEX_PROFILING", "1")),
                    choices=(0, 1, 2, 3, 4, 5))
    ap.add_argument("--kernel", default="vx_main", help="kernel name prefix (every image: vx_main_<image>)")
    ap.add_argument("--out", default="gpurun_out/vx_perf")
    ap.add_argument("--timeout", type=int, default=60)
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    args = ap.parse_args()
    cmd = args.cmd[1:] if args.cmd[:1] == ["--"] else args.cmd
    if not cmd:
        ap.error("no command")
    passes = BASE + PASSES.get(args.cls, [])
    v = collect(os.path.join(args.out, f"class{args.cls}"), passes, cmd, args.kernel, args.timeout)
    report(args.cls, v)


if __name__ == "__main__":
    main()
