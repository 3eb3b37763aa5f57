#!/usr/bin/env python3
"""bench.py -- headline benchmark: Mrays/s of the MI355X ray-tracing hot path.

Workload at N = 1 (BASELINE.json configs[2], the metric's config):
tekkaman.cgltrace, 1024x1024, one primary ray per pixel (raster-exact, from
the per-8x8-block candidate lists built on the device) + one any-hit shadow
ray per geometry hit (ballot/mbcnt-compacted into full waves, each lane
scanning its light-space cell list -- the cube map of triangle lists around
the point light, built on the device -- nearest to the light first).  Timed beside it in the same command, each
with its own kernel clock, roofline and PMC record (`series`): the same frame
by BVH traversal only (binary16 BVH4 wave-packet walks; series.bvh_walk),
config 4's 4-bounce path trace (series.path), config 2's 256^2 flat list
(series.flat), config 5's 4096^2 frame on this one GPU (series.strong_4096:
the N = 1 point of the multi-GPU curve) and frames whose light moves every
step (series.moving_light).
A "step" is one full frame: vx_start of the RT kernel image through
libvortex-hip.so (inputs already resident in HBM), every frame complete
inside the timed region.

With N > 1 GPUs (one rank per GPU over RCCL) the default workload is
BASELINE config 5: ONE 4096x4096 frame whose 32x32 tiles are dealt
tile t -> rank t % N (sim/simx/raster_unit.cpp:109-111 striding), each step
ending with an RCCL gather of the ranks' compact tile buffers to rank 0 and
the frame assembly there -- strong scaling (fixed total
work).  `value` is then the whole job's rays/s (metric "Mrays/sec, all N
GPUs"; per GPU in config.mrays_per_s_per_gpu).  `--gpus N` without
WORLD_SIZE launches the N ranks itself (torch.distributed.run, before
anything touches a GPU).  The communicator's start and the first gathers
run under a watchdog (BENCH_DIST_TIMEOUT_S, default 240 s): a hang ends the
rank with a message and the tracebacks on stderr.  The line also carries
series.weak_1024_sqrtN (~1M pixels per GPU).

Rank 0 prints one JSON line.  Everything else goes to stderr.
"""
from __future__ import annotations

import argparse
import gc
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SCENE = os.path.join(ROOT, "tests", "golden", "scenes", "tekkaman.cgltrace")
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
NODE_BYTES, TRI_BYTES, PIXEL_BYTES = 64, 36, 4
MT_FLOPS = 40          # fp32 ops per Moller-Trumbore test
FP32_VALU_TFLOPS = 157.3  # MI355X_MICROARCH.md: peak FP32 (vector)
NODE4_BYTES = 112      # BVH4 node: 6 SoA box float4 + the child-ref float4 (pad not read)
NODE4H_BYTES = 64      # BVH4 node with binary16 planes (rt_node4h_t): 48 B of planes + 16 B refs
# VALU issue peak: 1024 SIMDs, one wave64 VALU instruction per 2 cycles per
# SIMD (MI355X_MICROARCH.md "issues each VALU instruction over 2 cycles"),
# at the 2.4 GHz peak engine clock
VALU_ISSUE_PEAK_GIPS = 1024 * 2.4 / 2.0
CONFIG5_SIDE = 4096    # BASELINE config 5


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def algorithmic_bytes(st: dict, pixels: int, node_bytes: int = NODE_BYTES) -> int:
    """node bytes (64 B BVH2, 112 B BVH4, 64 B binary16 BVH4) x nodes visited + 36 B x triangles tested
    (BVH leaves and screen layers) + texel bytes per shaded pixel + 4 B per
    pixel written.  Counts come from the instrumented kernel variant, whose
    counters tests/test_gpu_rt.py checks equal to the oracle's traversal."""
    return (node_bytes * st["node_visits"] + TRI_BYTES * (st["tri_tests"] + st["layer_tests"])
            + st["texel_bytes"] + PIXEL_BYTES * pixels)


# the kernel images of one frame per workload (config 4: the one-kernel
# pt_kernel; pt_primary + pt_queue under RT_PT_QUEUE=1)
PMC_IMAGES = {"shadow": ("rt_kernel.co",), "path": ("pt_kernel.co",),
              "flat": ("rt_flat.co",), "bvh": ("rt_bvh.co",)}


def pmc_record(mode: str, side: int, images=None):
    """The committed rocprofv3 PMC record of this workload's kernel image
    (scripts/pmc_profile.sh -> profiles/pmc_<mode>.json): HBM traffic per
    launch (FETCH_SIZE x2 + WRITE_SIZE, the guide's gfx950 correction) and
    the SQ/TCP counters.  Returns (record or None, stale): stale = a record
    exists but was taken on another kernel image or size."""
    import hashlib
    t = None
    # profiles/pmc_<mode>.json at the mode's own size, pmc_<mode>_<side>.json
    # at another (e.g. config 5's 4096^2 frame on one GPU)
    for name in (f"pmc_{mode}.json", f"pmc_{mode}_{side}.json"):
        try:
            with open(os.path.join(ROOT, "profiles", name)) as fh:
                c = json.load(fh)
        except (OSError, ValueError):
            continue
        if t is None or (c.get("width") == side and t.get("width") != side):
            t = dict(c, _path=name)
    if t is None:
        return None, False
    try:
        h = hashlib.md5()  # the frame's images' bytes concatenated (scripts/pmc_profile.py)
        for co in images or PMC_IMAGES[mode]:
            h.update(open(os.path.join(ROOT, "skybox_rt_amd", "lib", co), "rb").read())
        md5 = h.hexdigest()
    except OSError:
        return None, True
    if t.get("kernel_md5") != md5 or t.get("width") != side or t.get("height") != side:
        return None, True
    return t, False


def issue_roofline(rec: dict, kernel_ms: float, mode: str):
    """VALU issue rate of the timed image (the PMC record's SQ_INSTS_VALU over
    the kernel's duration) against 1228.8 G wave-instructions/s, with the
    record's wait / utilisation / hit ratios; None without SQ counters."""
    if not rec or not rec.get("sq", {}).get("SQ_INSTS_VALU"):
        return None
    d = rec.get("derived", {})
    gips = rec["sq"]["SQ_INSTS_VALU"] / (kernel_ms * 1e-3) / 1e9
    return {"bound": "valu_issue", "achieved": round(gips, 2), "peak": VALU_ISSUE_PEAK_GIPS,
            "unit": "G wave-instr/s", "frac": round(gips / VALU_ISSUE_PEAK_GIPS, 4),
            "valu_insts_per_launch": int(rec["sq"]["SQ_INSTS_VALU"]),
            **{k: d[k] for k in ("wait_any_frac", "wait_inst_any_frac", "active_inst_any_frac",
                                 "active_inst_valu_frac", "valu_lane_utilisation",
                                 "l1_hit_rate", "l2_hit_rate") if k in d},
            "source": f"profiles/{rec.get('_path', f'pmc_{mode}.json')} (rocprofv3 --pmc passes, "
                      f"scripts/pmc_profile.sh)"}


COUNT_KEYS = ("node_visits", "tri_tests", "layer_tests", "texel_bytes", "primary_rays", "shadow_rays",
              "bounce_rays")


def make_roofline(inst: dict, kernel_ms: float, mode: str, side: int, node_bytes: int, images=None,
                  n_gpus: int = 1):
    """(roofline, roofline_issue) of one timed configuration: algorithmic bytes
    per launch (the instrumented pre-run's counts) over the kernel clock
    against 8 TB/s, the PMC record's measured traffic beside it, and the VALU
    issue roofline from the same record.  Config 2 (flat) reads its list from
    L2 and the scalar cache and prunes with integer rectangle tests: its
    roofline is the VALU-issue one, with the work executed per wave."""
    rec, stale = pmc_record(mode, side, images) if n_gpus == 1 else (None, False)
    traffic = rec["traffic_bytes"] if rec else None
    counts = {k: int(inst[k]) for k in COUNT_KEYS}
    alg = algorithmic_bytes(inst, inst["primary_rays"], node_bytes)
    ach = alg / (kernel_ms * 1e-3) / 1e9
    roof = {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
            "algorithmic_bytes_per_launch": int(alg), "counts": counts}
    if stale:
        roof["traffic_stale"] = True
    if rec:
        roof["traffic_calibrated"] = bool(rec.get("traffic_calibrated", False))
        if "traffic_bounds" in rec:
            roof["traffic_bounds"] = rec["traffic_bounds"]
        # measured HBM bytes per launch over the same kernel time: the share of
        # the HBM peak the kernel physically uses (the scene is cache-resident)
        roof["measured_hbm_gbs"] = round(traffic / (kernel_ms * 1e-3) / 1e9, 2)
        roof["measured_hbm_frac"] = round(traffic / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        roof["pmc_source"] = f"profiles/{os.path.basename(rec.get('_path', f'pmc_{mode}.json'))}"
    issue = issue_roofline(rec, kernel_ms, mode)
    if mode == "flat":
        work = {"rect_tests_per_wave": int(inst["rect_tests"]), "edge_tests_per_wave": int(inst["edge_tests"]),
                "list_entries_per_ray_algorithmic": int(inst["tri_tests"])}
        if issue is not None:
            roof = {**issue, "traffic": traffic, "work_executed": work, "counts": counts}
            if rec:
                roof["measured_hbm_gbs"] = round(traffic / (kernel_ms * 1e-3) / 1e9, 2)
            issue = None
        else:
            roof.pop("algorithmic_bytes_per_launch")
            roof.update({"bound": "valu_issue", "achieved": None, "frac": None, "work_executed": work,
                         "note": "no current PMC record"})
    return roof, issue


def moving_lights(k: int):
    """k distinct point lights (clip x, y, w) circling above the model, the
    metric's light (0, 60, 80) among them."""
    return [(float(np.float32(40.0 * math.sin(2 * math.pi * i / k))),
             float(np.float32(60.0 + 10.0 * (math.cos(2 * math.pi * i / k) - 1.0))),
             float(np.float32(80.0 + 5.0 * math.sin(4 * math.pi * i / k)))) for i in range(k)]


def cold_configure_probe(rt, scene, side, kw, n=3):
    """A cold configure -- new renderer, so new resolution and new light:
    records, block lists, shadow lists, work order, one stream-ordered
    sequence -- on n fresh renderers, each with its own light (VERDICT r03
    item 4; tests/test_gpu_light.py times the same).  Returns the setup_stats
    of the fastest."""
    best = None
    for i in range(n):
        r = rt.Renderer(scene)
        try:
            light = (float(kw["light"][0]), float(kw["light"][1]) - i, float(kw["light"][2]))
            r.configure(side, side, counters=False, **dict(kw, light=light))
            st = r.setup_stats()
        finally:
            r.close()
        if best is None or st["configure_ms"] < best["configure_ms"]:
            best = st
    return best


def moving_light_series(r, side, steps, warmup, kw):
    """Every step moves the light (rt_renderer_set_light) and renders a
    frame -- the reference's per-render re-binning regime
    (tests/regression/draw3d/main.cpp:179-211).  Frames back to back, no
    per-launch events, under the renderer's default list policy: a frame
    whose light just moved traces its shadow rays by the BVH packet walk
    (the same verdicts), the light-space lists are rebuilt only once a light
    stays (rt_renderer_set_list_policy).  Beside it the same steps with the
    lists rebuilt for every light before its frame (policy 0: 6 setup
    launches queued behind the previous frame) and the cost of one such
    rebuild alone (set_light + wait, median of 16: slist_build_ms).  The
    last frame is checked against a fresh configure with its light."""
    import torch
    lights = moving_lights(16)
    r.configure(side, side, counters=False, **dict(kw, light=lights[0]))
    r.render()
    r.set_list_policy(0)
    one = []
    for L in lights[1:] + lights[:1]:
        t0 = time.perf_counter()
        r.set_light(L)
        r.wait()
        one.append((time.perf_counter() - t0) * 1e3)
    defer = int(os.environ.get("RT_SLIST_DEFER", "8"))

    def steps_ms(policy):
        r.set_list_policy(policy)
        r.set_timing(False)
        try:
            for i in range(warmup):
                r.set_light(lights[i % 16])
                r.start()
            r.wait()
            torch.cuda.synchronize()
            _, _, n0 = r.run_totals()
            t0 = time.perf_counter()
            for i in range(steps):
                r.set_light(lights[i % 16])
                r.start()
            r.wait()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            _, _, n1 = r.run_totals()
        finally:
            r.set_timing(True)
        return el / steps * 1e3, (n1 - n0) / steps

    rebuild_ms, rebuild_runs = steps_ms(0)
    ms, runs = steps_ms(defer)
    last = lights[(steps - 1) % 16]
    fb = r.framebuffer().copy()
    st = r.setup_stats()
    r.configure(side, side, counters=False, **dict(kw, light=last))
    r.render()
    same = bool(np.array_equal(fb, r.framebuffer()))
    return {"steps": steps, "lights": 16, "ms_per_step": round(ms, 5), "runs_per_step": round(runs, 3),
            "list_policy": f"lists deferred until a light stays {defer} frames (rt_renderer_set_list_policy)",
            "slist_on_last": int(st["slist_on"]), "slist_stale_last": int(st["slist_stale"]),
            "ms_per_step_lists_rebuilt_every_step": round(rebuild_ms, 5),
            "runs_per_step_lists_rebuilt_every_step": round(rebuild_runs, 3),
            "slist_build_ms": round(float(np.median(one)), 4),
            "slist_build_ms_min": round(float(min(one)), 4),
            "last_frame_equals_configured_render": same}


def frame_side(n_gpus: int, base: int) -> int:
    return max(32, int(round(base * math.sqrt(n_gpus) / 32.0)) * 32)


def physical_cores(cpus) -> int:
    """Distinct (package, core) pairs among `cpus` (/proc/cpuinfo)."""
    try:
        pairs, cur = set(), {}
        with open("/proc/cpuinfo") as fh:
            for ln in list(fh) + [""]:
                if not ln.strip():
                    if cur.get("processor") is not None and int(cur["processor"]) in cpus:
                        pairs.add((cur.get("physical id"), cur.get("core id")))
                    cur = {}
                    continue
                k, _, v = ln.partition(":")
                cur[k.strip()] = v.strip()
        return len(pairs) or len(cpus)
    except OSError:
        return len(cpus)


def cgroup_cpus():
    """CPU bandwidth quota of this cgroup in CPUs (cpu.max), or None."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(shadows: bool, side: int, light, budget_s: float, path: bool = False,
                 bounces: int = 4, flat: bool = False, bvh4: bool = True):
    """Oracle (C port of the same algorithm, oracle/rt.c) on the host cores,
    BVH traversal identical to the kernel's: threads = every CPU this process
    may run on (SURVEY.md 8(d) / BASELINE.md: all host cores) -- the CPUs of
    its affinity set, capped by its cgroup's CPU quota when one is set (a GPU
    box job sees 256 CPUs but is granted 16: 256 threads there run slower
    than 16, so that rate is reported beside it) -- median of 5 timed runs
    of whole frames after a warm-up frame; the 1-thread frame must equal the
    N-thread frame bit for bit."""
    from oracle import py_oracle as po
    from skybox_rt_amd import rt as rtmod
    cpus = sorted(os.sched_getaffinity(0))
    quota = cgroup_cpus()
    threads = len(cpus) if quota is None else max(1, min(len(cpus), int(quota)))
    osc = po.OracleScene(po.cgltrace.load(SCENE))
    sc = rtmod.Scene.load(SCENE)
    bvh = None if flat else (sc.bvh() + ((sc.bvh4(),) if bvh4 else ()))

    def params(nt):
        return po.rt_params(side, side, shadows=shadows, light=light, nthreads=nt, path=path,
                            bounces=bounces)

    def rays_of(k):
        return k["primary_rays"] + k["shadow_rays"] + k["bounce_rays"]

    pn, p1 = params(threads), params(1)
    t = time.perf_counter()
    c1, _, _, k1 = po.rt_render(osc, p1, bvh=bvh)            # one single-thread frame
    el1 = time.perf_counter() - t
    cn, _, _, kn = po.rt_render(osc, pn, bvh=bvh)            # warm-up, all threads
    identical = bool(np.array_equal(c1, cn)) and k1 == kn
    runs = []
    frames_total = 0
    for _ in range(5):
        frames, rays, t0 = 0, 0, time.perf_counter()
        while True:
            _, _, _, k = po.rt_render(osc, pn, bvh=bvh)
            frames += 1
            rays += rays_of(k)
            el = time.perf_counter() - t0
            if el >= budget_s / 5:
                break
        frames_total += frames
        runs.append(rays / el / 1e6)
    all_aff = None
    if threads < len(cpus):  # one run with a thread per affinity CPU, for the record
        pa = params(len(cpus))
        frames, rays, t0 = 0, 0, time.perf_counter()
        while True:
            _, _, _, k = po.rt_render(osc, pa, bvh=bvh)
            frames += 1
            rays += rays_of(k)
            el = time.perf_counter() - t0
            if el >= budget_s / 5:
                break
        all_aff = rays / el / 1e6
    cpu_model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            cpu_model = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")),
                             cpu_model)
    except OSError:
        pass
    # the algorithm rt_params selects (oracle/py_oracle.py: vis_lists and
    # shadow_lists on by default), the same as the GPU image's
    if flat:
        algo = "brute force over the geometry list"
    else:
        algo = ("primary: 8x8-block candidate lists; "
                + ("shadow: light-space cell lists" if shadows or path else "no shadow rays")
                + (f"; bounce rays: {'BVH4' if bvh4 else 'BVH2'} traversal" if path else ""))
    return {"value": float(np.median(runs)), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"median of 5 timed runs ({frames_total} full {side}x{side} frames of the same "
                      f"workload in ~{budget_s:.0f} s; oracle/rt.c {algo}, "
                      f"{threads} threads = every CPU granted to this process: {len(cpus)} in the "
                      f"affinity set, cgroup quota {quota}) after a warm-up frame",
            "runs_mrays_per_s": [round(x, 3) for x in runs],
            "threads": threads, "affinity_cpus": len(cpus),
            "physical_cores": physical_cores(set(cpus)), "cgroup_cpu_quota": quota,
            "all_affinity_threads_value": all_aff,
            "single_thread_value": rays_of(k1) / el1 / 1e6,
            "one_vs_all_threads_bit_identical": identical,
            "cpu_model": cpu_model, "host_cpus": os.cpu_count()}


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """`--gpus N` outside a launcher: start N ranks (one per GPU) with
    torch.distributed.run as CHILD processes -- this process never touches a
    GPU -- and return their exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    log("bench.py: launching", " ".join(cmd))
    env = dict(os.environ, BENCH_LAUNCHED="1")
    return subprocess.call(cmd, env=env)


class Run:
    """One timed configuration of the renderer (+ the RCCL gather at N > 1)."""

    def __init__(self, r, rt, dist, coll_dev, rank, n_gpus, side, shadows, light, path, flat,
                 bounces, use_gather, bvh_walk=False):
        self.r, self.side, self.n = r, side, n_gpus
        self.kw = dict(shadows=shadows, light=light, shard_index=rank, shard_count=n_gpus,
                       path=path, bounces=bounces, flat=flat, bvh_walk=bvh_walk)
        # algorithmic bytes per launch and rays per frame from the instrumented
        # variant (untimed; its counters equal the oracle's traversal,
        # tests/test_gpu_rt.py): the timed product image writes no counters
        r.configure(side, side, instrumented=True, **self.kw)
        # the renderer's first configure at this size and light: the cold
        # per-resolution + per-light setup (records, lists, work order)
        self.first_setup = r.setup_stats()
        r.render()
        self.inst = r.stats()
        self.rays_local = (self.inst["primary_rays"] + self.inst["shadow_rays"]
                           + self.inst["bounce_rays"])
        r.configure(side, side, compact=use_gather, counters=False, **self.kw)
        self.gather = None
        self.fg = None
        if use_gather:
            self._setup_gather(dist, coll_dev)

    def _setup_gather(self, dist, coll_dev):
        import ctypes
        import torch
        from skybox_rt_amd.shard import FrameGather
        r = self.r
        hip = ctypes.CDLL("libamdhip64.so.7")  # torch's runtime, already loaded
        self.slots = 4
        fg = FrameGather(dist, self.side, self.side, coll_dev, slots=self.slots)
        self.fg = fg
        dev_ptr, nbytes = r.framebuffer_device()
        kind = 3 if coll_dev.type == "cuda" else 2  # hipMemcpyDeviceToDevice / ToHost
        nsteps = [0]
        drv_stream = torch.cuda.ExternalStream(r.device_stream()) if kind == 3 else None
        hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.c_int, ctypes.c_void_p]

        def gather():
            # frame k's compact tile buffer -> a free gather slot, then the
            # gather + frame assembly enqueued asynchronously: frame k's
            # exchange overlaps the next frames' renders (4 slots in flight).
            # RCCL: the copy is queued on the driver's stream right behind
            # frame k's kernel (the host does not wait for the frame) and the
            # gather follows that stream; a slot is reclaimed on the host
            # once its gather of 4 frames ago has completed
            slot = nsteps[0] % self.slots
            nsteps[0] += 1
            fg.reclaim(slot)
            if kind == 3:
                hip.hipMemcpyAsync(fg.locals[slot].data_ptr(), dev_ptr, nbytes, kind,
                                   drv_stream.cuda_stream)
                fg.start(slot, stream=drv_stream)
            else:  # host-staged rehearsal (gloo): the frame must be complete
                r.wait()
                hip.hipMemcpy(ctypes.c_void_p(fg.locals[slot].data_ptr()),
                              ctypes.c_void_p(dev_ptr), ctypes.c_size_t(nbytes), kind)
                fg.start(slot)
        self.gather = gather

    def step(self, render=True, exchange=True):
        if render:
            self.r.start()
        if exchange and self.gather is not None:
            self.gather()

    def drain(self):
        self.r.wait()
        if self.fg is not None:
            for slot in range(self.slots):
                self.fg.reclaim(slot)

    def timed(self, steps, warmup, dist, render=True, exchange=True):
        """W untimed steps, then EXACTLY `steps` steps between barrier +
        synchronize on both sides; returns the elapsed seconds.  The frames
        carry no per-launch events (rt_render_set_timing 0: an event costs
        the device an idle gap per timed launch), so they run back to back;
        the kernel's duration comes from kernel_clock.  render / exchange =
        False leave that half out of every step (N > 1: the render and the
        frame exchange timed apart)."""
        import torch
        self.r.set_timing(False)
        try:
            for _ in range(warmup):
                self.step(render, exchange)
            self.drain()
            if dist is not None:
                dist.barrier()
            torch.cuda.synchronize()
            _, _, n0 = self.r.run_totals()
            gc.disable()  # no collector pause inside the timed region
            try:
                t0 = time.perf_counter()
                for _ in range(steps):
                    self.step(render, exchange)
                # every frame rendered (and gathered + assembled) inside the
                # region: the device synchronize first (it returns when the
                # driver's stream is idle), then the driver's and the
                # exchange's bookkeeping (instant for frames already done;
                # host-staged gathers still block here)
                torch.cuda.synchronize()
                self.drain()
                if self.fg is not None:
                    torch.cuda.synchronize()
                if dist is not None:
                    dist.barrier()
                elapsed = time.perf_counter() - t0
            finally:
                gc.enable()
            _, _, n1 = self.r.run_totals()
        finally:
            self.r.set_timing(True)
        assert n1 - n0 == (steps if render else 0), (n0, n1)
        return elapsed


    def kernel_clock(self, steps, warmup):
        """Average kernel duration per frame over a back-to-back run: the
        driver untimed (no per-launch events, no queue bound), `steps` frames
        started back to back, bracketed by two HIP events recorded on the
        driver's stream (the stream the kernel runs on): (stop - start) /
        steps.  Per-launch events cost the timed launch an idle gap and start
        it cold (rocprofv3 kernel trace: ~+1.5 us on a 24 us frame), so this,
        not their average, is the duration the roofline divides by; it equals
        rocprofv3's per-dispatch average of the same command."""
        import torch
        r = self.r
        stream = torch.cuda.ExternalStream(r.device_stream())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        r.set_timing(False)
        try:
            for _ in range(warmup):
                r.start()
            r.wait()
            e0.record(stream)
            for _ in range(steps):
                r.start()
            e1.record(stream)
            r.wait()
            e1.synchronize()
        finally:
            r.set_timing(True)
        return e0.elapsed_time(e1) / steps


def reduce_max_sum(dist, coll_dev, elapsed, rays):
    import torch
    if dist is None:
        return elapsed, float(rays)
    t = torch.tensor([elapsed, float(rays)], dtype=torch.float64, device=coll_dev)
    mx, sm = t.clone(), t.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(sm, op=dist.ReduceOp.SUM)
    return float(mx[0]), float(sm[1])


def describe(side, mode, setup_st, shadows, bounces, bvh_kind):
    """The workload text of one timed configuration (what the kernel runs)."""
    if mode == "flat":
        return (f"{side}x{side} primary rays, flat triangle list (no BVH), tekkaman.cgltrace: every "
                f"ray tests the whole geometry list -- a 512-thread workgroup per 64-pixel chunk "
                f"splits the list 8 ways, each wave tests 64 rectangle words per instruction (read "
                f"from L2) against the chunk's 8x8 block, then the entries reaching it per pixel "
                f"(exact edge + depth test, records through the scalar cache); the waves' winners "
                f"meet in LDS and wave 0 shades and stores the chunk (no shadow rays: the other "
                f"waves leave at the barrier)")
    primary = ("primary: 8x8-block candidate lists built on the device (raster-exact)"
               if setup_st["blist_blocks"] else f"primary: {bvh_kind} packet walk (raster-exact)")
    if mode == "path":
        kind = f"{bounces}-bounce diffuse path trace (primary + bounce + shadow rays)"
        if setup_st.get("path_queue"):
            shadow_how = ("light-space shadow lists" if setup_st["slist_on"] else f"{bvh_kind} walk")
            return (f"{side}x{side} {kind}, tekkaman.cgltrace, two kernels per frame: {primary}, "
                    f"path starts appended to a compacted queue (wave64: one atomic per wave, "
                    f"ballot/mbcnt slots); then the queued paths on full waves: bounce rays a "
                    f"per-lane {bvh_kind} walk (LDS stack), shadow rays on the {shadow_how}")
        if setup_st["slist_on"]:
            return (f"{side}x{side} {kind}, tekkaman.cgltrace, one kernel; {primary}; then each "
                    f"path on its lane(s): bounce rays a {bvh_kind} walk (LDS stack), shadow rays "
                    f"on the light-space shadow lists; in the 32-pixel waves of geometry tiles "
                    f"two adjacent lanes per path (children / triangles / list records split two "
                    f"and two, DPP exchanges); no wave64 compaction of live paths in the timed "
                    f"kernel: the block-compacted (pt_compact) and queue-compacted "
                    f"(RT_PT_QUEUE=1) forms measured slower, DESIGN.md 2.1")
        return (f"{side}x{side} {kind}, tekkaman.cgltrace; {primary}; bounce + shadow rays: "
                f"per-lane {bvh_kind} walk, LDS stack, shadow/bounce lanes paired in the "
                f"32-pixel waves of geometry tiles")
    shadow_how = ("per lane over its light-space cell list (cube map around the light, built "
                  "on the device)" if setup_st["slist_on"]
                  else f"each wave a {bvh_kind} packet walk (stack in one VGPR)")
    return (f"{side}x{side} {'primary+shadow' if shadows else 'primary'} rays, "
            f"tekkaman.cgltrace; {primary}; shadow rays: ballot/mbcnt-compacted into full "
            f"waves, {shadow_how}")


class Watchdog:
    """N > 1: a phase that does not finish in `seconds` (a hung RCCL init or
    first gather) ends the rank with a message and every thread's traceback
    on stderr, exit status 1 (faulthandler), instead of hanging the driver's
    run until its own limit."""

    def __init__(self, on: bool, seconds: float):
        self.on, self.seconds = on, seconds

    def arm(self, what: str):
        if not self.on:
            return
        import faulthandler
        log(f"bench.py: rank {os.environ.get('RANK', '0')}: {what} (watchdog {self.seconds:.0f} s)")
        faulthandler.dump_traceback_later(self.seconds, exit=True)

    def disarm(self):
        if self.on:
            import faulthandler
            faulthandler.cancel_dump_traceback_later()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--size", type=int, default=None,
                    help="frame side (default: 1024 at N=1, config 3; 4096 at N>1, config 5)")
    ap.add_argument("--no-shadows", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-series", action="store_true",
                    help="skip the strong/weak scaling series runs (default at N>1)")
    ap.add_argument("--series", action="store_true",
                    help="N=1: also run the weak-scaling series point (~1024^2 sqrt(N))")
    ap.add_argument("--workload", choices=("shadow", "path", "flat"), default="shadow",
                    help="shadow: BASELINE config 3 (the metric's config, default); "
                         "path: config 4, 4-bounce diffuse path trace; "
                         "flat: config 2, 256^2 primary rays over the flat triangle list")
    ap.add_argument("--bounces", type=int, default=4)
    ap.add_argument("--no-bvh-series", action="store_true",
                    help="N=1: skip the series entries beside the headline (the BVH-walk frame, "
                         "configs 2 / 4 / 5's frame, the moving light)")
    ap.add_argument("--verify-gather", action="store_true",
                    help="N>1: rank 0 checks the gathered frame against its own full render")
    ap.add_argument("--plumbing-check", action="store_true",
                    help="stop after the ranks have joined the communicator: rank 0 prints "
                         "n_gpus / ranks_seen (CPU rehearsal of --gpus with BENCH_DIST_BACKEND=gloo)")
    args = ap.parse_args()
    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and world_env is None:
        sys.exit(launch_ranks(args.gpus))
    world = int(world_env or "1")
    if args.gpus > 1 and world != args.gpus:
        log(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
        sys.exit(2)
    # stdout carries exactly ONE line, the JSON result: anything else the
    # native libraries write to fd 1 (e.g. RCCL's version banner) goes to
    # stderr
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    path = args.workload == "path"
    flat = args.workload == "flat"
    mode = "path" if path else ("flat" if flat else "shadow")
    n_gpus = max(world, 1)
    if args.size is None:
        args.size = 256 if flat else (CONFIG5_SIDE if n_gpus > 1 else 1024)
    if flat:
        args.no_shadows = True
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # BENCH_FORCE_GATHER=1 (under torch.distributed.run): the N>1 exchange
    # path even at world size 1 -- RCCL on one GPU, to test its stream order
    use_gather = world > 1 or os.environ.get("BENCH_FORCE_GATHER") == "1" or args.plumbing_check
    dog = Watchdog(use_gather, float(os.environ.get("BENCH_DIST_TIMEOUT_S", "240")))
    dist = None
    import torch
    # RCCL ("nccl") between the GPUs; BENCH_DIST_BACKEND=gloo rehearses the
    # multi-rank flow with host-staged gathers (e.g. several ranks on one GPU)
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    coll_dev = torch.device("cpu")
    ranks_seen = 1
    if use_gather:
        import datetime
        import torch.distributed as dist
        ndev = torch.cuda.device_count()
        dev_index = local_rank % max(1, ndev)
        if ndev:
            torch.cuda.set_device(dev_index)
        dog.arm(f"joining the {backend} communicator ({world} ranks)")
        timeout = datetime.timedelta(seconds=dog.seconds)
        if backend == "nccl":
            coll_dev = torch.device("cuda", dev_index)
            dist.init_process_group("nccl", device_id=coll_dev, timeout=timeout)
        else:
            dist.init_process_group(backend, timeout=timeout)
        one = torch.ones(1, dtype=torch.float64, device=coll_dev)
        dist.all_reduce(one)  # ranks the communicator actually connects
        ranks_seen = int(one.item())
        dog.disarm()
        if ranks_seen != world:
            log(f"bench.py: communicator sees {ranks_seen} ranks, WORLD_SIZE={world}")
            sys.exit(3)
    if args.plumbing_check:
        if rank == 0:
            os.write(json_fd, (json.dumps({"n_gpus": n_gpus, "ranks_seen": ranks_seen,
                                           "backend": backend, "plumbing_check": True}) + "\n").encode())
        if dist is not None:
            dist.destroy_process_group()
        return
    from skybox_rt_amd import rt

    shadows = not args.no_shadows
    light = rt.DEFAULT_LIGHT
    side = args.size
    scene = rt.Scene.load(SCENE)
    r = rt.Renderer(scene)
    bvh_st = r.bvh_stats()  # the renderer's tree, built on the device at creation
    bvh_first_ms = bvh_st["build_ms"]  # including the build image's first load
    # the same build again (image resident): best of 3, before the renderer is configured
    bvh_rebuild_ms = min(r.build_bvh("sah")["build_ms"] for _ in range(3)) if bvh_st["method"] == 1 else None
    bvh_st = r.bvh_stats()

    def make_run(s, bvh_walk=False, m=None, gather=None):
        m = m or mode
        g = use_gather if gather is None else gather
        return Run(r, rt, dist, coll_dev, rank, n_gpus, s, shadows and m != "flat", light, m == "path",
                   m == "flat", args.bounces, g, bvh_walk)

    dog.arm("the first configure and gather set-up")
    run = make_run(side)
    dog.disarm()
    setup_st = r.setup_stats()  # the timed configuration's records (configure)
    inst = run.inst
    bvh_kind = ("BVH4 (binary16 boxes)" if r.bvh4_f16 else "BVH4") if r.bvh4 else "BVH2"
    node_bytes = (NODE4H_BYTES if r.bvh4_f16 else NODE4_BYTES) if r.bvh4 else NODE_BYTES
    # synchronous frames first (start + wait per frame, simx's blocking
    # start): reported beside the pipelined rate, not as `value`.  200 frames
    # (~5 ms) whatever --steps is: a steadier figure than a few frames, and
    # the device reaches its working clocks before the timed region instead
    # of inside it (at the driver's --steps 20 --warmup 5: 62.3-62.5 Grays/s
    # after 20 of them, 64.2-64.3 after 200 -- DESIGN 6, r05at)
    sync_ms = None
    sync_n = 0
    if not use_gather:
        sync_n = int(os.environ.get("BENCH_SYNC_FRAMES", "0")) or 200
        for _ in range(2):
            r.render()
        t_s = time.perf_counter()
        for _ in range(sync_n):
            r.render()
        sync_ms = (time.perf_counter() - t_s) / sync_n * 1e3
    # a step = one frame: vx_start queues the launch behind the in-flight
    # frame (driver VX_HIP_QUEUE_DEPTH, default 2) so the host's launch and
    # completion-poll overhead overlaps the previous frame; every frame is
    # complete before the timed region ends.  N > 1: the first steps carry
    # the first RCCL gathers (watchdog)
    dog.arm("the timed steps (render + RCCL gather)")
    elapsed = run.timed(args.steps, args.warmup, dist)
    dog.disarm()
    # the kernel's average duration: HIP events around a back-to-back run of
    # the same frames on the driver's stream (Run.kernel_clock)
    # (at least 200 frames after 20 untimed ones: at the driver's 20-step
    # command a 50-frame clock of a 0.03 ms frame is a 1.5 ms burst that
    # still runs below the device's working clock)
    clock_frames = max(200, min(args.steps, 1000))
    clock_warmup = 20
    avg_kernel_ms = run.kernel_clock(clock_frames, clock_warmup)
    st = r.stats()
    elapsed, rays_total = reduce_max_sum(dist, coll_dev, elapsed, run.rays_local)
    ms_per_step = elapsed / args.steps * 1e3
    value = rays_total * args.steps / elapsed / 1e6
    # N > 1: the same steps with only the render, and with only the frame
    # exchange (gather of the last frame + assembly), max over ranks -- which
    # half sets the step time at this N
    split = None
    if use_gather:
        split_steps = max(20, min(args.steps, 500))
        e_r = run.timed(split_steps, 5, dist, exchange=False)
        e_x = run.timed(split_steps, 5, dist, render=False)
        e_r, _ = reduce_max_sum(dist, coll_dev, e_r, 0)
        e_x, _ = reduce_max_sum(dist, coll_dev, e_x, 0)
        split = {"steps": split_steps, "render_ms_per_step": round(e_r / split_steps * 1e3, 5),
                 "exchange_ms_per_step": round(e_x / split_steps * 1e3, 5),
                 "exchange": (f"torch.distributed gather ({'RCCL' if backend == 'nccl' else backend}) "
                              f"of the compact tile buffers + rt_frame_assemble on rank 0, "
                              f"pipelined over 4 slots")}
    gather_ok = None
    if use_gather and args.verify_gather:
        image = run.fg.image.cpu().numpy() if rank == 0 else None
        r.configure(side, side, shadows=shadows, light=light, path=path, bounces=args.bounces,
                    flat=flat)
        if rank == 0:
            r.render()
            full = r.framebuffer().reshape(-1).view(np.int32)
            gather_ok = bool(np.array_equal(image, full))
            log(f"gathered frame == full render: {gather_ok}")
    series = {}

    def timed_series(name, s, m, image, bvh_walk=False, gather=None, note=None):
        """One more configuration timed like `value` (same steps and warm-up),
        with its own kernel clock, roofline and issue roofline (its own PMC
        record); rays summed over the ranks, time the max over the ranks."""
        sr = make_run(s, bvh_walk=bvh_walk, m=m, gather=gather)
        sst = r.setup_stats()
        e = sr.timed(args.steps, args.warmup, dist)
        k = sr.kernel_clock(clock_frames, clock_warmup)
        e, rays = reduce_max_sum(dist, coll_dev, e, sr.rays_local)
        roof, issue = make_roofline(sr.inst, k, "bvh" if bvh_walk else m, s, node_bytes, n_gpus=n_gpus)
        ent = {"workload": describe(s, m, sst, shadows and m != "flat", args.bounces, bvh_kind),
               "image": image, "side": s, "steps": args.steps, "warmup": args.warmup,
               "value": round(rays * args.steps / e / 1e6, 3),
               "ms_per_step": round(e / args.steps * 1e3, 5), "kernel_ms": round(k, 5),
               "rays_per_frame": int(rays), "roofline": roof, "roofline_issue": issue}
        if note:
            ent["note"] = note
        series[name] = ent
        return ent

    # N > 1: config 5's frame on these N GPUs is `value` itself; the weak
    # point (~1M pixels per GPU) beside it.  N = 1 (`--series`): the weak point
    if not args.no_series and not flat and (n_gpus > 1 or args.series):
        if side == CONFIG5_SIDE:
            series["strong_4096"] = {"side": side, "value": round(value, 3),
                                     "ms_per_step": round(ms_per_step, 5), "same_as": "value"}
        s = frame_side(n_gpus, 1024)
        if s != side:
            timed_series("weak_1024_sqrtN", s, mode, "rt_kernel (entry vx_main_rt_kernel)")
    extra = n_gpus == 1 and not args.no_bvh_series
    if extra and mode == "shadow" and shadows:
        # BASELINE config 3 by BVH traversal only (RT_RENDER_BVH_WALK, image
        # rt_bvh: primary visibility by the binary16-BVH4 packet walk, shadow
        # rays by the shadow packet walk; no block or light-space lists)
        b = timed_series("bvh_walk", side, "shadow", "rt_bvh (entry vx_main_rt_bvh)", bvh_walk=True)
        b["workload"] = (f"{side}x{side} primary+shadow rays, tekkaman.cgltrace, BVH traversal only "
                         f"(BASELINE config 3): primary visibility by a {bvh_kind} packet walk per "
                         f"8x8-block wave (raster-exact leaf tests, node/leaf records through the "
                         f"scalar cache, wave stack in one VGPR); shadow rays ballot/mbcnt-compacted "
                         f"into full waves, each a {bvh_kind} any-hit packet walk (its traversal stack "
                         f"in VGPR lanes, v_writelane/v_readlane, not LDS: measured neutral against "
                         f"an LDS stack, DESIGN.md 4.1)")
        # every other single-GPU BASELINE config in the same command, each
        # with its own kernel clock and PMC record: config
        # 4 (path), config 2 (flat), and config 5's 4096^2 frame on this one
        # GPU -- the N = 1 point of the driver's 4096^2 scaling curve
        timed_series("path", 1024, "path", "pt_kernel (entry vx_main_pt_kernel)")
        timed_series("flat", 256, "flat", "rt_flat (entry vx_main_rt_flat)")
        timed_series("strong_4096", CONFIG5_SIDE, "shadow", "rt_kernel (entry vx_main_rt_kernel)",
                     gather=True if os.environ.get("BENCH_FORCE_GATHER") == "1" else False,
                     note="BASELINE config 5's frame (4096^2 primary+shadow) on one GPU, whole frame, "
                          "no exchange: the N = 1 point of the --gpus N scaling curve, whose N > 1 "
                          "lines render this frame tile-sharded")
    # the moving light: a light change + a frame per step (N = 1)
    moving = None
    if extra and not flat and (shadows or path):
        mr = moving_light_series(r, side, args.steps, args.warmup,
                                 dict(shadows=shadows, path=path, bounces=args.bounces))
        mr["value"] = round(run.rays_local * mr["steps"] / (mr["ms_per_step"] * 1e-3 * mr["steps"]) / 1e6, 3)
        mr["workload"] = (f"{side}x{side} {'path trace' if path else 'primary+shadow'} frames, the light "
                          f"moved before every frame (rt_renderer_set_light, no host wait): the frames "
                          f"trace their shadow rays by the BVH4 packet walk while the light moves and "
                          f"the light-space lists are rebuilt on the device only once a light stays; "
                          f"ms_per_step_lists_rebuilt_every_step = the lists rebuilt for every light "
                          f"(6 stream-ordered setup launches before its frame)")
        series["moving_light"] = moving = mr
    cold = None
    if extra and not flat:
        cold = cold_configure_probe(rt, scene, side, dict(shadows=shadows, light=light, path=path,
                                                          bounces=args.bounces))
    if rank != 0:
        dist.destroy_process_group()
        return
    config5 = n_gpus > 1 and side == CONFIG5_SIDE
    what = {"shadow": f"{side}^2 primary+shadow tekkaman",
            "path": f"{side}^2 {args.bounces}-bounce diffuse path trace tekkaman (BASELINE config 4)",
            "flat": f"{side}^2 primary rays, tekkaman flat triangle list, no BVH (BASELINE config 2)"}[mode]
    if n_gpus == 1:
        # BASELINE.json's metric (config 3 at 1024^2)
        metric = f"Mrays/sec per GPU + achieved HBM GB/s, {what}"
    else:
        # `value` is the whole job's rays/s (all ranks' rays over the max
        # rank's time); the per-GPU figure is config.mrays_per_s_per_gpu
        metric = (f"Mrays/sec, all {n_gpus} GPUs (per GPU: config.mrays_per_s_per_gpu) + achieved HBM "
                  f"GB/s, {what}" + (", tile-sharded (BASELINE config 5)" if config5 else ", tile-sharded"))
    workload = describe(side, mode, setup_st, shadows, args.bounces, bvh_kind)
    if n_gpus > 1:
        workload += (f", tile-sharded over {n_gpus} GPUs (32x32 tile t -> rank t mod {n_gpus}) + "
                     f"{'RCCL' if backend == 'nccl' else backend} gather to rank 0"
                     + (" (BASELINE config 5)" if config5 else ""))
    images = None
    if path and setup_st.get("path_queue"):
        images = ("pt_primary.co", "pt_queue.co")  # the two-kernel form (RT_PT_QUEUE=1)
    roof, issue = make_roofline(inst, avg_kernel_ms, mode, side, node_bytes, images, n_gpus)
    info = scene.info()  # (after the timed region: parse time, host-side counts)
    out = {
        "metric": metric,
        "value": round(value, 3),
        "unit": "Mrays/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 5),
        "higher_is_better": True,
        # a fixed frame however many GPUs render it (N = 1: config 3's 1024^2
        # frame; N > 1: config 5's 4096^2 frame dealt over the ranks, whose
        # one-GPU point is series.strong_4096 of the N = 1 line)
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "tekkaman.cgltrace from the reference's regression data (tests/golden/scenes)",
        "config": {
            "workload": workload,
            "scene": "tekkaman.cgltrace", "width": side, "height": side,
            "shadow_rays": shadows, "light_clip_xyw": list(light),
            "parallelism": f"tiles32 mod {n_gpus}" + (f" + {'rccl' if backend == 'nccl' else backend} "
                                                      f"gather" if n_gpus > 1 else ""),
            "ranks_seen": ranks_seen,
            "bvh_nodes": bvh_st["nodes4" if r.bvh4 else "nodes"],
            "bvh_depth": bvh_st["depth4" if r.bvh4 else "depth"],
            # scene parse, BVH build and per-resolution setup
            # are reported separately, outside the timed frames
            "parse_ms": round(info["parse_ms"], 3),
            "bvh_build_ms": round(bvh_first_ms, 3),
            "bvh_rebuild_ms": round(bvh_rebuild_ms, 3) if bvh_rebuild_ms is not None else None,
            "bvh_build_launches": int(bvh_st["launches"]),
            "bvh_build": {0: "device LBVH", 1: "device binned SAH (kernels/bvh_sah.hip)",
                          2: "host binned SAH"}.get(bvh_st["method"], "?"),
            "configure_ms": round(setup_st["configure_ms"], 3),
            # the first configure of the renderer at this size and light:
            # records, block lists, shadow lists, work order (cold)
            "cold_configure_ms": round((cold or run.first_setup)["configure_ms"], 3),
            "cold_configure_setup_ms": round((cold or run.first_setup)["setup_ms"], 3),
            "cold_configure_launches": int((cold or run.first_setup)["launches"]),
            "cold_configure": ("best of 3 fresh renderers (new resolution + new light: records, "
                               "block lists, shadow lists, work order)" if cold else
                               "the renderer's first configure"),
            "first_configure_ms": round(run.first_setup["configure_ms"], 3),
            "slist_build_ms": moving["slist_build_ms"] if moving else None,
            "setup_ms": round(setup_st["setup_ms"], 3),
            "setup": ("device" if setup_st["device"] else "host") + f", {setup_st['launches']} launches",
            "block_list_entries": int(setup_st["blist_entries"]),
            "grid": st["grid"], "block": st["block"],
            "rays_per_frame": int(rays_total),
            "mrays_per_s_per_gpu": round(value / n_gpus, 3),
            "kernel_ms": round(avg_kernel_ms, 5),
            "frames": "back to back (vx_start queues behind the in-flight frames; no per-launch "
                      "events in the timed region); kernel_ms = two HIP events on the driver's "
                      f"stream around {clock_frames} such frames after the "
                      "timed region / frames (render only)",
            "sync_ms_per_step": round(sync_ms, 5) if sync_ms is not None else None,
            "sync_frames": (f"{sync_n} synchronous frames (vx_start + vx_ready_wait each), host "
                            "clock, before the timed region") if sync_ms is not None else None,
            "kernel_mrays_per_s": round(run.rays_local / (avg_kernel_ms * 1e-3) / 1e6, 3),
            "counters": "off in the timed frames (rays per frame from the instrumented pre-run)",
        },
        "series": series,
        "roofline": roof,
        "cpu_baseline": None,
    }
    if issue is not None:
        out["roofline_issue"] = issue
    if gather_ok is not None:
        out["config"]["gather_verified"] = gather_ok
    if split is not None:
        out["config"]["step_split"] = split
    if n_gpus == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(shadows, side, light, args.cpu_budget, path,
                                               args.bounces, flat, r.bvh4)
        except Exception as e:  # the baseline is reported, not required
            log(f"cpu baseline failed: {e}")
    os.write(json_fd, (json.dumps(out) + "\n").encode())
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
