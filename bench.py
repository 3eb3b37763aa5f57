#!/usr/bin/env python3
"""bench.py -- headline benchmark: Mrays/s of the MI355X ray-tracing hot path.

Workload (BASELINE.json configs[2], the metric's config): tekkaman.cgltrace,
1024x1024, one primary ray per pixel + one any-hit shadow ray per geometry
hit, BVH traversal with the per-wave LDS stack.  A "step" is one full frame:
vx_start + vx_ready_wait of the RT kernel image through libvortex-hip.so
(inputs already resident in HBM).  With N GPUs (torchrun, one rank per GPU)
the frame grows to ~1024*sqrt(N) on a side (weak scaling: ~1M pixels per
GPU), 32x32 tiles are dealt tile t -> rank t % N, and each step ends with an
RCCL gather of the compact tile buffers to rank 0 plus a de-interleave there
(SURVEY.md 8(e)).

Rank 0 prints one JSON line.  Everything else goes to stderr.
"""
from __future__ import annotations

import argparse
import json
import math
import os
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


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def algorithmic_bytes(st: dict, pixels: int, node_bytes: int = NODE_BYTES) -> int:
    """node bytes (64 B BVH2, 112 B BVH4, 64 B binary16 BVH4) x nodes visited + 36 B x triangles tested
    (BVH leaves and screen layers) + texel bytes per shaded pixel + 4 B per
    pixel written.  Counts come from the instrumented kernel variant, whose
    counters tests/test_gpu_rt.py checks equal to the oracle's traversal."""
    return (node_bytes * st["node_visits"] + TRI_BYTES * (st["tri_tests"] + st["layer_tests"])
            + st["texel_bytes"] + PIXEL_BYTES * pixels)


def pmc_traffic(side: int, shadows: bool, mode: str = "shadow"):
    """HBM bytes per launch from the committed rocprofv3 PMC summary
    (scripts/pmc_traffic.sh -> profiles/pmc_traffic[_path|_flat].json), used
    only when it was taken on this same kernel image and workload; else None."""
    import hashlib
    name, image = {"shadow": ("pmc_traffic.json", "rt_kernel.co"),
                   "path": ("pmc_traffic_path.json", "pt_kernel.co"),
                   "flat": ("pmc_traffic_flat.json", "rt_flat.co")}[mode]
    path = os.path.join(ROOT, "profiles", name)
    co = os.path.join(ROOT, "skybox_rt_amd", "lib", image)
    try:
        with open(path) as fh:
            t = json.load(fh)
        md5 = hashlib.md5(open(co, "rb").read()).hexdigest()
    except (OSError, ValueError):
        return None
    if (t.get("kernel_md5") != md5 or t.get("width") != side or t.get("height") != side
            or t.get("shadows") != shadows):
        return None
    return int(t["traffic_bytes"])


def frame_side(n_gpus: int, base: int) -> int:
    return max(32, int(round(base * math.sqrt(n_gpus) / 32.0)) * 32)


def cpu_baseline(shadows: bool, side: int, light, budget_s: float, path: bool = False,
                 bounces: int = 4, flat: bool = False, bvh4: bool = True):
    """Oracle (C port of the same algorithm, oracle/rt.c) on the host cores,
    BVH traversal identical to the kernel's, full frames until budget_s."""
    from oracle import py_oracle as po
    from skybox_rt_amd import rt as rtmod
    cores = max(1, min(16, os.cpu_count() or 1))
    osc = po.OracleScene(po.cgltrace.load(SCENE))
    sc = rtmod.Scene.load(SCENE)
    bvh = sc.bvh() + ((sc.bvh4(),) if bvh4 else ())
    p = po.rt_params(side, side, shadows=shadows, light=light, nthreads=cores, path=path,
                     bounces=bounces)
    frames, rays, t0 = 0, 0, time.perf_counter()
    while True:
        _, _, _, k = po.rt_render(osc, p, bvh=None if flat else bvh)
        frames += 1
        rays += k["primary_rays"] + k["shadow_rays"] + k["bounce_rays"]
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    value = rays / el / 1e6
    # the same port on ONE thread (single-threaded and all
    # cores; outputs are bit-identical for any thread count), a quarter of
    # the budget, at least one frame
    p1 = po.rt_params(side, side, shadows=shadows, light=light, nthreads=1, path=path,
                      bounces=bounces)
    frames1, rays1, t1 = 0, 0, time.perf_counter()
    while True:
        _, _, _, k = po.rt_render(osc, p1, bvh=None if flat else bvh)
        frames1 += 1
        rays1 += k["primary_rays"] + k["shadow_rays"] + k["bounce_rays"]
        el1 = time.perf_counter() - t1
        if el1 >= budget_s / 4:
            break
    cpu_model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            cpu_model = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")),
                             cpu_model)
    except OSError:
        pass
    return {"value": value, "unit": "Mrays/s", "cores": cores, "kind": "port",
            "sample": f"{frames} full {side}x{side} frames of the same workload "
                      f"({el:.1f} s, oracle/rt.c {'brute force' if flat else ('BVH4' if bvh4 else 'BVH2') + ' traversal'}, "
                      f"{cores} threads; single thread: {frames1} frames in {el1:.1f} s)",
            "single_thread_value": rays1 / el1 / 1e6, "cpu_model": cpu_model,
            "host_cpus": os.cpu_count()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--no-shadows", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workload", choices=("shadow", "path", "flat"), default="shadow",
                    help="shadow: BASELINE config 3 (the metric's config, default); "
                         "path: config 4, 4-bounce diffuse path trace; "
                         "flat: config 2, 256^2 primary rays over the flat triangle list")
    ap.add_argument("--bounces", type=int, default=4)
    ap.add_argument("--verify-gather", action="store_true",
                    help="N>1: rank 0 checks the gathered frame against its own full render")
    args = ap.parse_args()
    # stdout carries exactly ONE line, the JSON result: anything else the
    # native libraries write to fd 1 (e.g. RCCL's version banner) goes to
    # stderr
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    path = args.workload == "path"
    flat = args.workload == "flat"
    if flat and args.size == 1024:
        args.size = 256  # config 2 resolution
    if flat:
        args.no_shadows = True
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    n_gpus = max(world, 1)
    # BENCH_FORCE_GATHER=1 (under torch.distributed.run): the N>1 exchange
    # path even at world size 1 -- RCCL on one GPU, to test its stream order
    use_gather = world > 1 or os.environ.get("BENCH_FORCE_GATHER") == "1"
    dist = None
    import torch
    # RCCL ("nccl") between the GPUs; BENCH_DIST_BACKEND=gloo rehearses the
    # multi-rank flow with host-staged gathers (e.g. several ranks on one GPU)
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    coll_dev = torch.device("cpu")
    if use_gather:
        import torch.distributed as dist
        dev_index = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev_index)
        if backend == "nccl":
            coll_dev = torch.device("cuda", dev_index)
            dist.init_process_group("nccl", device_id=coll_dev)
        else:
            dist.init_process_group(backend)
    from skybox_rt_amd import rt

    shadows = not args.no_shadows
    light = rt.DEFAULT_LIGHT
    side = args.size if n_gpus == 1 else frame_side(n_gpus, args.size)
    scene = rt.Scene.load(SCENE)
    info = scene.info()
    r = rt.Renderer(scene)

    # algorithmic bytes per launch from the instrumented variant (untimed)
    r.configure(side, side, shadows=shadows, light=light, shard_index=rank, shard_count=n_gpus,
                instrumented=True, path=path, bounces=args.bounces, flat=flat)
    r.render()
    inst = r.stats()
    pixels_local = inst["primary_rays"]
    bvh_kind = ("BVH4 (binary16 boxes)" if r.bvh4_f16 else "BVH4") if r.bvh4 else "BVH2"
    alg_bytes = algorithmic_bytes(inst, pixels_local, (NODE4H_BYTES if r.bvh4_f16 else NODE4_BYTES)
                                  if r.bvh4 else NODE_BYTES)

    r.configure(side, side, shadows=shadows, light=light, shard_index=rank, shard_count=n_gpus,
                path=path, bounces=args.bounces, flat=flat, compact=use_gather)
    gather = None
    if use_gather:
        import ctypes
        from skybox_rt_amd.shard import FrameGather
        hip = ctypes.CDLL("libamdhip64.so.7")  # torch's runtime, already loaded
        fg_slots = 4
        fg = FrameGather(dist, side, side, coll_dev, slots=fg_slots)
        dev_ptr, nbytes = r.framebuffer_device()
        kind = 3 if coll_dev.type == "cuda" else 2  # hipMemcpyDeviceToDevice / ToHost

        nsteps = [0]
        if kind == 3:
            drv_stream = torch.cuda.ExternalStream(r.device_stream())
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
            slot = nsteps[0] % fg_slots
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

    # a step = one frame: vx_start queues the launch behind the in-flight
    # frame (driver VX_HIP_QUEUE_DEPTH, default 2) so the host's launch and
    # completion-poll overhead overlaps the previous frame; every frame is
    # complete before the timed region ends (wait + synchronize below)
    def step():
        r.start()
        if gather is not None:
            gather()

    # synchronous frames first (start + wait per frame, simx's blocking
    # start): reported beside the pipelined rate, not as `value`
    sync_n = max(5, min(args.steps, 50))
    for _ in range(2):
        r.render()
    t_s = time.perf_counter()
    for _ in range(sync_n):
        r.render()
    sync_ms = (time.perf_counter() - t_s) / sync_n * 1e3
    for _ in range(args.warmup):
        step()
    r.wait()
    if gather is not None:
        for slot in range(fg_slots):
            fg.reclaim(slot)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    ms0, nt0, n0 = r.run_totals()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    r.wait()
    if gather is not None:  # every frame gathered and assembled inside the timed region
        for slot in range(fg_slots):
            fg.reclaim(slot)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ms1, nt1, n1 = r.run_totals()
    assert n1 - n0 == args.steps and nt1 > nt0, (n0, n1, nt0, nt1)
    st = r.stats()
    rays_local = st["primary_rays"] + st["shadow_rays"] + st["bounce_rays"]
    if dist is not None:
        t = torch.tensor([elapsed, float(rays_local)], dtype=torch.float64, device=coll_dev)
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = t.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed, rays_total = float(mx[0]), float(sm[1])
    else:
        rays_total = float(rays_local)
    ms_per_step = elapsed / args.steps * 1e3
    value = rays_total * args.steps / elapsed / 1e6
    # HIP-event time of the timed launches of the timed region (one in
    # VX_HIP_TIME_EVERY of the queued frames carries events)
    avg_kernel_ms = (ms1 - ms0) / (nt1 - nt0)
    timed_launches = nt1 - nt0
    achieved = alg_bytes / (avg_kernel_ms * 1e-3) / 1e9
    gather_ok = None
    if gather is not None and args.verify_gather and rank == 0:
        r.configure(side, side, shadows=shadows, light=light, path=path, bounces=args.bounces,
                    flat=flat)
        r.render()
        full = r.framebuffer().reshape(-1).view(np.int32)
        gather_ok = bool(np.array_equal(fg.image.cpu().numpy(), full))
        log(f"gathered frame == full render: {gather_ok}")
    if rank != 0:
        dist.destroy_process_group()
        return
    metric = "Mrays/sec per GPU + achieved HBM GB/s, 1024^2 primary+shadow tekkaman"
    kind = "primary+shadow rays"
    if path:
        metric = (f"Mrays/sec per GPU + achieved HBM GB/s, 1024^2 {args.bounces}-bounce diffuse "
                  f"path trace tekkaman (BASELINE config 4)")
        kind = f"{args.bounces}-bounce diffuse path trace (primary + bounce + shadow rays)"
    if flat:
        metric = (f"Mrays/sec per GPU + achieved HBM GB/s, {side}^2 primary rays, tekkaman flat "
                  f"triangle list, no BVH (BASELINE config 2)")
        kind = "primary rays, flat triangle list (no BVH, LDS-staged)"
    out = {
        "metric": metric,
        "value": round(value, 3),
        "unit": "Mrays/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "tekkaman.cgltrace from the reference's regression data (tests/golden/scenes)",
        "config": {
            "workload": (f"{side}x{side} {kind}, tekkaman.cgltrace" if flat else
                         f"{side}x{side} {kind}, tekkaman.cgltrace, {bvh_kind} + LDS stack" if path else
                         f"{side}x{side} {'primary+shadow' if shadows else 'primary'} rays, "
                         f"tekkaman.cgltrace, {bvh_kind} + LDS stack"),
            "scene": "tekkaman.cgltrace", "width": side, "height": side,
            "shadow_rays": shadows, "light_clip_xyw": list(light),
            "parallelism": f"tiles32 mod {n_gpus}" + (f" + {'rccl' if backend == 'nccl' else backend} "
                                                      f"gather" if n_gpus > 1 else ""),
            "bvh_nodes": info["bvh4_nodes" if r.bvh4 else "bvh_nodes"],
            "bvh_depth": info["bvh4_depth" if r.bvh4 else "bvh_depth"],
            "grid": st["grid"], "block": st["block"],
            "rays_per_frame": int(rays_total),
            "mrays_per_s_per_gpu": round(value / n_gpus, 3),
            "kernel_ms": round(avg_kernel_ms, 5),
            "frames": "queued (vx_start behind the in-flight frame, depth "
                      f"{os.environ.get('VX_HIP_QUEUE_DEPTH', '2')}); kernel_ms = HIP events on "
                      f"{timed_launches} of the {args.steps} timed launches",
            "sync_ms_per_step": round(sync_ms, 5),
            "kernel_mrays_per_s": round(rays_local / (avg_kernel_ms * 1e-3) / 1e6, 3),
        },
        "roofline": {
            "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": pmc_traffic(side, shadows, "path" if path else ("flat" if flat else "shadow")),
            "algorithmic_bytes_per_launch": int(alg_bytes),
            "counts": {k: int(inst[k]) for k in ("node_visits", "tri_tests", "layer_tests",
                                                 "texel_bytes", "primary_rays", "shadow_rays",
                                                 "bounce_rays")},
        },
        "cpu_baseline": None,
    }
    if flat:
        # the flat list is read from LDS, never from HBM: its bound is the MT
        # arithmetic -- SURVEY 8(d): ~40 fp32 ops per test, 157.3 TFLOP/s vector peak
        tflops = MT_FLOPS * (inst["tri_tests"] + inst["layer_tests"]) / (avg_kernel_ms * 1e-3) / 1e12
        out["roofline"].update({"bound": "valu", "achieved": round(tflops, 3),
                                "peak": FP32_VALU_TFLOPS, "unit": "TFLOP/s",
                                "frac": round(tflops / FP32_VALU_TFLOPS, 4),
                                "lds_bytes_per_launch": int(alg_bytes)})
        out["roofline"].pop("algorithmic_bytes_per_launch")
    if gather_ok is not None:
        out["config"]["gather_verified"] = gather_ok
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
