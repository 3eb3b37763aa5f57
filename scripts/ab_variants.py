#!/usr/bin/env python3
"""Interleaved A/B timing of kernel-image variants in one process on one GPU
(cdna_hip_programming.md section 5.4 rule 24): per round each variant's
back-to-back frames (the bench's kernel clock: events on the driver's stream
around `frames` launches with per-launch timing off) and three synchronous
frames' device times.

A variant is `label=dir[:ENV=VAL[:ENV=VAL...]]`, where `dir` is `default`
(skybox_rt_amd/lib) or a directory name under skybox_rt_amd/lib/variants and
the ENV settings are applied while that variant's device is opened (e.g.
VX_HIP_BLOCKS_PER_CU).  A bare name means `name=name`.  Every variant must
render the identical framebuffer (checked against the first); prints median /
min kernel ms per variant as one JSON line."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse(spec):
    label, _, rest = spec.partition("=")
    if not rest:
        rest = label
    parts = rest.split(":")
    env = dict(p.split("=", 1) for p in parts[1:])
    return label, parts[0], env


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--scene", default=os.path.join(ROOT, "tests/golden/scenes/tekkaman.cgltrace"))
    ap.add_argument("--variants", default="")
    ap.add_argument("--no-shadows", action="store_true")
    ap.add_argument("--mode", choices=("shadow", "path", "flat", "raster"), default="shadow")
    ap.add_argument("--bounces", type=int, default=4)
    ap.add_argument("--bvh-walk", action="store_true", help="config 3 by BVH traversal only (rt_bvh)")
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime)
    from skybox_rt_amd import rt
    lib = os.path.join(ROOT, "skybox_rt_amd", "lib")
    vdir = os.path.join(lib, "variants")
    specs = args.variants.split(",") if args.variants else sorted(os.listdir(vdir))
    scene = rt.Scene.load(args.scene)
    rs, ref, names = {}, None, []
    for spec in specs:
        label, d, env = parse(spec)
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        # the scene (and its BVH: RT_BVH_* build knobs) is built under the variant's env
        sc = rt.Scene.load(args.scene) if any(k.startswith("RT_BVH_") for k in env) else scene
        r = rt.Renderer(sc, kernel_dir=lib if d == "default" else os.path.join(vdir, d))
        r.configure(args.size, args.size, shadows=not args.no_shadows, path=args.mode == "path",
                    flat=args.mode == "flat", raster=args.mode == "raster", bounces=args.bounces, bvh_walk=args.bvh_walk,
                    counters=False)  # the timed product configuration
        r.render()  # the driver reads its launch env when it loads the image
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        fb = r.framebuffer()
        if ref is None:
            ref = fb
        same = bool(np.array_equal(fb, ref))
        if not same and "RT_TILE_LIMIT" not in env and not d.startswith("x"):  # x*: ablations
            raise SystemExit(f"variant {label} renders a different frame")
        print(f"{label}: identical={same} stats={r.stats()}", file=sys.stderr)
        rs[label] = r
        names.append(label)
    times = {n: [] for n in names}
    sync = {n: [] for n in names}
    host = {n: [] for n in names}
    for _ in range(args.rounds):
        for n in names:
            r = rs[n]
            # back-to-back frames (no per-launch events, the bench's kernel
            # clock): two events on the driver's stream around them / frames
            times[n].append(back_to_back_ms(r, max(args.frames, 20)))
            for _ in range(3):  # and a synchronous frame's device time (completion stamps)
                r.render()
                sync[n].append(r.kernel_ms())
            t0 = time.perf_counter()  # the host's view of 10 synchronous frames (start + wait)
            for _ in range(10):
                r.render()
            host[n].append((time.perf_counter() - t0) / 10 * 1e3)
    out = {n: {"median_ms": round(float(np.median(t)), 5), "min_ms": round(float(np.min(t)), 5),
               "sync_median_ms": round(float(np.median(sync[n])), 5),
               "sync_host_median_ms": round(float(np.median(host[n])), 5),
               "grid": rs[n].stats()["grid"]} for n, t in times.items()}
    print(json.dumps(out))


def back_to_back_ms(r, frames):
    import torch
    stream = torch.cuda.ExternalStream(r.device_stream())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    r.set_timing(False)
    try:
        for _ in range(3):
            r.start()
        r.wait()
        e0.record(stream)
        for _ in range(frames):
            r.start()
        e1.record(stream)
        r.wait()
        e1.synchronize()
    finally:
        r.set_timing(True)
    return e0.elapsed_time(e1) / frames


if __name__ == "__main__":
    main()
