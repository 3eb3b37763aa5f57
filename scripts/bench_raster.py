#!/usr/bin/env python3
"""Throughput of the draw3d raster pipeline (raster_kernel.hip, SURVEY.md 8(f)
rank 1) on the GPU next to the oracle's C restatement of the reference's
software path (oracle/raster.c, single-threaded as the reference's draw3d
software path runs per core) on the same scene and size.  One JSON line per
scene."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", default="tekkaman,vase,evilskull,carnival")
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--cpu-frames", type=int, default=1)
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime)
    from conftest import scene_path
    from oracle import py_oracle as po
    from skybox_rt_amd import rt
    for name in args.scenes.split(","):
        s = rt.Scene.load(scene_path(name))
        r = rt.Renderer(s)
        r.configure(args.size, args.size, raster=True)
        for _ in range(5):
            r.render()
        ks = []
        t0 = time.perf_counter()
        for _ in range(args.steps):
            r.render()
            ks.append(r.kernel_ms())
        wall = (time.perf_counter() - t0) / args.steps * 1e3
        st = r.stats()
        osc = po.OracleScene(po.cgltrace.load(scene_path(name)))
        t0 = time.perf_counter()
        for _ in range(args.cpu_frames):
            c, _, _ = po.raster_render(osc, args.size, args.size)
        cpu_ms = (time.perf_counter() - t0) / args.cpu_frames * 1e3
        ok = bool(np.array_equal(c, r.framebuffer()))
        px = args.size * args.size
        km = float(np.median(ks))
        print(json.dumps({
            "scene": name, "size": args.size, "kernel_ms": round(km, 4), "wall_ms": round(wall, 4),
            "mpixels_per_s": round(px / km / 1e3, 1), "fragments": int(st["shaded"]),
            "grid": st["grid"], "block": st["block"],
            "cpu_oracle_ms": round(cpu_ms, 2), "cpu_threads": 1,
            "speedup_vs_cpu": round(cpu_ms / km, 1), "bit_exact_vs_oracle": ok}), flush=True)


if __name__ == "__main__":
    main()
