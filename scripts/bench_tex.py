#!/usr/bin/env python3
"""Throughput of the texture regression kernel (tex_kernel.hip, SURVEY.md
8(f) rank 3) on MI355X next to the oracle's C restatement of the
reference's software sampler (oracle/tex.c, single thread, as the
reference's tex kernel runs per core).  One JSON line per case.

Algorithmic HBM bytes per launch = 4 B per destination pixel written + the
bytes of the mip level(s) sampled (read once; every level texel is used when
the destination covers the whole texture).  roofline.frac = that / kernel
time / 8 TB/s."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0


def level_bytes(w, h, fmt, lod):
    stride = 4 if fmt == 0 else 1 if fmt in (5, 6) else 2
    return max(w >> lod, 1) * max(h >> lod, 1) * stride


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--cpu-budget", type=float, default=3.0)
    ap.add_argument("--ab", default="", help="variant directory under lib/variants: time the "
                    "default and that variant's images interleaved (kernel ms only)")
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime)
    from conftest import GOLDEN
    from oracle import py_oracle as po
    from skybox_rt_amd import tex
    rng = np.random.default_rng(7)
    synth = rng.integers(0, 2 ** 32, size=(4096, 4096), dtype=np.uint64).astype(np.uint32)
    rainbow = po.load_png_argb(f"{GOLDEN}/tex/rainbow.png")
    cases = [("synthetic4096 A8R8G8B8 point x1", synth, 0, 0, 0, 1.0),
             ("synthetic4096 R5G6B5 bilinear x0.5", synth, 1, 1, 0, 0.5),
             ("synthetic4096 A8R8G8B8 trilinear x0.37", synth, 0, 2, 1, 0.37),
             ("rainbow256 A8R8G8B8 trilinear x16", rainbow, 0, 2, 0, 16.0),
             ("rainbow256 R5G6B5 bilinear x8 mirror", rainbow, 1, 1, 2, 8.0)]
    a = tex.TexApp()
    if args.ab:
        b = tex.TexApp(os.path.join(ROOT, "skybox_rt_amd", "lib", "variants", args.ab))
        for label, src, fmt, filt, wrap, scale in cases:
            a.configure(src, fmt=fmt, filt=filt, wrap=wrap, scale=scale)
            b.configure(src, fmt=fmt, filt=filt, wrap=wrap, scale=scale)
            ka, kb = [], []
            for _ in range(8):
                for app, ks in ((a, ka), (b, kb)):
                    for _ in range(args.steps // 8 + 1):
                        app.render()
                        ks.append(app.stats()["kernel_ms"])
            same = bool(np.array_equal(a.image(), b.image()))
            print(json.dumps({"case": label, "default_ms": round(float(np.median(ka)), 5),
                              args.ab + "_ms": round(float(np.median(kb)), 5),
                              "identical": same}), flush=True)
        return
    for label, src, fmt, filt, wrap, scale in cases:
        a.configure(src, fmt=fmt, filt=filt, wrap=wrap, scale=scale)
        for _ in range(5):
            a.render()
        ks = []
        t0 = time.perf_counter()
        for _ in range(args.steps):
            a.render()
            ks.append(a.stats()["kernel_ms"])
        wall = (time.perf_counter() - t0) / args.steps * 1e3
        st = a.stats()
        km = float(np.median(ks))
        px = st["dst_width"] * st["dst_height"]
        h, w = src.shape
        alg = 4 * px + level_bytes(w, h, fmt, st["lod"]) + (
            level_bytes(w, h, fmt, min(st["lod"] + 1, 15)) if filt == 2 else 0)
        achieved = alg / (km * 1e-3) / 1e9
        # CPU: the oracle on a bounded band of rows (num_tasks = rows: same per-row coordinates)
        rows = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < args.cpu_budget and rows < st["dst_height"]:
            po.tex_render(src, fmt=fmt, wrap=wrap, filt=filt, scale=scale)
            rows += st["dst_height"]
        cpu_s = time.perf_counter() - t0
        cpu_mpx = rows * st["dst_width"] / cpu_s / 1e6
        ok = None
        if px <= 4096 * 4096:
            ok = bool(np.array_equal(a.image(), po.tex_render(src, fmt=fmt, wrap=wrap, filt=filt,
                                                               scale=scale)))
        print(json.dumps({
            "case": label, "dst": [st["dst_width"], st["dst_height"]], "lod": st["lod"],
            "frac": st["frac"], "kernel_ms": round(km, 5), "wall_ms": round(wall, 4),
            "gpixels_per_s": round(px / km / 1e6, 2),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 3),
                         "algorithmic_bytes": int(alg)},
            "grid": st["grid"], "block": st["block"],
            "cpu_oracle_mpixels_per_s": round(cpu_mpx, 2), "cpu_threads": 1,
            "bit_exact_vs_oracle": ok}), flush=True)


if __name__ == "__main__":
    main()
