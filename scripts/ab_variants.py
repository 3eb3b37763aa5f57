#!/usr/bin/env python3
"""Interleaved A/B timing of kernel-image variants (skybox_rt_amd/lib/variants/*)
in one process on one GPU (cdna_hip_programming.md section 5.4 rule 24).
Each variant must render the identical framebuffer (checked against the
first); prints median / min kernel ms per variant."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--scene", default=os.path.join(ROOT, "tests/golden/scenes/tekkaman.cgltrace"))
    ap.add_argument("--variants", default="")
    ap.add_argument("--no-shadows", action="store_true")
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime)
    from skybox_rt_amd import rt
    vdir = os.path.join(ROOT, "skybox_rt_amd", "lib", "variants")
    names = args.variants.split(",") if args.variants else sorted(os.listdir(vdir))
    scene = rt.Scene.load(args.scene)
    rs, ref = {}, None
    for n in names:
        r = rt.Renderer(scene, kernel_dir=os.path.join(vdir, n))
        r.configure(args.size, args.size, shadows=not args.no_shadows)
        r.render()
        fb = r.framebuffer()
        if ref is None:
            ref = fb
        same = bool(np.array_equal(fb, ref))
        print(f"{n}: identical={same} stats={r.stats()}", file=sys.stderr)
        rs[n] = r
    times = {n: [] for n in names}
    for _ in range(args.rounds):
        for n in names:
            r = rs[n]
            for _ in range(args.frames):
                r.render()
                times[n].append(r.stats()["kernel_ms"])
    out = {n: {"median_ms": float(np.median(t)), "min_ms": float(np.min(t)),
               "grid": rs[n].stats()["grid"]} for n, t in times.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
