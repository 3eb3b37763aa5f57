#!/usr/bin/env python3
"""Render N frames of the benchmark workload (for rocprofv3 passes)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--no-shadows", action="store_true")
    ap.add_argument("--kernel-dir", default=None)
    ap.add_argument("--mode", choices=("shadow", "path", "flat", "bvh"), default="shadow",
                    help="bvh: config 3 by BVH traversal only (RT_RENDER_BVH_WALK, image rt_bvh)")
    ap.add_argument("--counters", action="store_true",
                    help="counter rows on (default off: the timed product configuration)")
    args = ap.parse_args()
    import torch  # noqa: F401
    from skybox_rt_amd import rt
    s = rt.Scene.load(os.path.join(ROOT, "tests/golden/scenes/tekkaman.cgltrace"))
    r = rt.Renderer(s, kernel_dir=args.kernel_dir)
    flat = args.mode == "flat"
    size = 256 if flat and args.size == 1024 else args.size   # bench.py's config-2 size
    r.configure(size, size, shadows=not (args.no_shadows or flat), path=args.mode == "path",
                flat=flat, counters=args.counters, bvh_walk=args.mode == "bvh")
    for _ in range(args.frames):
        r.render()
    print(r.stats(), file=sys.stderr)


if __name__ == "__main__":
    main()
