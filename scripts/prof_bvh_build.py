#!/usr/bin/env python3
"""Builds the BVH of a synthetic scene on the GPU `--builds` times (for
rocprofv3 --kernel-trace: 17 vx_main dispatches per build, in phase order:
bounds, morton, 4 x (hist, scan, scatter), tree, boxes, emit)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tris", type=int, default=100000)
    ap.add_argument("--builds", type=int, default=3)
    args = ap.parse_args()
    import torch  # noqa: F401
    from synth_scene import make_scene
    from skybox_rt_amd import rt
    s = rt.Scene.load(make_scene(f"/tmp/prof_synth{args.tris}.cgltrace.gz", args.tris, seed=3, size=0.012))
    r = rt.Renderer(s)
    for _ in range(args.builds):
        print(r.build_bvh())


if __name__ == "__main__":
    main()
