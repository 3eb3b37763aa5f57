#!/usr/bin/env python3
"""Device SAH build times (kernels/bvh_sah.hip): the renderer's first build
(image load included) and the best of 5 rebuilds, per scene; one JSON line.
Scenes: tekkaman and synthetic ones (tests/synth_scene.py).  The driver's
grid follows env VX_HIP_BLOCKS_PER_CU when set (every image of the process).
--kdir DIR: the build image from DIR (an A/B variant), its arrays compared
with the shipped image's."""
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from skybox_rt_amd import rt  # noqa: E402
from synth_scene import make_scene  # noqa: E402


def main():
    import argparse
    import numpy as np
    ap = argparse.ArgumentParser()
    ap.add_argument("--kdir", default=None)
    args = ap.parse_args()
    out = {"blocks_per_cu": os.environ.get("VX_HIP_BLOCKS_PER_CU", "image"), "kdir": args.kdir}
    tmp = tempfile.mkdtemp()
    scenes = {"tekkaman": os.path.join(ROOT, "tests/golden/scenes/tekkaman.cgltrace")}
    for n in (20000, 100000):
        scenes[f"synth{n // 1000}k"] = make_scene(os.path.join(tmp, f"s{n}.cgltrace.gz"), n, seed=n)
    for name, path in scenes.items():
        s = rt.Scene.load(path)
        r = rt.Renderer(s, kernel_dir=args.kdir) if args.kdir else rt.Renderer(s)
        first = r.bvh_stats()["build_ms"]
        best = min(r.build_bvh("sah")["build_ms"] for _ in range(5))
        out[name] = {"first_ms": round(first, 3), "rebuild_ms": round(best, 3),
                     "launches": r.bvh_stats()["launches"]}
        if args.kdir:
            ref = rt.Renderer(s)
            a, b = r.export_bvh(), ref.export_bvh()
            out[name]["equal"] = bool(
                np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32))
                and np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32))
                and np.array_equal(r.export_bvh4().view(np.uint32), ref.export_bvh4().view(np.uint32))
                and np.array_equal(r.export_bvh4h(), ref.export_bvh4h()))
            ref.close()
        r.close()
        s.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
