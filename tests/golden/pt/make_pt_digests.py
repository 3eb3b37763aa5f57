#!/usr/bin/env python3
"""Regenerate tests/golden/pt/pt_digests.json: SHA-256 of the path-trace
oracle's framebuffer (uint32 ARGB, row 0 = bottom) plus its ray counters for
a few small cases.  Run only when the documented estimator (DESIGN.md "Path
tracing") changes on purpose."""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ.setdefault("SKYBOX_RT_NO_TORCH", "1")

from conftest import scene_path  # noqa: E402
from oracle import py_oracle as po  # noqa: E402
from skybox_rt_amd import rt  # noqa: E402

CASES = [("tekkaman", 128, 4, 0x5EED), ("tekkaman", 96, 1, 7), ("box", 64, 4, 0x5EED),
         ("scene", 64, 2, 0x5EED)]
KEYS = ("primary_rays", "shadow_rays", "geometry_hits", "occluded", "bounce_rays")


def main():
    out = []
    for name, size, bounces, seed in CASES:
        osc = po.OracleScene(po.cgltrace.load(scene_path(name)))
        bvh = rt.Scene.load(scene_path(name)).bvh()
        c, _, _, k = po.rt_render(osc, po.rt_params(size, size, path=True, bounces=bounces,
                                                    seed=seed, nthreads=8), bvh=bvh)
        out.append({"scene": name, "size": size, "bounces": bounces, "seed": seed,
                    "sha256": hashlib.sha256(np.ascontiguousarray(c).tobytes()).hexdigest(),
                    "counters": {key: k[key] for key in KEYS}})
    with open(os.path.join(HERE, "pt_digests.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
