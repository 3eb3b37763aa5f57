#!/usr/bin/env python3
"""GPU BVH build times -- the LBVH (kernels/bvh_build.hip, 19 launches incl.
the BVH4 collapse and its binary16 planes) and the binned-SAH restatement of
the host builder (kernels/bvh_sah.hip, one launch per level + 8; the host's
arrays bit for bit) -- vs the host binned-SAH build (app/bvh.cpp) on the
same triangles, and the traced frame time over each tree.  One JSON line per
scene."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def frame_ms(r, n=20):
    for _ in range(3):
        r.render()
    ks = []
    for _ in range(n):
        r.render()
        ks.append(r.kernel_ms())
    ks.sort()
    return ks[len(ks) // 2]


def main():
    import torch  # noqa: F401
    from conftest import scene_path
    from synth_scene import make_scene
    from skybox_rt_amd import rt
    scenes = [("tekkaman", scene_path("tekkaman")), ("scene", scene_path("scene")),
              ("synth20k", make_scene("/tmp/bench_synth20k.cgltrace.gz", 20000)),
              ("synth100k", make_scene("/tmp/bench_synth100k.cgltrace.gz", 100000, seed=3,
                                       size=0.012))]
    for name, path in scenes:
        s = rt.Scene.load(path)
        info = s.info()
        r = rt.Renderer(s)
        r.configure(1024, 1024, shadows=True)
        host_ms = frame_ms(r)
        r2 = rt.Renderer(s)
        r2.configure(1024, 1024, shadows=True, bvh_width=2)
        host2_ms = frame_ms(r2)
        builds = [r.build_bvh() for _ in range(5)]
        gpu_ms = frame_ms(r)            # over the device BVH4 collapse
        r3 = rt.Renderer(s)
        r3.configure(1024, 1024, shadows=True, bvh_width=2)
        r3.build_bvh()
        gpu2_ms = frame_ms(r3)          # over the device BVH2
        b = sorted(builds, key=lambda x: x["build_ms"])[len(builds) // 2]
        r4 = rt.Renderer(s)
        r4.configure(1024, 1024, shadows=True)
        sah = [r4.build_bvh("sah") for _ in range(5)]
        sah_ms = frame_ms(r4)           # over the device SAH tree (== the host tree)
        bs = sorted(sah, key=lambda x: x["build_ms"])[len(sah) // 2]
        print(json.dumps({"scene": name, "triangles": info["num_geometry"],
                          "host_sah_build_ms": round(info["bvh_ms"], 3),
                          "gpu_build_ms": round(b["build_ms"], 3),
                          "gpu_build_kernel_ms": round(b["kernel_ms"], 3),
                          "gpu_launches": b["launches"], "gpu_depth": b["depth"],
                          "gpu_stack4": b["stack4"],
                          "host_depth": info["bvh_depth"],
                          "frame_ms_host_bvh4": round(host_ms, 4),
                          "frame_ms_host_bvh2": round(host2_ms, 4),
                          "frame_ms_gpu_lbvh4": round(gpu_ms, 4),
                          "frame_ms_gpu_lbvh2": round(gpu2_ms, 4),
                          "gpu_sah_build_ms": round(bs["build_ms"], 3),
                          "gpu_sah_build_kernel_ms": round(bs["kernel_ms"], 3),
                          "gpu_sah_launches": bs["launches"],
                          "frame_ms_gpu_sah4": round(sah_ms, 4)}), flush=True)


if __name__ == "__main__":
    main()
