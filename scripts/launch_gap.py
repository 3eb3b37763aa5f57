#!/usr/bin/env python3
"""Frame-loop cost per frame for the driver's launch modes (diagnostic):
K back-to-back vx_start calls + one wait, wall ms per frame.  Run once per
VX_HIP_EXT_LAUNCH / VX_HIP_QUEUE_DEPTH / VX_HIP_TIME_EVERY setting (read when the device opens)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401
    from skybox_rt_amd import rt
    mode = sys.argv[1] if len(sys.argv) > 1 else "shadow"
    scene = rt.Scene.load(os.path.join(ROOT, "tests/golden/scenes/tekkaman.cgltrace"))
    r = rt.Renderer(scene)
    r.configure(1024, 1024, shadows=True, path=mode == "path")
    for _ in range(20):
        r.start()
    r.wait()
    out = {}
    for k in (50, 300):
        t0 = time.perf_counter()
        for _ in range(k):
            r.start()
        r.wait()
        out[f"ms_per_frame_{k}"] = round((time.perf_counter() - t0) / k * 1e3, 5)
    ms, nt, n = r.run_totals()
    out["kernel_ms_avg"] = round(ms / nt, 5) if nt else None
    out["timed"], out["runs"] = nt, n
    out.update(mode=mode, launch=os.environ.get("VX_HIP_EXT_LAUNCH", "1"),
               depth=os.environ.get("VX_HIP_QUEUE_DEPTH", "2"),
               time_every=os.environ.get("VX_HIP_TIME_EVERY", "4"))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
