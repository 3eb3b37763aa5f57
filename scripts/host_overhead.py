#!/usr/bin/env python3
"""Break down the host-side cost of one frame (vx_start + vx_ready_wait)
against the kernel's HIP-event time: render() loop, start()/wait() split,
kernel_ms() query.  Prints one JSON line (microseconds)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401
    from skybox_rt_amd import rt
    s = rt.Scene.load(os.path.join(ROOT, "tests/golden/scenes/tekkaman.cgltrace"))
    r = rt.Renderer(s)
    r.configure(int(sys.argv[1]) if len(sys.argv) > 1 else 1024,
                int(sys.argv[1]) if len(sys.argv) > 1 else 1024, shadows=True)
    for _ in range(20):
        r.render()
    n = 200
    out = {}
    t = []
    for _ in range(n):
        t0 = time.perf_counter(); r.render(); t.append(time.perf_counter() - t0)
    out["render_us"] = float(np.median(t)) * 1e6
    ts, tw, tk = [], [], []
    for _ in range(n):
        t0 = time.perf_counter(); r.start(); t1 = time.perf_counter(); r.wait(); t2 = time.perf_counter()
        k = r.kernel_ms(); t3 = time.perf_counter()
        ts.append(t1 - t0); tw.append(t2 - t1); tk.append(k)
        out.setdefault("kms_us", []).append(t3 - t2)
    out["start_us"] = float(np.median(ts)) * 1e6
    out["wait_us"] = float(np.median(tw)) * 1e6
    out["kernel_us"] = float(np.median(tk)) * 1e3
    out["kms_us"] = float(np.median(out["kms_us"])) * 1e6
    print(json.dumps({k: round(v, 2) for k, v in out.items()}))


if __name__ == "__main__":
    main()
