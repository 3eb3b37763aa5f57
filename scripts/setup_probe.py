#!/usr/bin/env python3
"""Configure-time probe: the per-resolution and per-light
setup of rt_renderer_configure on the device, cold and warm.

Sequence (tekkaman, one renderer): 1024^2 with light A (cold: new
resolution, new light), 1024^2 with light B (new light only: the shadow
lists), light B again (nothing new), 4096^2 with light A (cold), then
`--moving N` configures at 1024^2 with a new light each (the moving-light
regime: only the shadow lists rebuild), then as many rt_renderer_set_light changes (each waited
for and timed).  Prints one JSON line with every
configure's setup_stats.  Run with RT_SETUP_TRACE=1 for the per-launch
phases on stderr, under rocprofv3 --kernel-trace for their device times
(vx_main_rt_setup dispatches in launch order)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--moving", type=int, default=8)
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime)
    from skybox_rt_amd import rt
    s = rt.Scene.load(os.path.join(ROOT, "tests/golden/scenes/tekkaman.cgltrace"))
    r = rt.Renderer(s)
    la, lb = (0.0, 60.0, 80.0), (20.0, 50.0, 85.0)
    out = []

    def conf(tag, side, light):
        print(f"== {tag}", file=sys.stderr, flush=True)
        r.configure(side, side, shadows=True, light=light, counters=False)
        st = r.setup_stats()
        r.render()
        out.append({"tag": tag, "side": side, "light": list(light),
                    **{k: (round(v, 4) if isinstance(v, float) else v) for k, v in st.items()}})

    conf("cold_1024", 1024, la)
    conf("new_light_1024", 1024, lb)
    conf("cached_1024", 1024, lb)
    conf("cold_4096", 4096, la)
    for i in range(args.moving):
        conf(f"moving_{i}", 1024, (10.0 * (i % 5) - 20.0, 60.0 - i, 80.0 + 0.5 * i))
    # set_light: the shadow lists alone, queued (then waited for, timed)
    import time
    r.configure(1024, 1024, shadows=True, light=la, counters=False)
    r.render()
    for i in range(args.moving):
        L = (10.0 * (i % 5) - 20.0, 60.0 - i, 80.0 + 0.5 * i)
        print(f"== set_light_{i}", file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        r.set_light(L)
        r.wait()
        dt = (time.perf_counter() - t0) * 1e3
        st = r.setup_stats()
        out.append({"tag": f"set_light_{i}", "light": list(L), "set_light_wait_ms": round(dt, 4),
                    "slist_entries": st["slist_entries"], "slist_on": st["slist_on"]})
    print(json.dumps(out))
    r.close()
    s.close()


if __name__ == "__main__":
    main()
