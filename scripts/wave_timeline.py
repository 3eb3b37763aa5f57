#!/usr/bin/env python3
"""Per-wave timeline of one RT frame from the RT_STAMPS diagnostic image
(skybox_rt_amd/lib/variants/stamp): every one-wave workgroup records its start
(s_memrealtime, 100 MHz), duration and placement in its counter row.  Prints a
JSON summary: kernel span, wave-lifetime distribution, slot utilisation over
time, the tail, and the lifetime of model vs background waves.  Timing-only
diagnostic; the stamps never reach an output value."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    path = len(sys.argv) > 2 and sys.argv[2] == "path"   # pt_kernel (variants/ptstamp)
    bvh = len(sys.argv) > 2 and sys.argv[2] == "bvh"     # rt_bvh (variants/stamp): config 3 by BVH walks
    import torch  # noqa: F401
    from skybox_rt_amd import rt
    kdir = os.path.join(ROOT, "skybox_rt_amd/lib/variants", "ptstamp" if path else "stamp")
    image = os.path.join(kdir, "pt_kernel.vxbin" if path else ("rt_bvh.vxbin" if bvh else "rt_kernel.vxbin"))
    if not os.path.exists(image):  # the renderer would fall back to the stamp-less product image
        sys.exit(f"wave_timeline: {image} missing (make -C skybox_rt_amd/csrc diag)")
    s = rt.Scene.load(os.path.join(ROOT, "tests/golden/scenes/tekkaman.cgltrace"))
    r = rt.Renderer(s, kernel_dir=kdir)
    r.configure(size, size, shadows=True, path=path, bvh_walk=bvh)
    for _ in range(5):
        r.render()
    rows = r.launch_rows().astype(np.int64)
    kms = r.kernel_ms()
    # the same frame through the instrumented image: per-wave sums of the
    # lanes' node visits (slot 3 + RT_STAT_NODE_VISITS) and triangle tests
    r.configure(size, size, shadows=True, path=path, bvh_walk=bvh, instrumented=True)
    r.render()
    irows = r.launch_rows().astype(np.int64)
    base = rows[:, 12].min()
    t0 = rows[:, 12] - base
    end = rows[:, 13] - base
    dur = end - t0
    prim = rows[:, 14] - rows[:, 12]           # start -> primary traced
    drain = np.where(rows[:, 15] > 0, rows[:, 13] - rows[:, 15], 0)  # final shadow drain
    span = end.max()
    # slot utilisation: waves alive per 1 us bucket
    nb = int(span // 100) + 1
    alive = np.zeros(nb)
    for a, b in zip(t0, end):
        alive[a // 100:(b // 100) + 1] += 1
    q = lambda x, p: float(np.percentile(x, p))  # noqa: E731
    n = len(dur)
    # wave w renders chunk w (one chunk per wave): the model waves are the
    # slow ones; report the lifetime by chunk decile of duration
    out = {
        "size": size, "mode": "path" if path else "shadow", "waves": int(n), "event_kernel_us": round(kms * 1e3, 1),
        "stamp_span_us": round(span / 100.0, 1),
        "wave_us": {"p10": q(dur, 10) / 100, "p50": q(dur, 50) / 100, "p90": q(dur, 90) / 100,
                    "p99": q(dur, 99) / 100, "max": float(dur.max()) / 100},
        "start_us": {"p50": q(t0, 50) / 100, "p90": q(t0, 90) / 100, "max": float(t0.max()) / 100},
        "alive_per_us": [int(x) for x in alive[::max(1, nb // 40)]],
        "sum_wave_us_over_span": round(float(dur.sum()) / float(span), 1),
        "last_start_to_end_us": round(float(span - t0.max()) / 100, 1),
    }
    slow = np.argsort(dur)[-50:]
    out["slowest50"] = {"wave_us": float(dur[slow].mean()) / 100,
                        "primary_us": float(prim[slow].mean()) / 100,
                        "shadow_drain_us": float(drain[slow].mean()) / 100,
                        "start_us": float(t0[slow].mean()) / 100}
    out["all"] = {"primary_us": float(prim.mean()) / 100, "shadow_drain_us": float(drain.mean()) / 100}
    # wave-level loop iterations (RT_WAVE_ITER): primary node steps (slot 7),
    # primary leaf rounds (8), secondary-ray node steps + leaf rounds (9)
    it = rows[:, 7:10]
    out["slowest50"].update({"primary_node_iters": float(it[slow, 0].mean()),
                             "primary_leaf_iters": float(it[slow, 1].mean()),
                             "secondary_iters": float(it[slow, 2].mean()),
                             "us_per_iter": float(dur[slow].mean() / 100 / max(1.0, it[slow].sum(1).mean())),
                             "lane_visits_avg": float(irows[slow, 7].mean()) / 64,
                             "lane_tri_tests_avg": float(irows[slow, 8].mean()) / 64})
    if not path:  # phase stamps (RT_STAMPS rt_kernel): 3 before primary, 14 primary done,
        # 4 layers done, 11 shaded, 5 queued/stored, 6 non-final drain start, 15 final drain
        ph = lambda a, b: float((rows[slow, b] - rows[slow, a]).mean()) / 100  # noqa: E731
        out["slowest50"]["phases_us"] = {
            "to_primary": ph(12, 3), "primary": ph(3, 14), "layers": ph(14, 4), "shade": ph(4, 11),
            "plane_queue": ph(11, 5), "to_final_drain": ph(5, 15), "final_drain": ph(15, 13),
            "nonfinal_drains": int((rows[slow, 6] > 0).sum()),
            "final_drain_rays": float(rows[slow, 8].mean()),
            "final_drain_rays_hist": np.histogram(rows[slow, 8], bins=[0, 1, 9, 17, 33, 49, 64])[0].tolist()}
        # s_memtime cycles waiting on the packet walks' record loads (slot 0
        # primary, 1 shadow) per wave, and per loop iteration
        pi = np.maximum(it[slow, 0] + it[slow, 1], 1)
        si = np.maximum(it[slow, 2], 1)
        out["slowest50"]["load_wait_cycles"] = {
            "primary": float(rows[slow, 0].mean()), "shadow": float(rows[slow, 1].mean()),
            "primary_per_iter": float((rows[slow, 0] / pi).mean()),
            "shadow_per_iter": float((rows[slow, 1] / si).mean())}
    if path:  # pt stamp image: 10 wave cycles (s_memtime), 5 vertex steps, 6 bounce-hit
        # shading cycles; lane pairs (path_step<true>): 4 shadow-list cycles, 2
        # bounce-walk cycles; paired vertices: 4 paired-traversal cycles
        cyc = rows[:, 10].astype(np.float64)
        ghz = cyc[slow] / (dur[slow] * 10.0)
        out["slowest50"].update({
            "clock_ghz": float(ghz.mean()),
            "vertex_steps": float(rows[slow, 5].mean()),
            "traversal_frac": float((rows[slow, 4] / np.maximum(cyc[slow], 1)).mean()),
            "bounce_walk_frac": float((rows[slow, 2] / np.maximum(cyc[slow], 1)).mean()),
            "shade_frac": float((rows[slow, 6] / np.maximum(cyc[slow], 1)).mean()),
            "node_loop_frac": float((rows[slow, 11] / np.maximum(cyc[slow], 1)).mean()),
            "node_iters": float(rows[slow, 9].mean()),
            "cycles_per_iter": float((cyc[slow] / np.maximum(it[slow].sum(1), 1)).mean())})
        out["all"]["clock_ghz"] = float((cyc / np.maximum(dur * 10.0, 1)).mean())
    out["all"].update({"primary_node_iters": float(it[:, 0].mean()), "primary_leaf_iters": float(it[:, 1].mean()),
                       "secondary_iters": float(it[:, 2].mean())})
    # background (short) waves: where their time goes -- start -> primary
    # traced (prologue, task map, traversal) and primary traced -> end
    # (layers, shading, store, counter flush)
    fast = dur <= np.percentile(dur, 50)
    out["short_waves"] = {"n": int(fast.sum()), "wave_us": float(dur[fast].mean()) / 100,
                          "to_primary_us": float(prim[fast].mean()) / 100,
                          "after_primary_us": float((dur - prim)[fast].mean()) / 100}
    if not path:  # stamp image slots 10 (scene loaded) and 11 (pixel shaded)
        pro = rows[:, 10] - rows[:, 12]
        shd = rows[:, 11] - rows[:, 14]
        out["short_waves"].update({"prologue_us": float(pro[fast].mean()) / 100,
                                   "trace_us": float((prim - pro)[fast].mean()) / 100,
                                   "layers_shade_us": float(shd[fast].mean()) / 100,
                                   "store_flush_us": float((rows[:, 13] - rows[:, 11])[fast].mean()) / 100})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
