#!/usr/bin/env python3
"""Per-workgroup timeline of one config-2 frame (rt_flat) from the RT_STAMPS
diagnostic image (skybox_rt_amd/lib/variants/flatstamp, `make diag`): every
workgroup's counter row holds s_memrealtime stamps (100 MHz) at its start
(slot 12), scene loaded (10), list staged in LDS (11), wave 0's list scan
done (3), all waves' scans met (4), wave 0 shaded (5) and its end (13).
Prints a JSON summary: kernel span, workgroup start spread, per-phase
durations (median / p90 / max) of the workgroups that rendered a chunk, and
the phases of the last-ending workgroup.  Timing-only diagnostic."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def q(a):
    a = np.asarray(a, np.float64) * 0.01  # 100 MHz ticks -> us
    return {"median_us": round(float(np.median(a)), 3), "p90_us": round(float(np.percentile(a, 90)), 3),
            "max_us": round(float(a.max()), 3)}


def main():
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    import torch  # noqa: F401
    from skybox_rt_amd import rt
    kdir = os.path.join(ROOT, "skybox_rt_amd/lib/variants/flatstamp")
    if not os.path.exists(os.path.join(kdir, "rt_flat.vxbin")):
        sys.exit("flat_timeline: flatstamp image missing (make -C skybox_rt_amd/csrc diag)")
    s = rt.Scene.load(os.path.join(ROOT, "tests/golden/scenes/tekkaman.cgltrace"))
    r = rt.Renderer(s, kernel_dir=kdir)
    r.configure(size, size, shadows=False, flat=True)
    for _ in range(5):
        r.render()
    rows = r.launch_rows().astype(np.int64) & 0xffffffff
    kms = r.kernel_ms()
    st, ld, sg, s0, red, sh, en = (rows[:, k] for k in (12, 10, 11, 3, 4, 5, 13))
    base = st.min()
    work = s0 != 0
    out = {
        "size": size, "kernel_ms_events": round(kms, 5), "workgroups": int(len(rows)),
        "working_workgroups": int(work.sum()),
        "span_us": round(float((en.max() - base) * 0.01), 3),
        "start_spread_working_us": q(st[work] - base),
        "start_spread_idle_us": q(st[~work] - base) if (~work).any() else None,
        "end_working_us": q(en[work] - base),
        "end_idle_us": q(en[~work] - base) if (~work).any() else None,
        "phase_load_scene": q(ld[work] - st[work]),
        "phase_stage": q(sg[work] - ld[work]),
        "phase_scan_wave0": q(s0[work] - sg[work]),
        "phase_scan_all": q(red[work] - sg[work]),
        "phase_shade": q(sh[work] - red[work]),
        "phase_store_end": q(en[work] - sh[work]),
        "lifetime": q(en[work] - st[work]),
    }
    i = int(np.argmax(np.where(work, en, 0)))
    out["last_working_wg"] = {"index": i, "start_us": round(float((st[i] - base) * 0.01), 3),
                              **{k: round(float(v * 0.01), 3) for k, v in
                                 (("load", ld[i] - st[i]), ("stage", sg[i] - ld[i]),
                                  ("scan_all", red[i] - sg[i]), ("shade", sh[i] - red[i]),
                                  ("end", en[i] - sh[i]))}}
    print(json.dumps(out))
    r.close()
    s.close()


if __name__ == "__main__":
    main()
