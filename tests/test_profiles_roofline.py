"""The committed round-end evidence agrees with itself (CPU):
scripts/check_roofline.py recomputes the round-end bench line's roofline
fractions -- the headline's and every series entry's (the BVH walk, config
4, config 2, the 4096^2 frame) -- from the committed rocprofv3 summary +
per-dispatch trace of the same command and the PMC records, and each agrees
with the line within 5 % (the timed frames' rocprof average vs the line's
kernel clock)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
R06 = os.path.join(ROOT, "profiles", "r06")


def test_round_end_roofline_recomputes():
    bench = os.path.join(R06, "final", "bench_under_rocprof.json")
    stats = os.path.join(R06, "prof", "kernel_stats.csv")
    trace = os.path.join(R06, "prof", "kernel_trace.csv.gz")
    if not (os.path.exists(bench) and os.path.exists(stats) and os.path.exists(trace)):
        pytest.skip("round-end evidence not in this tree")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "check_roofline.py"), bench, stats,
                        "--trace", trace], capture_output=True, text=True, cwd=ROOT, timeout=120)
    out = json.loads(p.stdout)
    assert out["ok"], out["checks"]
    assert "timed dispatches" in out.get("rocprof_avg_of", ""), out
    line = json.load(open(bench))
    assert abs(out["rocprof_avg_ms"] - line["config"]["kernel_ms"]) <= 0.05 * line["config"]["kernel_ms"]
    # every HBM-bound series entry checked against its own image's dispatches
    for name in ("bvh_walk", "path", "strong_4096"):
        assert f"series.{name}.roofline.frac" in out["checks"], (name, sorted(out["checks"]))
        assert name in out and out[name]["kernel"] == line["series"][name]["image"].split("entry ")[-1].rstrip(")")
    assert "flat" in out


def test_timed_region_picks_the_timed_dispatches(tmp_path):
    """check_roofline.timed_region on a synthetic trace: sync frames (each
    followed by the completion kernel), the warmup, a ~1 ms gap, the timed
    frames with one host stall inside, a gap, the kernel-clock frames, then a
    series of slower frames with setup launches between -- the average is the
    timed frames' only."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import check_roofline as cr
    rows, t = [], 0

    def k(name, dur, gap=0):
        nonlocal t
        t += gap
        rows.append((t, t + dur, name))
        t += dur

    for _ in range(5):
        k("vx_main_rt_kernel", 18000, 9000)
        k("vx_main_rt_kernel_done", 1000)
    for _ in range(5):
        k("vx_main_rt_kernel", 17000, 500)
    for i in range(20):
        k("vx_main_rt_kernel", 16000, 1_000_000 if i == 0 else (40_000 if i == 7 else 0))
    for i in range(10):
        k("vx_main_rt_kernel", 16500, 130_000 if i == 0 else 0)
    for _ in range(5):
        k("vx_main_rt_setup", 2000, 1000)
        k("vx_main_rt_kernel", 18000)
    p = tmp_path / "trace.csv"
    with open(p, "w") as f:
        f.write('"Kernel_Name","Start_Timestamp","End_Timestamp"\n')
        for st, en, nm in rows:
            f.write(f'"{nm}",{st},{en}\n')
    assert abs(cr.timed_region(str(p), "vx_main_rt_kernel", 20) - 16e-6) < 1e-12
    assert cr.timed_region(str(p), "vx_main_rt_kernel", 50) is None
