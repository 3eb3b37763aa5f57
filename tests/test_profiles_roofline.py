"""The committed round-end evidence agrees with itself (CPU): for every bench
workload, scripts/check_roofline.py recomputes the bench line's roofline
fractions from the committed rocprofv3 summary + per-dispatch trace of the
same command and the PMC record, and each agrees with the line within 5 %
(the timed frames' rocprof average vs the line's kernel clock)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
R05 = os.path.join(ROOT, "profiles", "r05")


@pytest.mark.parametrize("workload", ["shadow", "path", "flat"])
def test_round_end_roofline_recomputes(workload):
    bench = os.path.join(R05, "final", f"bench_{workload}.json")
    stats = os.path.join(R05, "prof", f"kernel_stats_{workload}.csv")
    if not (os.path.exists(bench) and os.path.exists(stats)):
        pytest.skip("round-end evidence not in this tree")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "check_roofline.py"), bench, stats,
                        "--pmc", os.path.join(ROOT, "profiles", f"pmc_{workload}.json")],
                       capture_output=True, text=True, cwd=ROOT, timeout=120)
    out = json.loads(p.stdout)
    assert out["ok"], out["checks"]
    assert "timed dispatches" in out.get("rocprof_avg_of", ""), out
    line = json.load(open(bench))
    assert abs(out["rocprof_avg_ms"] - line["config"]["kernel_ms"]) <= 0.05 * line["config"]["kernel_ms"]
