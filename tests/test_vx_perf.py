"""The vx_dump_perf class -> gfx950 counter mapping (scripts/vx_perf.py):
every class's counter passes respect rocprofv3's per-block limits, and the
report prints the reference's PERF line layout (runtime/stub/utils.cpp)."""
import io
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import vx_perf  # noqa: E402

LIMITS = {"SQ": 8, "TCC": 4, "TCP": 4, "TA": 2, "TD": 2, "GRBM": 2}


def test_passes_within_hardware_limits():
    for cls, passes in vx_perf.PASSES.items():
        for counters in vx_perf.BASE + passes:
            per = {}
            for c in counters:
                blk = c.split("_")[0]
                if blk in LIMITS:
                    per[blk] = per.get(blk, 0) + 1
            for blk, n in per.items():
                assert n <= LIMITS[blk], (cls, counters)
            derived = [c for c in counters if "_" not in c]
            assert not derived or len(counters) == 1, counters   # derived metrics alone


def test_report_layout():
    v = {"SQ_INSTS": 1000, "GRBM_GUI_ACTIVE": 4000, "SQ_WAVE_CYCLES": 4000, "SQ_WAIT_ANY": 1000,
         "SQ_WAIT_INST_ANY": 2000, "SQ_ACTIVE_INST_VALU": 600, "SQ_ACTIVE_INST_SALU": 200,
         "SQ_ACTIVE_INST_VMEM": 200, "TCC_HIT_sum": 90, "TCC_MISS_sum": 10}
    for cls in range(6):
        out = io.StringIO()
        vx_perf.report(cls, v, out)
        lines = out.getvalue().splitlines()
        assert all(l.startswith("PERF: ") for l in lines)
        assert lines[-1] == "PERF: instrs=1000, cycles=500, IPC=2.000000"
    out = io.StringIO()
    vx_perf.report(2, v, out)
    assert "l2cache read misses=10 (hit ratio=90%)" in out.getvalue()
