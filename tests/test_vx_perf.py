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


def test_in_process_library_exports():
    """libvx_perf.so (runtime/vx_perf.cpp): the in-process collector the stub
    loads under VORTEX_PROFILING exports its three entry points."""
    import ctypes
    lib = os.path.join(ROOT, "skybox_rt_amd", "lib", "libvx_perf.so")
    h = ctypes.CDLL(lib)
    for sym in ("vx_perf_init", "vx_perf_dump", "vx_perf_dispatches"):
        assert hasattr(h, sym)
    h.vx_perf_dispatches.restype = ctypes.c_uint64
    assert h.vx_perf_dispatches() == 0       # nothing collected, no GPU touched
    assert h.vx_perf_init(9) == -1           # no such class


def _perf_lines(out):
    return [ln for ln in out.splitlines() if ln.startswith("PERF: ")]


import pytest  # noqa: E402


@pytest.mark.gpu
@pytest.mark.parametrize("cls", [1, 2])
def test_vx_dump_perf_in_process(tmp_path, cls):
    """VORTEX_PROFILING=<class> + VX_DUMP_PERF: the C host prints the class's
    hardware counters in process at vx_dev_close (stub.cpp / vx_perf.cpp),
    the reference's utils.cpp:159-805 report, over all its launches."""
    import subprocess
    exe = os.path.join(ROOT, "skybox_rt_amd", "lib", "rtapp")
    env = dict(os.environ, VORTEX_PROFILING=str(cls), VX_DUMP_PERF="1")
    scene = os.path.join(ROOT, "tests", "golden", "scenes", "tekkaman.cgltrace")
    out = subprocess.run([exe, "-t", scene, "-w", "256", "-h", "256", "-S", "-n", "6",
                          "-o", str(tmp_path / "o.png")], env=env, capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    lines = _perf_lines(out.stdout)
    instrs = [ln for ln in lines if ln.startswith("PERF: instrs=")]
    assert instrs, lines
    n = int(instrs[0].split("instrs=")[1].split(",")[0])
    assert n > 0
    assert any(f"class {cls}: " in ln and "vx_main launches profiled" in ln for ln in lines), lines
    key = "scheduler idle=" if cls == 1 else "dcache reads="
    assert any(key in ln for ln in lines), lines


GFX_APPS = {  # the CI's --perf=<class> runs (ci/regression.sh.in:142,165,183)
    3: ("texapp", ["-i", "soccer.png", "-r", "soccer_ref_g1.png", "-g1"], "tex", "tex memory reads="),
    4: ("rasterapp", ["-t", "triangle.cgltrace"], "scenes", "rcache read misses="),
    5: ("omapp", ["-r", "whitebox_128.png"], "om", "om memory writes="),
}


@pytest.mark.gpu
@pytest.mark.parametrize("cls", sorted(GFX_APPS))
def test_vx_dump_perf_graphics_classes(tmp_path, cls):
    """Classes 3 (TEX), 4 (RASTER), 5 (OM) (runtime/stub/utils.cpp:587-640,
    725-790) printed in process by the app the reference CI profiles with that
    class: texapp, rasterapp, omapp."""
    import subprocess
    exe, args, sub, key = GFX_APPS[cls]
    env = dict(os.environ, VORTEX_PROFILING=str(cls), VX_DUMP_PERF="1",
               RT_ASSETS_PATHS=os.path.join(ROOT, "tests", "golden", sub))
    out = subprocess.run([os.path.join(ROOT, "skybox_rt_amd", "lib", exe)] + args +
                         ["-o", str(tmp_path / "o.png")], env=env, capture_output=True, text=True,
                         timeout=120, cwd=str(tmp_path))
    assert out.returncode == 0, out.stdout + out.stderr
    lines = _perf_lines(out.stdout)
    assert any(key in ln for ln in lines), lines
    assert any(f"class {cls}: " in ln and "vx_main launches profiled" in ln for ln in lines), lines
    n = int([ln for ln in lines if ln.startswith("PERF: instrs=")][0].split("instrs=")[1].split(",")[0])
    assert n > 0
