"""The reference's own graphics CI command lines, run verbatim on the MI355X.

ci/regression.sh.in runs the regression apps as `blackbox.sh --app=<app>
--args="<args>"` from each app's directory (tests/regression/<app>/, whose
path the apps compile in as ASSETS_PATHS).  Every distinct `--args` string of
the draw3d, raster, om and tex apps is listed below with the line it first
appears on; each runs through this build's CLI for that app (rtapp, rasterapp,
omapp, texapp) with the app directory's files on RT_ASSETS_PATHS (the
committed copies under tests/golden/; the raster app's triangle_ref_*.png are
committed as raster/coverage_triangle_ref_*.png and linked back to their
reference names here) and must print PASSED! with exit status 0.  The
blackbox options (--cores/--warps/--threads/--perf, simulator configurations)
select the simulated machine, which this build replaces, so they have no
counterpart here."""
import os
import shlex
import subprocess

import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

from skybox_rt_amd import _lib  # noqa: E402

CI_LINES = [
    (131, "tex", "-itoad.png -rtoad_ref_f0.png -f0 -g0"),
    (132, "tex", "-itoad.png -rtoad_ref_f1.png -f1 -g0"),
    (133, "tex", "-itoad.png -rtoad_ref_f2.png -f2 -g0"),
    (134, "tex", "-itoad.png -rtoad_ref_f3.png -f3 -g0"),
    (135, "tex", "-itoad.png -rtoad_ref_f4.png -f4 -g0"),
    (136, "tex", "-itoad.png -rtoad_ref_f5.png -f5 -g0"),
    (137, "tex", "-itoad.png -rtoad_ref_f6.png -f6 -g0"),
    (139, "tex", "-isoccer.png -rsoccer_ref_g0.png -g0"),
    (142, "tex", "-isoccer.png -rsoccer_ref_g1.png -g1"),
    (144, "tex", "-isoccer.png -rsoccer_ref_g2.png -g2"),
    (149, "tex", "-isoccer.png -rsoccer_ref_g1.png -g1 -z"),
    (151, "tex", "-isoccer.png -rsoccer_ref_g1.png"),
    (165, "om", "-rwhitebox_128.png"),
    (183, "raster", "-ttriangle.cgltrace -rtriangle_ref_128.png"),
    (187, "raster", "-k4 -ttriangle.cgltrace -rtriangle_ref_128.png"),
    (188, "raster", "-k6 -ttriangle.cgltrace -rtriangle_ref_128.png"),
    (191, "draw3d", "-tbox.cgltrace -rbox_ref_128.png"),
    (198, "draw3d", "-tvase.cgltrace -rvase_ref_128.png"),
    (213, "draw3d", "-ttriangle.cgltrace -rtriangle_ref_8.png -w8 -h8"),
    (215, "draw3d", "-tvase.cgltrace -rvase_ref_32.png -w32 -h32"),
    (217, "draw3d", "-xy -w64 -h64 -ttriangle.cgltrace -rtriangle_ref_64.png"),
]

EXE = {"draw3d": "rtapp", "raster": "rasterapp", "om": "omapp", "tex": "texapp"}


def _assets(root, app):
    """The app directory of the reference tree, rebuilt from tests/golden/."""
    d = os.path.join(root, app)
    if os.path.isdir(d):
        return d
    os.makedirs(d)
    links = {}
    if app in ("draw3d", "raster"):
        for f in os.listdir(os.path.join(GOLDEN, "scenes")):
            links[f] = os.path.join(GOLDEN, "scenes", f)
    if app == "draw3d":
        for f in os.listdir(os.path.join(GOLDEN, "draw3d")):
            links[f] = os.path.join(GOLDEN, "draw3d", f)
    elif app == "raster":
        for f in os.listdir(os.path.join(GOLDEN, "raster")):
            links[f.replace("coverage_", "")] = os.path.join(GOLDEN, "raster", f)
    else:
        for f in os.listdir(os.path.join(GOLDEN, app)):
            links[f] = os.path.join(GOLDEN, app, f)
    for name, target in links.items():
        os.symlink(target, os.path.join(d, name))
    return d


@pytest.fixture(scope="module")
def assets_root(tmp_path_factory):
    return str(tmp_path_factory.mktemp("ci_assets"))


@pytest.mark.parametrize("line,app,args", CI_LINES, ids=[f"L{l}-{a}" for l, a, _ in CI_LINES])
def test_reference_ci_line_passes(assets_root, tmp_path, line, app, args):
    env = dict(os.environ, RT_ASSETS_PATHS=_assets(assets_root, app))
    exe = os.path.join(_lib.LIB_DIR, EXE[app])
    p = subprocess.run([exe] + shlex.split(args), cwd=str(tmp_path), env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "PASSED!" in p.stdout, (
        f"ci/regression.sh.in:{line} --app={app} --args=\"{args}\": rc {p.returncode}\n"
        + p.stdout[-2000:] + p.stderr[-2000:])
    assert os.path.exists(tmp_path / "output.png")


def test_rtapp_routes_unsupported_scene_to_raster(assets_root, tmp_path):
    """vase blends, so the RT path rejects it; draw3d's command line still
    renders it (through the raster pipeline) and says so."""
    env = dict(os.environ, RT_ASSETS_PATHS=_assets(assets_root, "draw3d"))
    p = subprocess.run([os.path.join(_lib.LIB_DIR, "rtapp"), "-tvase.cgltrace",
                        "-rvase_ref_32.png", "-w32", "-h32"], cwd=str(tmp_path), env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "PASSED!" in p.stdout
    assert "rendering through the draw3d raster pipeline" in p.stdout


def test_rtapp_draw_range_and_tile_size(assets_root, tmp_path, oracle_lib):
    """-s / -e draw only drawcalls start..end (draw3d/main.cpp:179-181), -k
    bins at 2^k (raster pipeline): both equal the oracle on the same subset."""
    import numpy as np
    from conftest import scene_path
    po = oracle_lib
    env = dict(os.environ, RT_ASSETS_PATHS=_assets(assets_root, "draw3d"))
    full = po.cgltrace.load(scene_path("tekkaman"))
    for flags, k, dcs in ((["-s1"], 5, [1]), (["-e0"], 5, [0]), (["-k4"], 4, [0, 1]),
                          (["-s1", "-e1", "-k3"], 3, [1])):
        out = str(tmp_path / "o.png")
        p = subprocess.run([os.path.join(_lib.LIB_DIR, "rtapp"), "-ttekkaman.cgltrace", "-w128",
                            "-h128", "-o", out] + flags, cwd=str(tmp_path), env=env,
                           capture_output=True, text=True, timeout=120)
        assert p.returncode == 0, p.stdout + p.stderr
        sub = po.cgltrace.select_drawcalls(full, dcs)
        ref, _, _ = po.raster_render(po.OracleScene(sub), 128, 128, k)
        assert np.array_equal(po.load_png_argb(out)[::-1], ref), flags
