"""GPU parity of the draw3d raster pipeline (raster_kernel.hip; SURVEY.md
8(f) rank 1) against the reference's own golden images and the oracle's
restatement (oracle/raster.c, itself pinned to those goldens): colour AND
depth/stencil buffers bit-exact, on every scene the reference ships --
including the blending scenes (vase, mouse, evilskull, polybump) the RT path
cannot trace."""
import numpy as np
import pytest
from PIL import Image

from conftest import GOLDEN, scene_path

pytestmark = pytest.mark.gpu

from skybox_rt_amd import rt  # noqa: E402

_cache = {}


def setup(po, name):
    if name not in _cache:
        s = rt.Scene.load(scene_path(name))
        _cache[name] = (s, rt.Renderer(s), po.OracleScene(po.cgltrace.load(scene_path(name))))
    return _cache[name]


@pytest.fixture(scope="module")
def po(oracle_lib):
    return oracle_lib


GOLDENS = [("triangle", n) for n in (8, 16, 32, 64, 128)] + [
    ("tekkaman", 128), ("box", 128), ("carnival", 128), ("scene", 128),
    ("evilskull", 32), ("evilskull", 128), ("mouse", 32), ("mouse", 128),
    ("polybump", 32), ("polybump", 128), ("vase", 32), ("vase", 128)]


@pytest.mark.parametrize("name,size", GOLDENS)
def test_raster_matches_draw3d_golden(po, name, size):
    _, r, _ = setup(po, name)
    r.configure(size, size, raster=True)
    r.render()
    img = po.argb_to_rgba_image(r.framebuffer())
    ref = np.array(Image.open(f"{GOLDEN}/draw3d/{name}_ref_{size}.png").convert("RGBA"))
    assert po.compare_images(img, ref, tol=0) == 0


@pytest.mark.parametrize("name,size", [("tekkaman", 1024), ("tekkaman", 333), ("vase", 200),
                                       ("evilskull", 512), ("mouse", 96), ("polybump", 257),
                                       ("carnival", 640), ("scene", 1000), ("box", 64)])
def test_raster_color_and_depth_bit_exact_vs_oracle(po, name, size):
    _, r, osc = setup(po, name)
    r.configure(size, size, raster=True)
    r.render()
    color, depth, _ = po.raster_render(osc, size, size)
    assert np.array_equal(r.framebuffer(), color)
    assert np.array_equal(r.depthbuffer(), depth)
    st = r.stats()
    assert st["primary_rays"] == size * size          # pixels owned by the kernel


def test_raster_tekkaman_1024_reference_render(po):
    _, r, _ = setup(po, "tekkaman")
    r.configure(1024, 1024, raster=True)
    r.render()
    ref = np.array(Image.open(f"{GOLDEN}/draw3d/tekkaman_1024x1024.png").convert("RGBA"))
    assert po.compare_images(po.argb_to_rgba_image(r.framebuffer()), ref, tol=0) == 0


def test_rtapp_cli_raster_mode_against_golden():
    import os
    import subprocess
    from skybox_rt_amd import _lib
    exe = os.path.join(_lib.LIB_DIR, "rtapp")
    out = subprocess.run([exe, "-R", "-t", scene_path("vase"), "-w", "128", "-h", "128", "-o",
                          "/tmp/rtapp_vase128.png", "-r", f"{GOLDEN}/draw3d/vase_ref_128.png"],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "PASSED!" in out.stdout


def test_raster_repeatable_and_rt_modes_rejected_on_blend_scenes(po):
    _, r, _ = setup(po, "vase")
    r.configure(128, 128, raster=True)
    r.render()
    a = r.framebuffer()
    r.render()
    assert np.array_equal(a, r.framebuffer())          # each frame starts from the clears
    with pytest.raises(rt.RtError):
        r.configure(128, 128, shadows=True)            # blending: raster only
