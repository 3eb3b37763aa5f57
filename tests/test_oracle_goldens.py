"""Pin the oracle against the reference's own golden images (data copied to
tests/golden/): draw3d goldens (CompareImages tolerance 1 in the reference,
draw3d/main.cpp:507 -- we require exact), raster coverage goldens
(tests/regression/raster/triangle_ref_*.png) and the 1024x1024 tekkaman render
in docs/assets/img/."""
import numpy as np
import pytest
from PIL import Image

from conftest import GOLDEN, scene_path


def _png(path):
    return np.array(Image.open(path).convert("RGBA"))


DRAW3D = [("triangle", n) for n in (8, 16, 32, 64, 128)] + [
    ("tekkaman", 128), ("box", 128), ("carnival", 128), ("scene", 128),
    ("evilskull", 32), ("evilskull", 128), ("mouse", 32), ("mouse", 128),
    ("polybump", 32), ("polybump", 128), ("vase", 32), ("vase", 128)]


@pytest.mark.parametrize("name,size", DRAW3D)
def test_raster_oracle_matches_draw3d_golden(oracle_lib, name, size):
    po = oracle_lib
    sc = po.OracleScene(po.cgltrace.load(scene_path(name)))
    color, _, _ = po.raster_render(sc, size, size)
    img = po.argb_to_rgba_image(color)
    ref = _png(f"{GOLDEN}/draw3d/{name}_ref_{size}.png")
    assert po.compare_images(img, ref, tol=1) == 0       # the reference's own bar
    assert po.compare_images(img, ref, tol=0) == 0       # and bit-exact


@pytest.mark.parametrize("size", (8, 16, 32, 64, 128))
def test_raster_oracle_coverage_matches_raster_golden(oracle_lib, size):
    po = oracle_lib
    sc = po.OracleScene(po.cgltrace.load(scene_path("triangle")))
    _, _, pid = po.raster_render(sc, size, size)
    ref = _png(f"{GOLDEN}/raster/coverage_triangle_ref_{size}.png")
    assert np.array_equal(pid[::-1] >= 0, ref[..., :3].max(-1) > 0)


def test_raster_oracle_tile_size_invariance(oracle_lib):
    # raster CI runs -k4/-k5/-k6 against the same golden (ci/regression.sh.in:179-200)
    po = oracle_lib
    sc = po.OracleScene(po.cgltrace.load(scene_path("tekkaman")))
    base, _, _ = po.raster_render(sc, 128, 128, 5)
    for k in (4, 6):
        other, _, _ = po.raster_render(sc, 128, 128, k)
        assert np.array_equal(base, other)


@pytest.mark.slow
def test_raster_oracle_matches_tekkaman_1024(oracle_lib):
    po = oracle_lib
    sc = po.OracleScene(po.cgltrace.load(scene_path("tekkaman")))
    color, _, _ = po.raster_render(sc, 1024, 1024)
    ref = _png(f"{GOLDEN}/draw3d/tekkaman_1024x1024.png")
    assert po.compare_images(po.argb_to_rgba_image(color), ref, tol=0) == 0


def test_raster_binning_granularity_is_semantic(oracle_lib):
    """Fixed-point coverage can reach past a primitive's float bbox; the
    reference covers such a pixel only inside a 32x32 tile the primitive was
    binned to.  The oracle reproduces that (mouse at 128^2 differs in one pixel
    with 16x16 binning), so the GPU raster binning always uses the 32x32
    granularity whatever its workgroup tile (raster_kernel.hip)."""
    po = oracle_lib
    sc = po.OracleScene(po.cgltrace.load(scene_path("mouse")))
    a, _, _ = po.raster_render(sc, 128, 128, 5)
    b, _, _ = po.raster_render(sc, 128, 128, 4)
    assert int((a != b).sum()) == 1
    ref = _png(f"{GOLDEN}/draw3d/mouse_ref_128.png")
    assert po.compare_images(po.argb_to_rgba_image(a), ref, tol=0) == 0


@pytest.mark.parametrize("size,k", [(s, 5) for s in (8, 16, 32, 64, 128)] + [(128, 4), (128, 6)])
def test_raster_app_coverage_oracle_matches_raster_golden(oracle_lib, size, k):
    """The raster regression app's own image (white coverage over the
    0xff000000 clear), at the CI's -k4/-k5/-k6 (ci/regression.sh.in:184-189)."""
    po = oracle_lib
    sc = po.OracleScene(po.cgltrace.load(scene_path("triangle")))
    fb = po.raster_coverage(sc, size, size, k)
    ref = po.load_png_argb(f"{GOLDEN}/raster/coverage_triangle_ref_{size}.png")
    assert np.array_equal(fb[::-1], ref)
