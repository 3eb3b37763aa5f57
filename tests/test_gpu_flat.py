"""GPU parity of the flat-triangle-list image (rt_flat: no BVH, the geometry
list staged in LDS; BASELINE config 2 = 256^2 tekkaman primary rays, and
config 1 = the 64^2 triangle) against the oracle's brute force, bit-exact
including the per-triangle test counts, and against the BVH image."""
import numpy as np
import pytest

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


@pytest.mark.parametrize("name,size,shadows", [("tekkaman", 256, False), ("tekkaman", 256, True),
                                               ("tekkaman", 100, True), ("triangle", 64, False),
                                               ("box", 128, True), ("scene", 128, True),
                                               # more chunks than workgroups: each workgroup runs
                                               # several chunks (the winner words' chunk-parity
                                               # double buffer of the no-shadow early out)
                                               ("tekkaman", 512, False), ("scene", 384, True)])
def test_flat_bit_exact_vs_oracle_bruteforce(po, name, size, shadows):
    _, r, osc = setup(po, name)
    c, _, _, k = po.rt_render(osc, po.rt_params(size, size, shadows=shadows, nthreads=8))
    r.configure(size, size, shadows=shadows, flat=True, instrumented=True)
    r.render()
    st = r.stats()
    assert np.array_equal(r.framebuffer(), c)
    for key in ("primary_rays", "shadow_rays", "geometry_hits", "occluded", "tri_tests",
                "layer_tests", "shaded", "texel_bytes"):
        assert st[key] == k[key], key
    r.configure(size, size, shadows=shadows, flat=True)
    r.render()
    flat = r.framebuffer()
    assert np.array_equal(flat, c)
    r.configure(size, size, shadows=shadows)
    r.render()
    assert np.array_equal(r.framebuffer(), flat)          # == the BVH image


def test_flat_config1_triangle_golden(po):
    from oracle.py_oracle import argb_to_rgba_image, compare_images
    from PIL import Image
    _, r, _ = setup(po, "triangle")
    r.configure(64, 64, shadows=False, flat=True)
    r.render()
    ref = np.array(Image.open(f"{GOLDEN}/draw3d/triangle_ref_64.png").convert("RGBA"))
    assert compare_images(argb_to_rgba_image(r.framebuffer()), ref, tol=1) == 0
