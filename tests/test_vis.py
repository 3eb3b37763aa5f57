"""Raster-exact primary rays (CPU): the RT path resolves a primary ray the
way draw3d's rasterizer resolves that pixel -- Q15.16 edge coverage inside
the binned 32x32 tiles (sim/common/graphics.cpp:813-825, gfxutil.cpp:237-271)
and the 24-bit depth test's winner (graphics.cpp:564-596, gpu_sw.h:46-60) --
found by a BVH walk over per-node pixel rectangles and depth bounds
(kernels/rt_common.h "primary visibility", app/vis.cpp; oracle/vis.c).

  * the product's per-primitive records (rt_scene_setup_vis: exact integer
    row solving) == the oracle's brute force over the binned tiles;
  * the depth lower bound holds at every covered pixel (numpy restatement
    of the shader's z interpolation);
  * the oracle's RT primary frame (BVH4, BVH2 and flat list) == the oracle
    raster frame (colour and winning pid), and == the reference's golden
    images with 0 mismatching pixels (tekkaman_1024x1024.png included)."""
import numpy as np
import pytest

from conftest import GOLDEN, scene_path
from skybox_rt_amd import rt

RT_SCENES = ("triangle", "tekkaman", "box", "scene", "carnival")


def _png(path):
    from PIL import Image
    return np.array(Image.open(path).convert("RGBA"))


_c = {}


def scenes(po, name):
    if name not in _c:
        _c[name] = (po.OracleScene(po.cgltrace.load(scene_path(name))), rt.Scene.load(scene_path(name)))
    return _c[name]


@pytest.mark.parametrize("name", RT_SCENES)
@pytest.mark.parametrize("w,h", [(8, 8), (64, 64), (100, 37), (128, 128), (200, 200), (1024, 1024)])
def test_vis_records_equal_oracle_bruteforce(oracle_lib, name, w, h):
    osc, sc = scenes(oracle_lib, name)
    assert np.array_equal(sc.setup_vis(w, h), oracle_lib.vis_prims(osc, w, h))


def _depth_words(edges, zat, xs, ys):
    """numpy restatement of the shader's depth word at pixels (xs, ys) of a
    primitive (gfx_device.h shade_edges / oracle orc_vis_depth), float32 and
    int32-wrap arithmetic exactly as on the device; also the coverage mask."""
    x = xs.astype(np.uint32)
    y = ys.astype(np.uint32)
    E = [(np.uint32(e[0] & 0xffffffff) * x + np.uint32(e[1] & 0xffffffff) * y
          + np.uint32(e[2] & 0xffffffff)).view(np.int32) for e in edges]
    cov = (E[0] >= 0) & (E[1] >= 0) & (E[2] >= 0)
    f = [e.astype(np.float32) * np.float32(1.0 / (1 << 24)) for e in E]
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        r = np.float32(1.0) / ((f[0] + f[1]) + f[2])
        dx = (r * f[0]) * np.float32(1 << 24)
        dy = (r * f[1]) * np.float32(1 << 24)
    def fx(v):
        out = np.where(np.isnan(v) | (v >= 2147483648.0), 2147483647, 0).astype(np.int64)
        ok = ~np.isnan(v) & (v < 2147483648.0) & (v >= -2147483648.0)
        out[ok] = np.trunc(v[ok]).astype(np.int64)
        out[~np.isnan(v) & (v < -2147483648.0)] = -2147483648
        return out
    dxi, dyi = fx(dx), fx(dy)
    t = ((np.int64(zat[0]) * dxi) >> 24).astype(np.int64) + np.int64(zat[2])
    t = ((np.int64(zat[1]) * dyi) >> 24) + ((t + 2**31) % 2**32 - 2**31)
    return cov, (t % (1 << 24)).astype(np.uint32)


@pytest.mark.parametrize("name,size", [("tekkaman", 256), ("scene", 200), ("box", 64)])
def test_depth_lower_bound_holds_at_every_covered_pixel(oracle_lib, name, size):
    osc, sc = scenes(oracle_lib, name)
    vis = sc.setup_vis(size, size)
    prims = sc.setup_prims(size, size)
    checked = 0
    for g in range(len(vis)):
        rx, ry, zmin = (int(v) for v in vis[g])
        if rx == 0xFFFF:
            continue
        x0, x1, y0, y1 = rx & 0xFFFF, rx >> 16, ry & 0xFFFF, ry >> 16
        ys, xs = np.mgrid[y0:y1 + 1, x0:x1 + 1]
        edges = prims[g, 0:9].reshape(3, 3).astype(np.int64)
        cov, z = _depth_words(edges, prims[g, 9:12].astype(np.int64), xs.ravel(), ys.ravel())
        assert cov.any()
        assert (z[cov] >= zmin).all(), (name, g, int(z[cov].min()), zmin)
        checked += int(cov.sum())
    assert checked > 0


@pytest.mark.parametrize("name", ("tekkaman", "box", "scene", "carnival", "triangle"))
@pytest.mark.parametrize("size", (8, 32, 128, 200))
def test_rt_primary_equals_raster(oracle_lib, name, size):
    po = oracle_lib
    osc, sc = scenes(po, name)
    rc, _, rp = po.raster_render(osc, size, size)
    p = po.rt_params(size, size, shadows=False, nthreads=8)
    for bvh in (sc.bvh() + (sc.bvh4(),), sc.bvh(), None):
        c, pid, _, _ = po.rt_render(osc, p, bvh=bvh)
        assert np.array_equal(c, rc)
        assert np.array_equal(pid, rp)


@pytest.mark.parametrize("name,size", [("triangle", n) for n in (8, 16, 32, 64, 128)] +
                         [(n, 128) for n in ("tekkaman", "box", "scene", "carnival")])
def test_rt_primary_matches_reference_golden(oracle_lib, name, size):
    po = oracle_lib
    osc, sc = scenes(po, name)
    c, _, _, _ = po.rt_render(osc, po.rt_params(size, size, shadows=False, nthreads=8),
                              bvh=sc.bvh() + (sc.bvh4(),))
    ref = _png(f"{GOLDEN}/draw3d/{name}_ref_{size}.png")
    assert po.compare_images(po.argb_to_rgba_image(c), ref, tol=0) == 0


def test_rt_primary_tekkaman_1024_equals_reference_render(oracle_lib):
    po = oracle_lib
    osc, sc = scenes(po, "tekkaman")
    c, _, _, _ = po.rt_render(osc, po.rt_params(1024, 1024, shadows=False, nthreads=8),
                              bvh=sc.bvh() + (sc.bvh4(),))
    ref = _png(f"{GOLDEN}/draw3d/tekkaman_1024x1024.png")
    assert po.compare_images(po.argb_to_rgba_image(c), ref, tol=0) == 0
