"""The light-space shadow lists are conservative (rt_common.h, oracle/rt.c
sl_build): any-hit over a ray's cell list must give the brute-force verdict
for every shadow ray.  Oracle only (CPU): frames and occlusion counts of
primary+shadow and path-traced frames over the lists == brute force over the
whole geometry list, for every RT scene and lights around, inside and far
from the models (including a light on a cube-face diagonal)."""
import numpy as np
import pytest

from conftest import scene_path

SCENES = ("triangle", "tekkaman", "box", "scene", "carnival")
LIGHTS = ((0.0, 60.0, 80.0), (30.0, -20.0, 95.0), (0.0, 0.0, 0.5), (-200.0, 150.0, 50.0),
          (5.0, 5.0, 99.5), (40.0, 40.0, 140.0))


@pytest.fixture(scope="module")
def scenes(oracle_lib):
    po = oracle_lib
    from skybox_rt_amd import rt
    out = {}
    for n in SCENES:
        s = rt.Scene.load(scene_path(n))
        out[n] = (po.OracleScene(po.cgltrace.load(scene_path(n))), s.bvh() + (s.bvh4(),))
    return out


@pytest.mark.parametrize("name", SCENES)
@pytest.mark.parametrize("light", LIGHTS)
def test_shadow_lists_equal_bruteforce(oracle_lib, scenes, name, light):
    po = oracle_lib
    osc, bvh = scenes[name]
    p = po.rt_params(96, 96, shadows=True, light=light, nthreads=4, shadow_lists=True)
    c1, _, _, k1 = po.rt_render(osc, p, bvh=bvh)
    c0, _, _, k0 = po.rt_render(osc, po.rt_params(96, 96, shadows=True, light=light, nthreads=4))
    assert np.array_equal(c1, c0)
    assert (k1["shadow_rays"], k1["occluded"]) == (k0["shadow_rays"], k0["occluded"])


@pytest.mark.parametrize("name", ("tekkaman", "box"))
@pytest.mark.parametrize("light", LIGHTS[:3])
def test_path_shadow_lists_equal_bvh(oracle_lib, scenes, name, light):
    po = oracle_lib
    osc, bvh = scenes[name]
    kw = dict(shadows=True, light=light, nthreads=4, path=True, bounces=4)
    c1, _, _, k1 = po.rt_render(osc, po.rt_params(96, 96, shadow_lists=True, **kw), bvh=bvh)
    c0, _, _, k0 = po.rt_render(osc, po.rt_params(96, 96, shadow_lists=False, **kw), bvh=bvh)
    assert np.array_equal(c1, c0)
    for key in ("shadow_rays", "occluded", "bounce_rays"):
        assert k1[key] == k0[key], key
