"""CPU tests of the BVH8 collapse (app/bvh.cpp Collapser<8>, the RT_BVH8
images' tree) and of the oracle's 8-wide step (oracle/rt.c bvh8_step): the
host builder's binary16 BVH8 is a different tree over the same leaves, so
every traversal over it must decide what the BVH4 traversal and the brute
force decide -- the same frames, hits, shadow verdicts and bounce rays --
while taking fewer node steps than the BVH4 per ray (its depth is lower).
No GPU: the scene's host-built arrays (rt_scene_export_bvh8) and the C
oracle only."""
import os

import numpy as np
import pytest

from conftest import scene_path

os.environ.setdefault("SKYBOX_RT_NO_TORCH", "1")

from skybox_rt_amd import rt  # noqa: E402

NAMES = ("tekkaman", "scene", "box")


@pytest.fixture(scope="module")
def scenes(oracle_lib):
    po = oracle_lib
    out = {}
    for name in NAMES:
        s = rt.Scene.load(scene_path(name))
        out[name] = (po.OracleScene(po.cgltrace.load(scene_path(name))), s.bvh() + (s.bvh4(),), s.bvh8(),
                     s.info())
    return out


@pytest.mark.parametrize("name", NAMES)
def test_bvh8_shape(scenes, name):
    """Collapsing opens the largest-area internal child until 8 slots are
    full: no more nodes than the BVH4, no deeper, and a node count that
    covers every BVH2 leaf (each BVH8 node holds at most 8 children)."""
    _, bvh, nodes8, info = scenes[name]
    assert nodes8.shape[0] == info["bvh8_nodes"] >= 1
    assert info["bvh8_nodes"] <= info["bvh4_nodes"]
    assert info["bvh8_depth"] <= info["bvh4_depth"]
    assert 8 * info["bvh8_nodes"] >= info["bvh_leaves"]


@pytest.mark.parametrize("name,size", [("tekkaman", 96), ("scene", 64), ("box", 48)])
def test_bvh8_walk_equals_bvh4_and_bruteforce(oracle_lib, scenes, name, size):
    """Shadow rays by the any-hit walk (block / light-space lists off) over
    the BVH8 == over the BVH4 == brute force: frame, primary ids, verdicts."""
    po = oracle_lib
    osc, bvh, nodes8, _ = scenes[name]
    p = po.rt_params(size, size, shadows=True, nthreads=8, vis_lists=False, shadow_lists=False)
    cb, pb, _, kb = po.rt_render(osc, p)
    c4, p4, _, k4 = po.rt_render(osc, p, bvh=bvh)
    c8, p8, _, k8 = po.rt_render(osc, p, bvh=bvh + (nodes8,))
    assert np.array_equal(cb, c4) and np.array_equal(c4, c8)
    assert np.array_equal(pb, p4) and np.array_equal(p4, p8)
    for key in ("primary_rays", "shadow_rays", "geometry_hits", "occluded"):
        assert kb[key] == k4[key] == k8[key], key


@pytest.mark.parametrize("name,size,bounces", [("tekkaman", 96, 4), ("scene", 64, 3)])
def test_bvh8_path_trace_equals_bvh4(oracle_lib, scenes, name, size, bounces):
    """The path tracer's closest-hit bounce walks over the BVH8: the same
    frame and ray counts as over the BVH4 (closer() is a strict total order,
    so the nearest hit does not depend on the visit order), with fewer
    node visits (the lower tree)."""
    po = oracle_lib
    osc, bvh, nodes8, _ = scenes[name]
    p = po.rt_params(size, size, path=True, bounces=bounces, nthreads=8)
    c4, _, _, k4 = po.rt_render(osc, p, bvh=bvh)
    c8, _, _, k8 = po.rt_render(osc, p, bvh=bvh + (nodes8,))
    assert np.array_equal(c4, c8)
    for key in ("shadow_rays", "occluded", "bounce_rays", "shaded", "texel_bytes"):
        assert k4[key] == k8[key], key
    assert 0 < k8["node_visits"] < k4["node_visits"]
