"""BASELINE config 3 by BVH traversal only (RT_RENDER_BVH_WALK, kernel image
rt_bvh: entry vx_main_rt_bvh): primary visibility by the binary16-BVH4 packet
walk of the tree (raster-exact leaf tests), shadow rays by the any-hit
packet walk -- no per-block or light-space lists.  The frame and every
counter equal the oracle's restatement of the same walks (oracle/rt.c
vis_trace_packet, bvh_trace with vis_lists / shadow_lists off); the frame
equals the default (list) image's and, at 1024^2, the oracle's brute force.
The bench's `series.bvh_walk` line times this image (bench.py)."""
import numpy as np
import pytest

from conftest import scene_path

pytestmark = pytest.mark.gpu

from skybox_rt_amd import rt  # noqa: E402

_osc = {}


def _oscene(po, name):
    if name not in _osc:
        _osc[name] = po.OracleScene(po.cgltrace.load(scene_path(name)))
    return _osc[name]


@pytest.mark.parametrize("name,w,h", [("tekkaman", 1024, 1024), ("tekkaman", 257, 129),
                                      ("carnival", 256, 256), ("scene", 200, 300), ("box", 128, 128)])
def test_bvh_walk_equals_oracle_with_counts(oracle_lib, name, w, h):
    po = oracle_lib
    s = rt.Scene.load(scene_path(name))
    r = rt.Renderer(s)
    r.configure(w, h, shadows=True, instrumented=True, bvh_walk=True)
    st = r.setup_stats()
    assert st["blist_blocks"] == 0 and st["slist_on"] == 0, st
    r.render()
    k_gpu = r.stats()
    refs, pids = r.export_vis_tree()
    c, _, _, k = po.rt_render(_oscene(po, name),
                              po.rt_params(w, h, shadows=True, nthreads=8, vis_lists=False,
                                           shadow_lists=False),
                              bvh=s.bvh() + (s.bvh4(),), vis_tree=(refs, pids))
    fb = r.framebuffer()
    assert np.array_equal(fb, c)
    assert k_gpu["node_visits"] > 0
    for key in ("node_visits", "tri_tests", "layer_tests", "shaded", "texel_bytes", "primary_rays",
                "shadow_rays", "geometry_hits", "occluded"):
        assert k_gpu[key] == k[key], key
    # the product (list) image renders the same frame; so does its timed
    # configuration of the BVH image (no counters)
    r.configure(w, h, shadows=True, counters=False)
    r.render()
    assert np.array_equal(r.framebuffer(), fb)
    r.configure(w, h, shadows=True, counters=False, bvh_walk=True)
    r.render()
    assert np.array_equal(r.framebuffer(), fb)
    r.close()
    s.close()


def test_bvh_walk_1024_equals_brute_force(oracle_lib):
    """The traversal decides nothing the brute force would not: every ray
    against every triangle (oracle, no BVH) gives the same 1024^2 frame."""
    po = oracle_lib
    s = rt.Scene.load(scene_path("tekkaman"))
    r = rt.Renderer(s)
    r.configure(1024, 1024, shadows=True, counters=False, bvh_walk=True)
    r.render()
    c, _, _, _ = po.rt_render(_oscene(po, "tekkaman"), po.rt_params(1024, 1024, shadows=True, nthreads=8),
                              bvh=None)
    assert np.array_equal(r.framebuffer(), c)
    r.close()
    s.close()
