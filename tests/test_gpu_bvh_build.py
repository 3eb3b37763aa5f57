"""GPU BVH build (kernels/bvh_build.hip): the device
build's node and triangle arrays equal the oracle's restatement
(oracle/lbvh.c) bit for bit -- on the reference's scenes and on a
synthetic 20k-triangle scene that exercises the multi-block radix sort --
and frames traced over the device-built tree equal brute force."""
import numpy as np
import pytest

from conftest import scene_path

pytestmark = pytest.mark.gpu

from skybox_rt_amd import rt  # noqa: E402
from test_native_cpu import lbvh_inputs  # noqa: E402


@pytest.fixture(scope="module")
def synth(tmp_path_factory):
    from synth_scene import make_scene
    return make_scene(str(tmp_path_factory.mktemp("synth") / "synth20k.cgltrace.gz"), 20000)


def _scene(name, synth):
    return synth if name == "synth20k" else scene_path(name)


@pytest.mark.parametrize("name", ["tekkaman", "scene", "box", "carnival", "mouse", "vase",
                                  "synth20k"])
def test_gpu_bvh_equals_oracle_build(oracle_lib, synth, name):
    po = oracle_lib
    s = rt.Scene.load(_scene(name, synth))
    r = rt.Renderer(s)
    st = r.build_bvh()
    nodes, tris = r.export_bvh()
    verts, geom, _ = lbvh_inputs(s)
    on, ot, od = po.lbvh_build(verts, geom)
    assert st["depth"] == od and st["nodes"] == len(on)
    assert np.array_equal(nodes.view(np.uint32), on.view(np.uint32))
    assert np.array_equal(tris.view(np.uint32), ot.view(np.uint32))
    assert st["launches"] == 19
    # the device BVH4 collapse == oracle/lbvh.c orc_lbvh_collapse4, and its
    # binary16 planes (BVHB_HALF) == orc_half4, bit for bit: the fp32 nodes
    # with every plane rounded outward and the 64-B half records
    o4, ostack = po.lbvh_collapse4(on)
    o4r, oh = po.half4(o4)
    assert np.array_equal(r.export_bvh4().view(np.uint32), o4r.view(np.uint32))
    assert np.array_equal(r.export_bvh4h(), oh)
    assert st["stack4"] == ostack and r.gpu_bvh4


@pytest.mark.parametrize("name,size,mode,width", [
    ("tekkaman", 1024, "shadow", 0), ("tekkaman", 256, "path", 0), ("scene", 256, "shadow", 0),
    ("box", 128, "shadow", 0), ("synth20k", 192, "shadow", 0), ("tekkaman", 1024, "shadow", 2),
    ("synth20k", 192, "path", 2)])
def test_frames_over_gpu_bvh_equal_bruteforce(oracle_lib, synth, name, size, mode, width):
    """Frames over the device-built tree -- its BVH4 collapse by default,
    its BVH2 with width=2 -- equal the brute-force oracle."""
    po = oracle_lib
    path = _scene(name, synth)
    s = rt.Scene.load(path)
    r = rt.Renderer(s)
    r.configure(size, size, shadows=True, path=mode == "path", bvh_width=width)
    r.build_bvh()                       # reconfigures the renderer onto the new tree
    assert r.bvh4 == (width != 2) and r.bvh4_f16 == (width != 2)
    r.render()
    osc = po.OracleScene(po.cgltrace.load(path))
    c, _, _, k = po.rt_render(osc, po.rt_params(size, size, shadows=True, nthreads=8,
                                                path=mode == "path"))
    fb = r.framebuffer()
    assert np.array_equal(fb, c), f"{int((fb != c).sum())} pixels differ"
    st = r.stats()
    assert st["shadow_rays"] == k["shadow_rays"] and st["occluded"] == k["occluded"]


def test_instrumented_counts_over_gpu_bvh_equal_oracle_traversal(oracle_lib):
    po = oracle_lib
    s = rt.Scene.load(scene_path("tekkaman"))
    r = rt.Renderer(s)
    r.build_bvh()
    r.configure(512, 512, shadows=True, instrumented=True)
    r.render()
    st = r.stats()
    nodes, tris = r.export_bvh()
    assert r.bvh4
    _, _, _, k = po.rt_render(po.OracleScene(po.cgltrace.load(scene_path("tekkaman"))),
                              po.rt_params(512, 512, shadows=True, nthreads=8),
                              bvh=(nodes, tris, r.export_bvh4()))
    for key in ("node_visits", "tri_tests", "shadow_rays", "occluded"):
        assert st[key] == k[key], key


def test_build_rejects_scene_without_geometry():
    r = rt.Renderer(rt.Scene.load(scene_path("triangle")))
    with pytest.raises(rt.RtError):
        r.build_bvh()
