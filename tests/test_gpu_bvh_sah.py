"""GPU binned-SAH build (kernels/bvh_sah.hip): the
device restatement of the host builder app/bvh.cpp -- binned SAH over x, y
and w, leaves of <= 4, stable partitions, padded boxes, the BVH4 collapse
that opens the largest-area internal child, binary16 planes -- produces the
scene's host-built arrays bit for bit (BVH2 nodes in preorder, triangle
records in leaf order, BVH4 nodes, rt_node4h_t records, depth, BVH4 depth
and worst-case stack), on the reference's scenes and on synthetic ones
(20k / 100k triangles: many levels and wide top-level segments; 3-9
triangles: the small-root and median paths; chain96: a tree deeper than the
build's level budget, so its launch sequence continues once); frames over it
== the oracle.  The build is one launch sequence with one read-back: a
rebuild (image resident) repeats the arrays exactly."""
import math
import os

import numpy as np
import pytest

from conftest import scene_path

pytestmark = pytest.mark.gpu

from skybox_rt_amd import rt  # noqa: E402

_paths = {}


def _host_renderer(s):
    """A renderer on the scene's host-built tree (app/bvh.cpp uploaded: env
    RT_BVH=host while it is created) -- the arrays the device build must equal."""
    old = os.environ.get("RT_BVH")
    os.environ["RT_BVH"] = "host"
    try:
        r = rt.Renderer(s)
    finally:
        if old is None:
            del os.environ["RT_BVH"]
        else:
            os.environ["RT_BVH"] = old
    assert r.bvh_stats()["method"] == rt.RT_BVH_BUILD_HOST
    return r


def _scene(name, tmp_path_factory):
    if name in _paths:
        return _paths[name]
    if name.startswith("chain"):
        from synth_scene import make_chain_scene
        path = make_chain_scene(str(tmp_path_factory.mktemp("sah") / f"{name}.cgltrace.gz"), int(name[5:]))
    elif name.startswith("synth"):
        from synth_scene import make_scene
        n = int(name[5:].replace("k", "000"))
        path = make_scene(str(tmp_path_factory.mktemp("sah") / f"{name}.cgltrace.gz"), n, seed=n)
    else:
        path = scene_path(name)
    _paths[name] = path
    return path


@pytest.mark.parametrize("name", ["tekkaman", "scene", "box", "carnival", "mouse", "vase",
                                  "evilskull", "polybump", "synth3", "synth4", "synth5",
                                  "synth9", "synth20k", "synth100k", "chain96"])
def test_gpu_sah_equals_host_build(tmp_path_factory, name):
    s = rt.Scene.load(_scene(name, tmp_path_factory))
    info = s.info()
    if info["num_geometry"] == 0:
        pytest.skip("no depth-tested geometry")
    host = _host_renderer(s)                  # the scene's host-built tree
    hn, ht = host.export_bvh()
    h4, hh = host.export_bvh4(), host.export_bvh4h()
    r = rt.Renderer(s)
    st = r.build_bvh("sah")
    dn, dt = r.export_bvh()
    assert dn.shape == hn.shape and np.array_equal(dn.view(np.uint32), hn.view(np.uint32))
    assert dt.shape == ht.shape and np.array_equal(dt.view(np.uint32), ht.view(np.uint32))
    d4 = r.export_bvh4()
    assert d4.shape == h4.shape and np.array_equal(d4.view(np.uint32), h4.view(np.uint32))
    assert np.array_equal(r.export_bvh4h(), hh)
    assert st["depth"] == info["bvh_depth"] and st["nodes"] == info["bvh_nodes"]
    assert st["nodes4"] == info["bvh4_nodes"] and st["depth4"] == info["bvh4_depth"]
    assert st["stack4"] == info["bvh4_stack"] and st["method"] == 1
    # one sequence: the init, the level budget's split launches, 7 finishing
    # launches (BVH2, BVH4) -- and, past the budget, a reset, the next levels,
    # 7 again
    budget = math.ceil(math.log2(info["num_geometry"] + 1)) + 4
    rounds = 1 if info["bvh_depth"] <= budget else 2
    assert st["launches"] == 1 + min(rounds * budget, 63) + 7 * rounds + (rounds - 1)
    if name == "chain96":
        assert rounds == 2
    print(f"{name}: {info['num_geometry']} tris, {st['nodes']} nodes, {st['launches']} launches, "
          f"build {st['build_ms']:.2f} ms (kernels {st['kernel_ms']:.2f}), host {info['bvh_ms']:.2f} ms")
    r.close()
    host.close()
    s.close()


@pytest.mark.parametrize("mode", ["shadow", "path"])
def test_frames_over_gpu_sah_equal_oracle(oracle_lib, mode):
    po = oracle_lib
    path = scene_path("tekkaman")
    s = rt.Scene.load(path)
    r = rt.Renderer(s)
    r.configure(1024, 1024, shadows=True, path=mode == "path", instrumented=True)
    r.render()
    host_fb, host_st = r.framebuffer(), r.stats()
    r.build_bvh("sah")                      # reconfigures onto the device tree
    assert r.bvh4 and r.bvh4_f16
    r.render()
    fb, st = r.framebuffer(), r.stats()
    c, _, _, k = po.rt_render(po.OracleScene(po.cgltrace.load(path)),
                              po.rt_params(1024, 1024, shadows=True, nthreads=8, path=mode == "path"))
    assert np.array_equal(fb, c) and np.array_equal(fb, host_fb)
    # the same tree: the same traversal, counter for counter
    for key in ("node_visits", "tri_tests", "layer_tests", "shadow_rays", "occluded", "bounce_rays"):
        assert st[key] == host_st[key], key
    assert st["shadow_rays"] == k["shadow_rays"] and st["occluded"] == k["occluded"]
    r.close()
    s.close()


def test_gpu_sah_deep_tree_on_stale_scratch(tmp_path_factory):
    """A tree deeper than the level budget built in arena memory another
    build has just left dirty: synth20k's SAH scratch is freed, chain96's
    build reuses those addresses, and its first sequence's finishing phases
    must not run on the partial tree (they skip on the device while the
    level after the budget still holds segments, bvh_sah.hip) -- the arrays
    still equal the host builder's."""
    big = rt.Scene.load(_scene("synth20k", tmp_path_factory))
    rb = rt.Renderer(big)
    rb.build_bvh("sah")
    rb.build_bvh("sah")
    rb.close()
    big.close()
    s = rt.Scene.load(_scene("chain96", tmp_path_factory))
    info = s.info()
    host = _host_renderer(s)
    hn, ht = host.export_bvh()
    h4, hh = host.export_bvh4(), host.export_bvh4h()
    r = rt.Renderer(s)
    for _ in range(2):
        st = r.build_bvh("sah")
        dn, dt = r.export_bvh()
        assert np.array_equal(dn.view(np.uint32), hn.view(np.uint32))
        assert np.array_equal(dt.view(np.uint32), ht.view(np.uint32))
        assert np.array_equal(r.export_bvh4().view(np.uint32), h4.view(np.uint32))
        assert np.array_equal(r.export_bvh4h(), hh)
        assert st["depth"] == info["bvh_depth"] and st["stack4"] == info["bvh4_stack"]
    r.close()
    host.close()
    s.close()


def test_gpu_sah_rebuild(tmp_path_factory):
    """A rebuild with the image and scratch resident: the same arrays every
    time, in well under a millisecond for tekkaman (one launch sequence, one
    read-back; the first build also loads the image)."""
    s = rt.Scene.load(_scene("tekkaman", tmp_path_factory))
    r = rt.Renderer(s)
    first = r.bvh_stats()
    ref = r.export_bvh(), r.export_bvh4(), r.export_bvh4h()
    times = []
    for _ in range(4):
        st = r.build_bvh("sah")
        times.append(st["build_ms"])
        (n2, t2), n4, h4 = r.export_bvh(), r.export_bvh4(), r.export_bvh4h()
        assert np.array_equal(n2.view(np.uint32), ref[0][0].view(np.uint32))
        assert np.array_equal(t2.view(np.uint32), ref[0][1].view(np.uint32))
        assert np.array_equal(n4.view(np.uint32), ref[1].view(np.uint32)) and np.array_equal(h4, ref[2])
    print(f"tekkaman SAH build: first {first['build_ms']:.3f} ms, rebuilds {[round(t, 3) for t in times]} ms, "
          f"{st['launches']} launches")
    assert min(times) < 1.0
    # the build stops at the BVH4: 7 finishing launches
    budget = math.ceil(math.log2(s.info()["num_geometry"] + 1)) + 4
    assert st["launches"] == 1 + budget + 7
    r.close()
    s.close()
