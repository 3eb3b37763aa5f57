"""Device-side per-resolution setup (kernels/rt_setup.hip; SURVEY.md 8(f)
rank 2, the reference's per-drawcall host pre-pass draw3d/main.cpp:179-211
-> graphics::Binning, gfxutil.cpp:103-276).

Every record the device builds -- rt_prim_t shading records, primary
visibility (covered-pixel rectangle, depth bound), rt_vtri_t leaf / layer /
flat-list records, the traversed tree's rt_vnode_t, the tile work order,
the triangle records of creation -- equals the host restatement
(app/setup.cpp, app/vis.cpp; RT_RENDER_HOST_SETUP) bit for bit; the
visibility records also equal the oracle's brute force (oracle/vis.c), and
frames built on the device records equal the oracle incl. traversal counts.
Scenes: the reference's RT scenes, a 20k-triangle synthetic scene, a fuzz
scene with corners behind the eye and far outside the viewport (culled
setups), a scene of huge triangles (rows whose edge values wrap int32: the
pixel-by-pixel path) with zero-area ones (degenerate setups), the
device-built tree (absorbed zero nodes) and shards."""
import os

import numpy as np
import pytest

from conftest import scene_path

pytestmark = pytest.mark.gpu

from skybox_rt_amd import rt  # noqa: E402

REC_RT = ("prims", "vis", "vnodes", "vtris", "vlayers", "vgeom", "order")

_cache = {}


def _scene(name, tmp_path_factory=None):
    if name in _cache:
        return _cache[name]
    if name == "synth20k":
        from synth_scene import make_scene
        path = make_scene(str(tmp_path_factory.mktemp("s") / "synth20k.cgltrace.gz"), 20000)
    elif name == "fuzz":
        from synth_scene import make_scene
        path = make_scene(str(tmp_path_factory.mktemp("f") / "fuzz.cgltrace.gz"), 3000, seed=7,
                          size=1.2, w_range=(0.5, 110.0), spread=1.6, w_jitter=3.0)
    elif name == "huge":  # triangles ~100 viewports wide: rows whose edge values wrap int32
        from synth_scene import make_scene
        path = make_scene(str(tmp_path_factory.mktemp("h") / "huge.cgltrace.gz"), 300, seed=3,
                          size=300.0, w_range=(60.0, 110.0), spread=1.0, degenerate=20)
    else:
        path = scene_path(name)
    _cache[name] = path
    return path


def _records(r, names):
    out = {n: r.records(n) for n in names}
    if r.setup_stats()["blist_blocks"]:  # the per-block candidate lists
        out.update({n: r.records(n) for n in ("bidx", "blist")})
    return out


def _equal(a, b, what):
    assert a.shape == b.shape, (what, a.shape, b.shape)
    bad = np.nonzero((a.view(np.uint32) != b.view(np.uint32)).any(axis=-1))[0]
    assert bad.size == 0, f"{what}: {bad.size} records differ, first {bad[:8]}"


def _device_vs_host(r, w, h, **kw):
    r.configure(w, h, host_setup=True, **kw)
    host = _records(r, REC_RT)
    hs = r.setup_stats()
    r.render()
    fb_host = r.framebuffer()
    r.configure(w, h, **kw)
    dev = _records(r, REC_RT)
    ds = r.setup_stats()
    assert ds["device"] == 1 and hs["device"] == 0
    assert ds["heavy_tiles"] == hs["heavy_tiles"]
    assert sorted(dev) == sorted(host)
    for n in dev:
        _equal(dev[n], host[n], n)
    r.render()
    assert np.array_equal(r.framebuffer(), fb_host)
    return dev, ds


@pytest.mark.parametrize("name", ["tekkaman", "triangle", "box", "scene", "carnival"])
@pytest.mark.parametrize("w,h", [(8, 8), (64, 64), (100, 37), (128, 128), (1024, 1024)])
def test_device_setup_equals_host_setup(oracle_lib, name, w, h):
    s = rt.Scene.load(scene_path(name))
    r = rt.Renderer(s)
    dev, _ = _device_vs_host(r, w, h, shadows=True)
    # the visibility records also equal the oracle's brute force
    osc = oracle_lib.OracleScene(oracle_lib.cgltrace.load(scene_path(name)))
    assert np.array_equal(dev["vis"][:, :3], oracle_lib.vis_prims(osc, w, h))
    assert np.array_equal(dev["vis"][:, 3] != 0, dev["vis"][:, 0] != 0xFFFF)
    r.close()
    s.close()


def test_device_setup_4096_and_path_split(oracle_lib):
    """Config 5's resolution and config 4's split tiles (heavy count) on the
    device setup == host setup."""
    s = rt.Scene.load(scene_path("tekkaman"))
    r = rt.Renderer(s)
    _, ds = _device_vs_host(r, 4096, 4096, shadows=True, counters=False)
    assert ds["heavy_tiles"] > 0
    _device_vs_host(r, 1024, 1024, path=True)
    r.close()
    s.close()


@pytest.mark.parametrize("index,count", [(0, 8), (3, 8), (1, 3)])
def test_device_setup_shards(index, count):
    s = rt.Scene.load(scene_path("tekkaman"))
    r = rt.Renderer(s)
    _device_vs_host(r, 1024, 1024, shadows=True, shard_index=index, shard_count=count)
    r.close()
    s.close()


@pytest.mark.parametrize("name,size", [("synth20k", 512), ("fuzz", 256), ("fuzz", 1000),
                                       ("huge", 512), ("huge", 257)])
def test_device_setup_synthetic(oracle_lib, tmp_path_factory, name, size):
    path = _scene(name, tmp_path_factory)
    s = rt.Scene.load(path)
    r = rt.Renderer(s)
    dev, _ = _device_vs_host(r, size, size, shadows=True)
    if size <= 512:
        osc = oracle_lib.OracleScene(oracle_lib.cgltrace.load(path))
        assert np.array_equal(dev["vis"][:, :3], oracle_lib.vis_prims(osc, size, size))
    if name == "fuzz":  # the fuzz scene does reach the culled / empty paths
        assert (dev["vis"][:, 3] == 0).sum() > 0
    if name == "huge":  # zero-area triangles: degenerate setups (all-zero records)
        assert (dev["prims"][:, :30] == 0).all(axis=1).sum() == 20
    r.close()
    s.close()


@pytest.mark.parametrize("name,width", [("tekkaman", 0), ("tekkaman", 2), ("synth20k", 0)])
def test_device_setup_over_device_tree(tmp_path_factory, name, width):
    """The device-built tree (BVH4 with zero records at absorbed nodes, or
    its BVH2) under the device setup == under the host setup."""
    s = rt.Scene.load(_scene(name, tmp_path_factory))
    r = rt.Renderer(s)
    r.build_bvh()
    _device_vs_host(r, 512, 512, shadows=True, bvh_width=width)
    r.close()
    s.close()


def test_device_setup_frames_equal_oracle_with_counts(oracle_lib):
    """Instrumented frames on device-built records: image and traversal
    counts == the oracle's (the block lists drive the primary tests, the
    BVH4 the shadow rays' visits)."""
    po = oracle_lib
    path = scene_path("tekkaman")
    s = rt.Scene.load(path)
    r = rt.Renderer(s)
    r.configure(512, 512, shadows=True, instrumented=True)
    assert r.setup_stats()["device"] == 1
    r.render()
    st = r.stats()
    refs, pids = r.export_vis_tree()
    c, _, _, k = po.rt_render(po.OracleScene(po.cgltrace.load(path)),
                              po.rt_params(512, 512, shadows=True, nthreads=8),
                              bvh=s.bvh() + (s.bvh4(),))
    assert np.array_equal(r.framebuffer(), c)
    for key in ("node_visits", "tri_tests", "layer_tests", "shadow_rays", "occluded"):
        assert st[key] == k[key], key
    assert len(refs) == s.info()["bvh4_nodes"] and len(pids) == s.info()["bvh_tris"]
    r.close()
    s.close()


def test_device_setup_raster_and_creation_records():
    """Raster mode: device prims / bbox == host; the creation-time triangle
    records (ptris, geom) built on the device == the host loop's."""
    s = rt.Scene.load(scene_path("scene"))
    os.environ["RT_SETUP"] = "host"
    try:
        rh = rt.Renderer(s)
    finally:
        del os.environ["RT_SETUP"]
    rd = rt.Renderer(s)
    for n in ("ptris", "geom"):
        rh.configure(64, 64, shadows=True)
        rd.configure(64, 64, shadows=True)
        _equal(rd.records(n), rh.records(n), n)
    for size in (32, 128, 333):
        rd.configure(size, size, raster=True, host_setup=True)
        hp, hb = rd.records("prims"), rd.records("bbox")
        rd.render()
        fh = rd.framebuffer()
        rd.configure(size, size, raster=True)
        _equal(rd.records("prims"), hp, "prims")
        _equal(rd.records("bbox"), hb, "bbox")
        rd.render()
        assert np.array_equal(rd.framebuffer(), fh)
    rh.close()
    rd.close()
    s.close()


def test_device_setup_is_faster_at_4096():
    """The point of moving the pre-pass: configure at 4096^2 (records +
    64 MiB clear) on the device vs the host loops; printed for the log."""
    s = rt.Scene.load(scene_path("tekkaman"))
    r = rt.Renderer(s)
    t = {}
    for host in (True, False, True, False):
        r.configure(4096, 4096, shadows=True, counters=False, host_setup=host)
        t[host] = r.setup_stats()
    print(f"configure 4096^2: host {t[True]['configure_ms']:.2f} ms (setup {t[True]['setup_ms']:.2f}), "
          f"device {t[False]['configure_ms']:.2f} ms (setup {t[False]['setup_ms']:.2f}, "
          f"{t[False]['launches']} launches)")
    assert t[False]["setup_ms"] < t[True]["setup_ms"]
    r.close()
    s.close()
