"""Per-8x8-block candidate lists built on the device (kernels/rt_setup.hip
BCOUNT .. BSORT; rt_common.h rt_bentry_t) -- the finer-grained form of the
reference's per-drawcall tile binning (sim/common/gfxutil.cpp:237-271,
tests/regression/draw3d/main.cpp:179-211), moved off the host.

* the device lists (every local block's first entry and count, every entry's
  geometry index, suffix-union rectangle and depth bound) equal the oracle's
  restatement (oracle/rt.c orc_vis_block_lists) and the host restatement
  (rt_app.cpp build_block_lists) bit for bit, for whole frames and for shards;
* frames at sizes that are not multiples of the 32x32 tile (edge waves whose
  8x8 block lies outside the image) equal the oracle with their counts;
* the lists and the tree walk (RT_BLOCK_LISTS=0) give the same frames, each
  with the oracle's counts for its mode; the size caps fall back to the walk;
* configure at 4096^2 (records + lists + 64 MiB clear) is timed."""
import os

import numpy as np
import pytest

from conftest import scene_path

pytestmark = pytest.mark.gpu

from skybox_rt_amd import rt  # noqa: E402

PAD = np.array([0, 0xFFFFFFFF, 0xFFFEFFFE, 0xFFFFFFFF], np.uint32)
_osc = {}


def _oscene(po, name):
    if name not in _osc:
        _osc[name] = po.OracleScene(po.cgltrace.load(scene_path(name)))
    return _osc[name]


def _device_lists(r):
    st = r.setup_stats()
    assert st["blist_blocks"] > 0, st
    return r.records("bidx"), r.records("blist"), st


def _check_vs_oracle(po, name, r, w, h, index=0, count=1):
    idx, ent, st = _device_lists(r)
    oidx, oent = po.vis_block_lists(_oscene(po, name), w, h, index, count)
    assert idx.shape == oidx.shape, (idx.shape, oidx.shape)
    bad = np.nonzero((idx != oidx).any(axis=1))[0]
    assert bad.size == 0, f"bidx: {bad.size} blocks differ, first {bad[:8]}"
    assert st["blist_entries"] == len(oent)
    assert ent.shape == (len(oent) + 3, 4)
    bad = np.nonzero((ent[:-3] != oent).any(axis=1))[0]
    assert bad.size == 0, f"blist: {bad.size} entries differ, first {bad[:8]}"
    assert (ent[-3:] == PAD).all()
    assert st["blist_max"] == (int(oidx[:, 1].max()) if len(oidx) else 0)


@pytest.mark.parametrize("name", ["tekkaman", "box", "scene", "carnival"])
@pytest.mark.parametrize("size", [128, 1024, 4096])
def test_device_lists_equal_oracle(oracle_lib, name, size):
    s = rt.Scene.load(scene_path(name))
    r = rt.Renderer(s)
    r.configure(size, size, shadows=True, counters=False)
    assert r.setup_stats()["device"] == 1
    _check_vs_oracle(oracle_lib, name, r, size, size)
    r.close()
    s.close()


@pytest.mark.parametrize("index,count", [(0, 8), (3, 8), (7, 8), (1, 3)])
def test_device_lists_shards_equal_oracle(oracle_lib, index, count):
    """Config 5: a rank builds the lists of its own tiles only."""
    s = rt.Scene.load(scene_path("tekkaman"))
    r = rt.Renderer(s)
    r.configure(4096, 4096, shadows=True, counters=False, shard_index=index, shard_count=count)
    _check_vs_oracle(oracle_lib, "tekkaman", r, 4096, 4096, index, count)
    assert r.setup_stats()["blist_blocks"] == r.stats()["local_tiles"] * 16
    r.close()
    s.close()


@pytest.mark.parametrize("size,path", [(1024, False), (1024, True), (257, False)])
def test_device_lists_equal_host_lists(size, path):
    s = rt.Scene.load(scene_path("tekkaman"))
    r = rt.Renderer(s)
    r.configure(size, size, shadows=True, path=path, host_setup=True)
    hidx, hent, hst = _device_lists(r)
    r.configure(size, size, shadows=True, path=path)
    didx, dent, dst = _device_lists(r)
    assert dst["device"] == 1 and hst["device"] == 0
    assert np.array_equal(didx, hidx) and np.array_equal(dent, hent)
    r.close()
    s.close()


@pytest.mark.parametrize("w,h", [(100, 37), (257, 257), (33, 65), (1000, 999)])
@pytest.mark.parametrize("name", ["tekkaman", "carnival"])
def test_ragged_frames_equal_oracle(oracle_lib, name, w, h):
    """Edge tiles overhang the image: waves whose 8x8 block lies wholly
    outside it read their block's (empty) list, never past the index."""
    po = oracle_lib
    s = rt.Scene.load(scene_path(name))
    r = rt.Renderer(s)
    r.configure(w, h, shadows=True, instrumented=True)
    assert r.setup_stats()["blist_blocks"] > 0
    r.render()
    st = r.stats()
    c, _, _, k = po.rt_render(_oscene(po, name), po.rt_params(w, h, shadows=True, nthreads=8),
                              bvh=s.bvh() + (s.bvh4(),))
    assert np.array_equal(r.framebuffer(), c)
    for key in ("tri_tests", "layer_tests", "shadow_rays", "occluded", "node_visits"):
        assert st[key] == k[key], key
    r.close()
    s.close()


@pytest.mark.parametrize("lists", [1, 0])
@pytest.mark.parametrize("path", [False, True])
def test_lists_and_walk_equal_oracle_with_counts(oracle_lib, lists, path):
    """RT_BLOCK_LISTS=0 keeps the packet walk of the tree (vnodes drive the
    primary visits); either way the frame and every count equal the oracle
    in the same mode."""
    po = oracle_lib
    os.environ["RT_BLOCK_LISTS"] = str(lists)
    try:
        s = rt.Scene.load(scene_path("tekkaman"))
        r = rt.Renderer(s)
        r.configure(512, 512, shadows=True, path=path, bounces=2, instrumented=True)
        assert (r.setup_stats()["blist_blocks"] > 0) == bool(lists)
        r.render()
        st = r.stats()
        refs, pids = r.export_vis_tree()
        c, _, _, k = po.rt_render(_oscene(po, "tekkaman"),
                                  po.rt_params(512, 512, shadows=True, path=path, bounces=2, nthreads=8,
                                               vis_lists=bool(lists)),
                                  bvh=s.bvh() + (s.bvh4(),), vis_tree=(refs, pids))
        assert np.array_equal(r.framebuffer(), c)
        for key in ("node_visits", "tri_tests", "layer_tests", "shadow_rays", "occluded", "bounce_rays"):
            assert st[key] == k[key], key
        r.close()
        s.close()
    finally:
        del os.environ["RT_BLOCK_LISTS"]


@pytest.mark.parametrize("host", [False, True])
def test_list_cap_falls_back_to_the_walk(oracle_lib, host):
    po = oracle_lib
    os.environ["RT_BLIST_MAX_ENTRIES"] = "100"
    try:
        s = rt.Scene.load(scene_path("tekkaman"))
        r = rt.Renderer(s)
        r.configure(256, 256, shadows=True, instrumented=True, host_setup=host)
        st = r.setup_stats()
        assert st["blist_blocks"] == 0 and st["blist_entries"] > 100
        r.render()
        k_gpu = r.stats()
        c, _, _, k = po.rt_render(_oscene(po, "tekkaman"),
                                  po.rt_params(256, 256, shadows=True, nthreads=8, vis_lists=False,
                                               shadow_lists=False),
                                  bvh=s.bvh() + (s.bvh4(),))
        assert np.array_equal(r.framebuffer(), c)
        assert k_gpu["tri_tests"] == k["tri_tests"] and k_gpu["node_visits"] == k["node_visits"]
        r.close()
        s.close()
    finally:
        del os.environ["RT_BLIST_MAX_ENTRIES"]


def test_configure_4096_with_lists_is_timed():
    """configure at 4096^2 (device records + lists +
    64 MiB clear) <= 2 ms; printed for the log, asserted with slack."""
    s = rt.Scene.load(scene_path("tekkaman"))
    r = rt.Renderer(s)
    best = None
    for _ in range(5):
        r.configure(4096, 4096, shadows=True, counters=False)
        st = r.setup_stats()
        best = st if best is None or st["configure_ms"] < best["configure_ms"] else best
    print(f"configure 4096^2 (device, lists): {best['configure_ms']:.3f} ms, setup {best['setup_ms']:.3f} ms, "
          f"{best['launches']} launches, {best['blist_entries']} list entries (longest {best['blist_max']})")
    assert best["blist_blocks"] == 16384 * 16
    assert best["configure_ms"] < 5.0
    r.close()
    s.close()


# ---- light-space shadow lists (rt_common.h; rt_setup.hip SCOUNT .. SSORT) ----
@pytest.mark.parametrize("name", ["tekkaman", "scene", "box"])
@pytest.mark.parametrize("light", [(0.0, 60.0, 80.0), (30.0, -20.0, 95.0), (0.0, 0.0, 0.5)])
def test_shadow_lists_equal_oracle(oracle_lib, name, light):
    """The device-built light-space lists == the oracle's (every cell's first
    entry and count, every entry's triangle record in (key, index) order, the
    key -- the squared distance from the light to the triangle's bounding box
    -- in the record's e1.w word, equal to a float32 restatement)."""
    po = oracle_lib
    s = rt.Scene.load(scene_path(name))
    r = rt.Renderer(s)
    r.configure(64, 64, shadows=True, light=light)
    st = r.setup_stats()
    assert st["slist_on"] == 1
    idx, ent = po.shadow_lists(_oscene(po, name), light)
    didx = r.records("sidx")
    slist = r.records("slist")
    assert np.array_equal(didx, idx)
    assert st["slist_entries"] == len(ent) and slist.shape == (len(ent) + 1, 12)
    geom = r.records("geom")
    got = slist[:-1].copy()
    keys = got[:, 7].copy()
    got[:, 7] = 0.0
    assert np.array_equal(got.view(np.uint32), geom[ent].view(np.uint32))
    # sl_key in float32, the kernels' operation order
    g = geom[ent].astype(np.float32)
    L = np.asarray(light, dtype=np.float32)
    ks = np.zeros(len(ent), dtype=np.float32)
    for k in range(3):
        p, q, u = g[:, k], g[:, k] + g[:, 4 + k], g[:, k] + g[:, 8 + k]
        lo = np.minimum(p, np.minimum(q, u))
        hi = np.maximum(p, np.maximum(q, u))
        d = np.where(L[k] < lo, lo - L[k], np.where(L[k] > hi, L[k] - hi, np.float32(0.0)))
        ks = (ks + d * d).astype(np.float32)
    assert np.array_equal(keys.view(np.uint32), ks.view(np.uint32))
    # each cell ascending by key
    n = idx.reshape(-1, 2)
    for o, c in n[n[:, 1] > 1][:200]:
        assert np.all(np.diff(keys[o:o + c]) >= 0)
    r.close()
    s.close()


def test_shadow_list_export_right_after_set_light(oracle_lib):
    """rt_renderer_set_light queues the new light's lists without waiting;
    an export straight after it reads their status first, so the SLIST
    export is sized by the NEW light's entry count."""
    po = oracle_lib
    s = rt.Scene.load(scene_path("tekkaman"))
    r = rt.Renderer(s)
    first, second = (0.0, 0.0, 0.5), (0.0, 60.0, 80.0)  # few entries, then many
    r.configure(64, 64, shadows=True, light=first)
    r.set_list_policy(0)  # the lists queued by set_light itself
    n_first = r.setup_stats()["slist_entries"]
    r.set_light(second)
    slist = r.records("slist")        # no setup_stats() in between
    didx = r.records("sidx")
    idx, ent = po.shadow_lists(_oscene(po, "tekkaman"), second)
    assert len(ent) != n_first
    assert slist.shape == (len(ent) + 1, 12) and np.array_equal(didx, idx)
    geom = r.records("geom")
    got = slist[:-1].copy()
    got[:, 7] = 0.0
    assert np.array_equal(got.view(np.uint32), geom[ent].view(np.uint32))
    r.close()
    s.close()


@pytest.mark.parametrize("lists", [1, 0])
@pytest.mark.parametrize("light", [(0.0, 60.0, 80.0), (-200.0, 150.0, 50.0), (5.0, 5.0, 99.5)])
def test_shadow_lists_frames_equal_oracle_with_counts(oracle_lib, lists, light):
    """Shadow rays over the light-space lists (or, RT_SHADOW_LISTS=0, the BVH
    packet walk): frame, occlusions and every count == the oracle's in the
    same mode; both frames equal."""
    po = oracle_lib
    os.environ["RT_SHADOW_LISTS"] = str(lists)
    try:
        s = rt.Scene.load(scene_path("tekkaman"))
        r = rt.Renderer(s)
        r.configure(512, 512, shadows=True, light=light, instrumented=True)
        assert r.setup_stats()["slist_on"] == lists
        r.render()
        st = r.stats()
        c, _, _, k = po.rt_render(_oscene(po, "tekkaman"),
                                  po.rt_params(512, 512, shadows=True, light=light, nthreads=8,
                                               shadow_lists=bool(lists)),
                                  bvh=s.bvh() + (s.bvh4(),))
        assert np.array_equal(r.framebuffer(), c)
        for key in ("node_visits", "tri_tests", "layer_tests", "shadow_rays", "occluded"):
            assert st[key] == k[key], key
        r.close()
        s.close()
    finally:
        del os.environ["RT_SHADOW_LISTS"]
