"""The setup as one stream-ordered launch sequence and the moving light
(rt_renderer_set_light; kernels/rt_setup.hip SPROJ .. SSORT, setup_common.h
launch sequences).  The reference re-bins its scene on the host for every
render (tests/regression/draw3d/main.cpp:179-211 -> gfxutil.cpp:103-276);
here only the light-dependent structure, the light-space shadow lists, is
rebuilt when the light moves, queued on the driver's stream behind the
frames already started.

* set_light with the lists queued at once (set_list_policy(0)): a frame
  after it equals the oracle for the new light, counters included (the
  lists' own scan), and the device lists equal the oracle's;
* the default policy (the moving light): the frames after a light change
  trace their shadow rays by the BVH packet walk -- frame and counters the
  oracle's BVH mode -- until the light has stayed for the policy's frames,
  then the lists are queued and the frames scan them (list-mode counters);
* frames started back to back with a light change between them: the last
  frame is the new light's (stream order, no host wait);
* the path tracer's shadow rays follow the light too;
* list capacities too small for the entries (env RT_SETUP_BCAP /
  RT_SETUP_SCAP) overflow, the host refills at the exact size: lists and
  frames still equal the oracle; a set_light whose lists overflow falls back
  to the BVH walk for its frames (the device's verdict) until settled;
* cold configures (new resolution, new light) are timed: 4096^2 <= 2 ms."""
import os

import numpy as np
import pytest

from conftest import scene_path

pytestmark = pytest.mark.gpu

from skybox_rt_amd import rt  # noqa: E402

LIGHTS = [(0.0, 60.0, 80.0), (20.0, 50.0, 85.0), (-200.0, 150.0, 50.0), (5.0, 5.0, 99.5),
          (30.0, -20.0, 95.0)]
_osc = {}


def _oscene(po, name):
    if name not in _osc:
        _osc[name] = po.OracleScene(po.cgltrace.load(scene_path(name)))
    return _osc[name]


def _oracle(po, s, w, h, light, **kw):
    return po.rt_render(_oscene(po, "tekkaman"),
                        po.rt_params(w, h, shadows=True, light=light, nthreads=8, **kw),
                        bvh=s.bvh() + (s.bvh4(),))


def _lists_equal_oracle(po, r, light):
    idx, ent = po.shadow_lists(_oscene(po, "tekkaman"), light)
    assert np.array_equal(r.records("sidx"), idx)
    slist = r.records("slist")
    assert slist.shape == (len(ent) + 1, 12)
    got = slist[:-1].copy()
    got[:, 7] = 0.0
    assert np.array_equal(got.view(np.uint32), r.records("geom")[ent].view(np.uint32))


def test_set_light_frames_and_lists_equal_oracle(oracle_lib):
    po = oracle_lib
    s = rt.Scene.load(scene_path("tekkaman"))
    r = rt.Renderer(s)
    r.configure(512, 512, shadows=True, light=LIGHTS[0], instrumented=True)
    r.set_list_policy(0)
    assert r.setup_stats()["slist_built"] == 1
    for L in LIGHTS[1:]:
        r.set_light(L)
        # the status read settles the lists: a light whose entries exceed
        # the capacity (LIGHTS[3], next to the model) is refilled at the
        # exact size here, so the frame below scans the lists either way
        ss = r.setup_stats()
        assert ss["slist_on"] == 1 and ss["slist_built"] == 1, ss
        r.render()
        st = r.stats()
        c, _, _, k = _oracle(po, s, 512, 512, L)
        assert np.array_equal(r.framebuffer(), c), L
        for key in ("tri_tests", "layer_tests", "shadow_rays", "occluded", "geometry_hits"):
            assert st[key] == k[key], (L, key)
        _lists_equal_oracle(po, r, L)
    r.close()
    s.close()


@pytest.mark.parametrize("defer", [0, 8])
def test_set_light_between_queued_frames(oracle_lib, defer):
    """start(A) ; set_light(B) ; start ; set_light(C) ; start ; wait: the last
    frame is C's, and the light changes never waited for the frames (lists
    queued at once, or deferred: the frames walk the BVH)."""
    po = oracle_lib
    s = rt.Scene.load(scene_path("tekkaman"))
    r = rt.Renderer(s)
    r.configure(1024, 1024, shadows=True, light=LIGHTS[0], counters=False)
    r.set_list_policy(defer)
    r.render()
    for _ in range(3):
        for L in LIGHTS[1:4]:
            r.start()
            r.set_light(L)
        r.start()
    r.wait()
    c, _, _, _ = _oracle(po, s, 1024, 1024, LIGHTS[3])
    assert np.array_equal(r.framebuffer(), c)
    ss = r.setup_stats()
    assert (ss["slist_on"], ss["slist_stale"]) == ((1, 0) if defer == 0 else (0, 1)), ss
    r.close()
    s.close()


@pytest.mark.parametrize("path", [False, True])
def test_moving_light_defers_lists(oracle_lib, path):
    """The default policy with 3 frames: after a light change the frames
    trace their shadow rays by the BVH packet walk (frame, occlusions and
    counters == the oracle's BVH mode) and no lists are built; the 4th frame
    with the same light has its lists queued before it and scans them
    (list-mode counters, lists == the oracle's)."""
    po = oracle_lib
    s = rt.Scene.load(scene_path("tekkaman"))
    r = rt.Renderer(s)
    kw = dict(path=True, bounces=2) if path else {}
    r.configure(256, 256, shadows=True, light=LIGHTS[0], instrumented=True, **kw)
    r.set_list_policy(3)
    keys = ("tri_tests", "node_visits", "shadow_rays", "occluded") + (("bounce_rays",) if path else ())
    for L in LIGHTS[1:3]:
        r.set_light(L)
        cb, _, _, kb = _oracle(po, s, 256, 256, L, shadow_lists=False, **kw)
        for i in range(4):
            r.render()
            st, ss = r.stats(), r.setup_stats()
            if i < 3:
                assert ss["slist_on"] == 0 and ss["slist_stale"] == 1, (L, i, ss)
                assert np.array_equal(r.framebuffer(), cb), (L, i)
                for key in keys:
                    assert st[key] == kb[key], (L, i, key)
        assert ss["slist_on"] == 1 and ss["slist_stale"] == 0, ss
        c, _, _, k = _oracle(po, s, 256, 256, L, **kw)
        assert np.array_equal(r.framebuffer(), c) and np.array_equal(c, cb)
        for key in keys:
            assert st[key] == k[key], (L, key)
        if not path:
            _lists_equal_oracle(po, r, L)
    r.close()
    s.close()


def test_set_light_path_tracer(oracle_lib):
    po = oracle_lib
    s = rt.Scene.load(scene_path("tekkaman"))
    r = rt.Renderer(s)
    r.configure(256, 256, shadows=True, path=True, bounces=2, light=LIGHTS[0], instrumented=True)
    r.set_list_policy(0)
    for L in LIGHTS[1:3]:
        r.set_light(L)
        r.render()
        st = r.stats()
        c, _, _, k = _oracle(po, s, 256, 256, L, path=True, bounces=2)
        assert np.array_equal(r.framebuffer(), c), L
        for key in ("tri_tests", "node_visits", "shadow_rays", "occluded", "bounce_rays"):
            assert st[key] == k[key], (L, key)
    r.close()
    s.close()


def test_set_light_without_lists(oracle_lib):
    """bvh_walk: no lists -- set_light moves only the light; the shadow
    packet walk sees it."""
    po = oracle_lib
    s = rt.Scene.load(scene_path("tekkaman"))
    r = rt.Renderer(s)
    r.configure(256, 256, shadows=True, light=LIGHTS[0], bvh_walk=True, instrumented=True)
    r.set_light(LIGHTS[2])
    r.render()
    st = r.stats()
    c, _, _, k = _oracle(po, s, 256, 256, LIGHTS[2], vis_lists=False, shadow_lists=False)
    assert np.array_equal(r.framebuffer(), c)
    assert st["occluded"] == k["occluded"] and st["node_visits"] == k["node_visits"]
    assert r.setup_stats()["slist_on"] == 0
    r.close()
    s.close()


def test_list_capacity_overflow_refills(oracle_lib, monkeypatch):
    """Capacities far below the entries: the block lists and the shadow lists
    overflow, the host refills them at the exact size (configure), and a
    set_light whose lists overflow renders by the BVH walk until its status
    is read, then by the refilled lists -- every frame the oracle's."""
    po = oracle_lib
    monkeypatch.setenv("RT_SETUP_BCAP", "100")
    monkeypatch.setenv("RT_SETUP_SCAP", "1000")
    s = rt.Scene.load(scene_path("tekkaman"))
    r = rt.Renderer(s)
    r.configure(512, 512, shadows=True, light=LIGHTS[0], instrumented=True)
    r.set_list_policy(0)
    ss = r.setup_stats()
    assert ss["blist_blocks"] > 0 and ss["blist_entries"] > 100 and ss["slist_on"] == 1, ss
    oidx, oent = po.vis_block_lists(_oscene(po, "tekkaman"), 512, 512, 0, 1)
    assert np.array_equal(r.records("bidx"), oidx)
    assert np.array_equal(r.records("blist")[:-3], oent)
    _lists_equal_oracle(po, r, LIGHTS[0])
    r.render()
    c, _, _, k = _oracle(po, s, 512, 512, LIGHTS[0])
    assert np.array_equal(r.framebuffer(), c)
    # LIGHTS[3] (next to the model) has far more entries than LIGHTS[0]'s
    r.set_light(LIGHTS[3])
    r.render()
    c3, _, _, k3 = _oracle(po, s, 512, 512, LIGHTS[3])
    assert np.array_equal(r.framebuffer(), c3)
    ss = r.setup_stats()  # reads the status: overflow -> exact refill
    assert ss["slist_on"] == 1 and ss["slist_entries"] > 1000
    r.render()
    assert np.array_equal(r.framebuffer(), c3)
    assert r.stats()["tri_tests"] == k3["tri_tests"]
    _lists_equal_oracle(po, r, LIGHTS[3])
    r.close()
    s.close()


@pytest.mark.parametrize("side,limit_ms", [(1024, 0.25), (4096, 2.0)])
def test_cold_configure_is_timed(side, limit_ms):
    """a cold configure -- new resolution, new light:
    records, block lists, shadow lists, work order, one stream-ordered
    sequence -- timed on fresh renderers (best of 3), printed for the log."""
    s = rt.Scene.load(scene_path("tekkaman"))
    best = None
    for i in range(3):
        r = rt.Renderer(s)
        r.configure(side, side, shadows=True, light=(0.0, 60.0 - i, 80.0), counters=False)
        st = r.setup_stats()
        assert st["slist_built"] == 1 and st["slist_on"] == 1 and st["blist_blocks"] > 0
        best = st if best is None or st["configure_ms"] < best["configure_ms"] else best
        r.close()
    print(f"cold configure {side}^2: {best['configure_ms']:.3f} ms (setup {best['setup_ms']:.3f}, "
          f"{best['launches']} launches, {best['blist_entries']} block-list + {best['slist_entries']} "
          f"shadow-list entries)")
    assert best["configure_ms"] < limit_ms
    s.close()


@pytest.mark.parametrize("env", [{"RT_SETUP_FOLD": "0"}, {"RT_SETUP_PART": "0"},
                                 {"RT_SETUP_FOLD": "0", "RT_SETUP_PART": "0"}])
def test_setup_sequence_forms_equal_oracle(oracle_lib, monkeypatch, env):
    """The setup sequence's other forms -- the one-workgroup scan launches
    instead of the folded scans (RT_SETUP_FOLD=0), every sub-phase on the
    whole grid in turn instead of side by side (RT_SETUP_PART=0) -- build
    the same block lists, shadow lists and frames as the oracle."""
    po = oracle_lib
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    s = rt.Scene.load(scene_path("tekkaman"))
    r = rt.Renderer(s)
    r.configure(512, 512, shadows=True, light=LIGHTS[1], instrumented=True)
    ss = r.setup_stats()
    assert ss["slist_on"] == 1 and ss["blist_blocks"] > 0
    oidx, oent = po.vis_block_lists(_oscene(po, "tekkaman"), 512, 512, 0, 1)
    assert np.array_equal(r.records("bidx"), oidx)
    assert np.array_equal(r.records("blist")[:-3], oent)
    _lists_equal_oracle(po, r, LIGHTS[1])
    r.render()
    c, _, _, k = _oracle(po, s, 512, 512, LIGHTS[1])
    assert np.array_equal(r.framebuffer(), c)
    r.set_list_policy(0)
    r.set_light(LIGHTS[2])
    assert r.setup_stats()["slist_on"] == 1  # settles the lists (their entry count)
    r.render()
    c2, _, _, _ = _oracle(po, s, 512, 512, LIGHTS[2])
    assert np.array_equal(r.framebuffer(), c2)
    _lists_equal_oracle(po, r, LIGHTS[2])
    r.close()
    s.close()
