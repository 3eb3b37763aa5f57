"""Renderer and device lifecycle in one process: the
round-5 work-in-progress runs r05c / r05d died with SIGSEGV inside
rt_renderer_create while the driver's pinned completion block was being
introduced.  Several renderers created and closed in turn, two alive at once
on one device, each rendering synchronous frames (start + wait: the
completion kernel and its pinned word) and back-to-back frames: every frame
equals the first renderer's, nothing faults."""
import numpy as np
import pytest

from conftest import scene_path

pytestmark = pytest.mark.gpu

from skybox_rt_amd import rt  # noqa: E402


def _frames(r, n_sync=4, n_queued=6):
    for _ in range(n_sync):
        r.render()                      # synchronous: completion kernel + pinned word
    a = r.framebuffer().copy()
    r.set_timing(False)
    try:
        for _ in range(n_queued):       # back to back, no per-launch timing
            r.start()
        r.wait()
    finally:
        r.set_timing(True)
    b = r.framebuffer()
    assert np.array_equal(a, b)
    return a


def test_renderers_created_and_closed_in_turn():
    s = rt.Scene.load(scene_path("tekkaman"))
    ref = None
    for i in range(6):
        r = rt.Renderer(s)
        r.configure(256, 256, shadows=True, counters=False, bvh_walk=(i % 2 == 1))
        fb = _frames(r)
        ref = fb if ref is None else ref
        assert np.array_equal(fb, ref), i
        assert r.kernel_ms() > 0.0
        r.close()
    s.close()


def test_two_renderers_alive_at_once():
    s = rt.Scene.load(scene_path("tekkaman"))
    r1, r2 = rt.Renderer(s), rt.Renderer(s)
    r1.configure(256, 256, shadows=True, counters=False)
    r2.configure(256, 256, shadows=True, path=True, bounces=2, counters=False)
    a1, a2 = _frames(r1), _frames(r2)
    for _ in range(3):                  # interleaved synchronous frames
        r1.render()
        r2.render()
        assert np.array_equal(r1.framebuffer(), a1) and np.array_equal(r2.framebuffer(), a2)
    r2.close()
    assert np.array_equal(_frames(r1), a1)
    r1.close()
    s.close()
