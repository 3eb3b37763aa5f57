"""GPU parity tests of the path tracer (pt_kernel.hip; SURVEY.md 8(a) row A7,
BASELINE config 4) through the C-ABI against the oracle's restatement
(oracle/rt.c path_trace): framebuffers and ray counters bit-exact.  No
reference exists for this row (parity unpinned beyond the oracle)."""
import numpy as np
import pytest

from conftest import scene_path

pytestmark = pytest.mark.gpu

from skybox_rt_amd import rt  # noqa: E402

_cache = {}


def setup(po, name):
    if name not in _cache:
        s = rt.Scene.load(scene_path(name))
        _cache[name] = (s, rt.Renderer(s), po.OracleScene(po.cgltrace.load(scene_path(name))),
                        s.bvh() + (s.bvh4(),))
    return _cache[name]


@pytest.fixture(scope="module")
def po(oracle_lib):
    return oracle_lib


CASES = [("tekkaman", 128, 4, 0x5EED), ("tekkaman", 256, 4, 0x5EED), ("tekkaman", 1024, 4, 0x5EED),
         ("tekkaman", 333, 4, 0x5EED), ("tekkaman", 256, 0, 0x5EED), ("tekkaman", 256, 1, 99),
         ("tekkaman", 256, 8, 3), ("box", 128, 4, 0x5EED), ("scene", 256, 4, 0x5EED),
         ("carnival", 128, 4, 0x5EED), ("triangle", 64, 4, 0x5EED)]


@pytest.mark.parametrize("name,size,bounces,seed", CASES)
def test_pt_kernel_bit_exact_vs_oracle(po, name, size, bounces, seed):
    s, r, osc, bvh = setup(po, name)
    r.configure(size, size, path=True, bounces=bounces, seed=seed)
    r.render()
    fb = r.framebuffer()
    st = r.stats()
    c, _, _, k = po.rt_render(osc, po.rt_params(size, size, path=True, bounces=bounces, seed=seed,
                                                nthreads=8), bvh=bvh)
    assert np.array_equal(fb, c), f"{int((fb != c).sum())} pixels differ"
    assert st["primary_rays"] == k["primary_rays"] == size * size
    for key in ("geometry_hits", "shadow_rays", "occluded", "bounce_rays"):
        assert st[key] == k[key], key
    if r.setup_stats()["path_queue"]:
        # + pt_queue's tasks: 64 segments x (deepest segment's waves) x 64 lanes,
        # the deepest segment holding at most every geometry hit
        extra = st["tasks"] - st["num_tasks"]
        per = 64 * 64
        assert extra >= per and extra % per == 0
        assert extra <= per * max(1, -(-st["geometry_hits"] // 16))
    else:
        assert st["tasks"] == st["num_tasks"]


def test_pt_sharded_reassembles(po):
    s, r, _, _ = setup(po, "tekkaman")
    W = H = 384
    r.configure(W, H, path=True)
    r.render()
    full = r.framebuffer()
    parts, rays = [], 0
    for i in range(3):
        r.configure(W, H, path=True, shard_index=i, shard_count=3)
        r.render()
        parts.append(r.framebuffer().copy())
        rays += r.stats()["bounce_rays"]
    r.configure(W, H, path=True)
    r.render()
    assert rays == r.stats()["bounce_rays"]
    assert np.array_equal(rt.deinterleave_tiles(parts, W, H), full)


def test_pt_repeatable_and_primary_mode_unaffected(po):
    s, r, _, _ = setup(po, "tekkaman")
    r.configure(512, 512, shadows=True)
    r.render()
    a = r.framebuffer()
    r.configure(512, 512, path=True)
    r.render()
    p1 = r.framebuffer()
    r.render()
    assert np.array_equal(p1, r.framebuffer())
    r.configure(512, 512, shadows=True)
    r.render()
    assert np.array_equal(a, r.framebuffer())


@pytest.mark.parametrize("width", (0, 2))
def test_pt_instrumented_counters_equal_oracle_traversal(po, width):
    s, r, osc, bvh = setup(po, "tekkaman")
    for size in (256, 1024):
        r.configure(size, size, path=True, instrumented=True, bvh_width=width)
        r.render()
        st = r.stats()
        c, _, _, k = po.rt_render(osc, po.rt_params(size, size, path=True, nthreads=8,
                                                    path_queue=r.setup_stats()["path_queue"]),
                                  bvh=bvh if r.bvh4 else bvh[:2])
        for key in ("node_visits", "tri_tests", "layer_tests", "shaded", "texel_bytes",
                    "shadow_rays", "bounce_rays", "occluded"):
            assert st[key] == k[key], key
        assert np.array_equal(r.framebuffer(), c)


@pytest.mark.parametrize("size,bounces", [(256, 4), (1024, 4), (333, 2)])
def test_pt_compact_image_bit_exact_vs_oracle(po, size, bounces):
    """The block-compacted path tracer (PT_MODE 0, lib/pt_compact/) renders
    the same frame as the default per-lane image and the oracle."""
    import os
    from skybox_rt_amd import _lib
    s, _, osc, bvh = setup(po, "tekkaman")
    r = rt.Renderer(s, kernel_dir=os.path.join(_lib.LIB_DIR, "pt_compact"))
    r.configure(size, size, path=True, bounces=bounces)
    r.render()
    st = r.stats()
    c, _, _, k = po.rt_render(osc, po.rt_params(size, size, path=True, bounces=bounces, nthreads=8),
                              bvh=bvh)
    assert np.array_equal(r.framebuffer(), c)
    for key in ("geometry_hits", "shadow_rays", "occluded", "bounce_rays"):
        assert st[key] == k[key], key
    assert st["block"] == 256                              # the compacting image ran
    r.close()


@pytest.mark.parametrize("queue", [1, 0])
@pytest.mark.parametrize("size,bounces", [(1024, 4), (333, 3)])
def test_pt_two_kernels_and_one_kernel_equal_oracle(po, queue, size, bounces):
    """Config 4 in two kernels (pt_primary appends path starts to a compacted
    queue, pt_queue runs them on full waves: one launch group) or, with
    RT_PT_QUEUE=0, in the one-kernel pt_kernel: the same frame, every count
    equal to the oracle's in the same mode (the primary pass counts per 8x8
    block in the two-kernel form), repeatable frame after frame (the queue
    counters are reset by the last pt_queue wave)."""
    import os
    os.environ["RT_PT_QUEUE"] = str(queue)
    try:
        s, _, osc, bvh = setup(po, "tekkaman")
        r = rt.Renderer(s)
        r.configure(size, size, path=True, bounces=bounces, instrumented=True)
        assert r.setup_stats()["path_queue"] == queue
        r.render()
        st = r.stats()
        c, _, _, k = po.rt_render(osc, po.rt_params(size, size, path=True, bounces=bounces, nthreads=8,
                                                    path_queue=bool(queue)), bvh=bvh)
        assert np.array_equal(r.framebuffer(), c)
        for key in ("primary_rays", "geometry_hits", "node_visits", "tri_tests", "layer_tests",
                    "shaded", "texel_bytes", "shadow_rays", "bounce_rays", "occluded"):
            assert st[key] == k[key], key
        r.configure(size, size, path=True, bounces=bounces, counters=False)
        for _ in range(3):
            r.render()
            assert np.array_equal(r.framebuffer(), c)
        r.close()
    finally:
        del os.environ["RT_PT_QUEUE"]
