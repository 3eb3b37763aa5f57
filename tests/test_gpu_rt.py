"""GPU parity tests (MI355X): the HIP path through the C-ABI against the
oracle.  Integer/byte outputs (ARGB pixels, counters) must be bit-exact; the
fp32 hit distance t is compared through the pixels it selects (pid/colour)."""
import ctypes as C
import os
import subprocess
import struct

import numpy as np
import pytest

from conftest import GOLDEN, scene_path

pytestmark = pytest.mark.gpu

from skybox_rt_amd import _lib, rt, vortex  # noqa: E402


@pytest.fixture(scope="module")
def po(oracle_lib):
    return oracle_lib


def _png(path):
    from PIL import Image
    return np.array(Image.open(path).convert("RGBA"))


_cache = {}


def renderer(name):
    if name not in _cache:
        s = rt.Scene.load(scene_path(name))
        _cache[name] = (s, rt.Renderer(s))
    return _cache[name]


def oracle_scene(po, name):
    key = ("oracle", name)
    if key not in _cache:
        _cache[key] = po.OracleScene(po.cgltrace.load(scene_path(name)))
    return _cache[key]


# ---------------------------------------------------------------- driver/ABI --
def test_device_caps_and_memory_roundtrip():
    d = vortex.Device()
    try:
        assert d.caps(vortex.VX_CAPS_NUM_THREADS) == 64
        assert d.caps(vortex.VX_CAPS_NUM_CORES) >= 1
        isa = d.caps(vortex.VX_CAPS_ISA_FLAGS)
        assert isa & vortex.VX_ISA_EXT_RASTER and isa & vortex.VX_ISA_EXT_TEX
        with pytest.raises(vortex.VortexError):
            d.caps(0x99)
        b = d.mem_alloc(1 << 20)
        addr = b.address
        assert addr >= 0x10000 and addr % 64 == 0 and (addr // 64) < (1 << 32)
        data = np.random.default_rng(1).integers(0, 256, 1 << 20, dtype=np.uint8).tobytes()
        b.write(data)
        assert b.read() == data
        assert b.read(4096, offset=12345) == data[12345:12345 + 4096]
        with pytest.raises(vortex.VortexError):
            b.write(b"x" * 16, offset=(1 << 20) - 8)       # past the buffer: -1
        fr0, used0 = d.mem_info()
        b.free()
        fr1, used1 = d.mem_info()
        assert used1 < used0 and fr1 > fr0
        d.dcr_write(0x30, 0x1234)
        assert d.dcr_read(0x30) == 0x1234
        with pytest.raises(vortex.VortexError):
            d.dcr_read(0x31)                                # never written
    finally:
        d.close()


@pytest.mark.parametrize("dim,grid", [(1, (1,)), (1, (100003,)), (2, (300, 7)), (3, (5, 9, 11)),
                                      (1, (3 * 256 * 256 + 17,))])
def test_vx_spawn_threads_decomposition(dim, grid):
    d = vortex.Device()
    try:
        k = d.upload_kernel_file(os.path.join(_lib.LIB_DIR, "spawn_test.vxbin"))
        n = int(np.prod(grid))
        out = d.mem_alloc(4 * n)
        hits = d.mem_alloc(4 * n)
        hits.write(bytes(4 * n))
        g = list(grid) + [1] * (3 - len(grid))
        args = d.upload_bytes(struct.pack("<IIIIQQ", dim, *g, out.address, hits.address))
        d.start(k, args)
        d.ready_wait()
        assert d.mpm_query(vortex.VX_CSR_MINSTRET) == n
        assert d.mpm_query(vortex.VX_CSR_MCYCLE) > 0
        o = np.frombuffer(out.read(), np.uint32)
        h = np.frombuffer(hits.read(), np.uint32)
        assert np.all(h == 1)
        t = np.arange(n, dtype=np.int64)
        exp = (t % g[0]) | (((t // g[0]) % g[1]) << 10) | ((t // (g[0] * g[1])) << 20)
        assert np.array_equal(o, exp.astype(np.uint32))
    finally:
        d.close()


# ------------------------------------------------------------ RT parity -----
CASES = [("tekkaman", 128, False), ("tekkaman", 128, True), ("tekkaman", 256, True),
         ("tekkaman", 1024, True), ("tekkaman", 1000, True), ("tekkaman", 333, False),
         ("triangle", 64, False), ("box", 128, True), ("scene", 256, True),
         ("carnival", 128, True)]


@pytest.mark.parametrize("name,size,shadows,width",
                         [c + (0,) for c in CASES] +
                         [("tekkaman", 1024, True, 2), ("scene", 256, True, 2), ("box", 128, True, 2)])
def test_rt_kernel_bit_exact_vs_oracle(po, name, size, shadows, width):
    """Both traversals (4-wide default, binary with width=2) against the
    brute-force oracle: the BVH may only change the work, never the frame."""
    s, r = renderer(name)
    r.configure(size, size, shadows=shadows, bvh_width=width)
    r.render()
    fb = r.framebuffer()
    st = r.stats()
    c, p, t, k = po.rt_render(oracle_scene(po, name), po.rt_params(size, size, shadows=shadows,
                                                                    nthreads=8))
    assert np.array_equal(fb, c), f"{int((fb != c).sum())} pixels differ"
    assert st["primary_rays"] == k["primary_rays"] == size * size
    assert st["shadow_rays"] == k["shadow_rays"]
    assert st["geometry_hits"] == k["geometry_hits"]
    assert st["occluded"] == k["occluded"]
    assert st["tasks"] == st["num_tasks"]


@pytest.mark.parametrize("width", (0, 2))
def test_rt_instrumented_counters_equal_oracle_traversal(po, width):
    s, r = renderer("tekkaman")
    for size in (256, 1024):
        r.configure(size, size, shadows=True, instrumented=True, bvh_width=width)
        r.render()
        st = r.stats()
        _, _, _, k = po.rt_render(oracle_scene(po, "tekkaman"),
                                  po.rt_params(size, size, shadows=True, nthreads=8),
                                  bvh=s.bvh() + ((s.bvh4(),) if r.bvh4 else ()))
        for key in ("node_visits", "tri_tests", "layer_tests", "shaded", "texel_bytes",
                    "shadow_rays", "occluded"):
            assert st[key] == k[key], key
        fb = r.framebuffer()
        r.configure(size, size, shadows=True)
        r.render()
        assert np.array_equal(fb, r.framebuffer())   # both variants render the same image


def test_rt_fp32_bvh4_layout_equals_oracle(po, monkeypatch):
    """RT_BVH_F16=0: unrounded BVH4 boxes in the 128-B fp32 node layout
    (the kernel's other node4_step form) -- frame == brute-force oracle,
    counters == the oracle's traversal of that tree, and the frame equals the
    default binary16-node render."""
    monkeypatch.setenv("RT_BVH_F16", "0")
    s = rt.Scene.load(scene_path("tekkaman"))
    assert s.info()["bvh4_f16"] == 0
    r = rt.Renderer(s)
    try:
        for size in (256, 1024):
            r.configure(size, size, shadows=True, instrumented=True)
            assert r.bvh4 and not r.bvh4_f16
            r.render()
            st = r.stats()
            fb = r.framebuffer()
            c, _, _, k = po.rt_render(oracle_scene(po, "tekkaman"),
                                      po.rt_params(size, size, shadows=True, nthreads=8),
                                      bvh=s.bvh() + (s.bvh4(),))
            assert np.array_equal(fb, c)
            for key in ("node_visits", "tri_tests", "layer_tests", "shadow_rays", "occluded"):
                assert st[key] == k[key], key
            _, rd = renderer("tekkaman")
            rd.configure(size, size, shadows=True)
            assert rd.bvh4_f16
            rd.render()
            assert np.array_equal(fb, rd.framebuffer())
    finally:
        r.close()
        s.close()


@pytest.mark.parametrize("n", (8, 16, 32, 64, 128))
def test_rt_triangle_matches_draw3d_golden(n):
    _, r = renderer("triangle")
    r.configure(n, n, shadows=False)
    r.render()
    img = _png(f"{GOLDEN}/draw3d/triangle_ref_{n}.png")
    from oracle.py_oracle import argb_to_rgba_image, compare_images
    assert compare_images(argb_to_rgba_image(r.framebuffer()), img, tol=1) == 0


def test_rt_tekkaman_1024_vs_reference_render(po):
    """Primary rays at 1024^2 are raster-exact: the RT kernel's frame equals
    the reference's tekkaman_1024x1024.png with 0 differing pixels (tol 0)
    and the golden-pinned oracle raster frame bit for bit."""
    _, r = renderer("tekkaman")
    r.configure(1024, 1024, shadows=False)
    r.render()
    fb = r.framebuffer()
    from oracle.py_oracle import argb_to_rgba_image, compare_images
    ref = _png(f"{GOLDEN}/draw3d/tekkaman_1024x1024.png")
    assert compare_images(argb_to_rgba_image(fb), ref, tol=0) == 0
    rc, _, _ = po.raster_render(oracle_scene(po, "tekkaman"), 1024, 1024)
    assert np.array_equal(fb, rc)


@pytest.mark.parametrize("name", ("tekkaman", "box", "scene", "carnival"))
def test_rt_primary_matches_draw3d_golden_128(name):
    """RT kernel primary rays (no shadows) vs the reference's *_ref_128.png:
    0 differing pixels."""
    _, r = renderer(name)
    r.configure(128, 128, shadows=False)
    r.render()
    from oracle.py_oracle import argb_to_rgba_image, compare_images
    ref = _png(f"{GOLDEN}/draw3d/{name}_ref_128.png")
    assert compare_images(argb_to_rgba_image(r.framebuffer()), ref, tol=0) == 0


@pytest.mark.parametrize("name", ("tekkaman", "box", "scene", "carnival"))
def test_pt_primary_pass_equals_oracle_128(po, name):
    """The path tracer's primary pass at 0 bounces (pt_kernel: every path is
    one shadow-ray vertex) == the oracle's path_trace(bounces=0) bit for bit,
    counters included; and every pixel that starts no path (no geometry
    hit) keeps the reference's raster colour (the *_ref_128.png golden)."""
    s, r = renderer(name)
    r.configure(128, 128, shadows=False, path=True, bounces=0, instrumented=True)
    r.render()
    st = r.stats()
    fb = r.framebuffer()
    c, _, tout, k = po.rt_render(oracle_scene(po, name),
                                po.rt_params(128, 128, shadows=False, path=True, bounces=0, nthreads=4),
                                bvh=s.bvh() + (s.bvh4(),))
    assert np.array_equal(fb, c)
    for key in ("primary_rays", "geometry_hits", "shadow_rays", "occluded", "bounce_rays", "node_visits",
                "tri_tests", "layer_tests"):
        assert st[key] == k[key], key
    from oracle.py_oracle import argb_to_rgba_image, compare_images
    ref = _png(f"{GOLDEN}/draw3d/{name}_ref_128.png")
    # the oracle's t is 0 exactly where the primary ray has no geometry
    # winner (rt.c rt_row); rows flipped like argb_to_rgba_image's
    nogeo = (tout.reshape(128, 128) == 0.0)[::-1]
    assert nogeo.sum() < 128 * 128 and (nogeo.any() or name == "carnival")  # carnival: all geometry
    got = argb_to_rgba_image(fb)
    assert compare_images(got[nogeo], ref[nogeo], tol=0) == 0


@pytest.mark.parametrize("shards", (2, 3, 8))
def test_tile_sharding_reassembles_full_frame(shards):
    _, r = renderer("tekkaman")
    W = H = 512
    r.configure(W, H, shadows=True)
    r.render()
    full = r.framebuffer()
    parts, rays = [], 0
    for i in range(shards):
        r.configure(W, H, shadows=True, shard_index=i, shard_count=shards)
        r.render()
        parts.append(r.framebuffer().copy())
        rays += r.stats()["primary_rays"]
    assert rays == W * H
    assert np.array_equal(rt.deinterleave_tiles(parts, W, H), full)


def test_render_is_deterministic_and_repeatable():
    _, r = renderer("tekkaman")
    r.configure(1024, 1024, shadows=True)
    r.render()
    a = r.framebuffer()
    for _ in range(3):
        r.render()
    assert np.array_equal(a, r.framebuffer())
    assert r.stats()["kernel_ms"] > 0


def test_compact_single_shard_is_the_shard_layout():
    _, r = renderer("tekkaman")
    W = H = 200  # edge tiles overhang the image
    r.configure(W, H, shadows=True)
    r.render()
    full = r.framebuffer()
    r.configure(W, H, shadows=True, compact=True)
    r.render()
    part = r.framebuffer()
    assert part.size == 7 * 7 * 1024
    assert np.array_equal(rt.deinterleave_tiles([part], W, H), full)


@pytest.mark.parametrize("path", (False, True))
def test_queued_frames_equal_synchronous_frames(path):
    # back-to-back vx_start calls queue behind the in-flight frame (driver
    # VX_HIP_QUEUE_DEPTH); every queued frame is a complete, identical render
    _, r = renderer("tekkaman")
    r.configure(512, 512, shadows=True, path=path)
    r.render()
    ref = r.framebuffer()
    ms0, nt0, n0 = r.run_totals()
    for _ in range(7):
        r.start()
    r.wait()
    ms1, nt1, n1 = r.run_totals()
    assert n1 - n0 == 7 and nt1 > nt0 and ms1 > ms0
    assert np.array_equal(r.framebuffer(), ref)
    assert r.stats()["primary_rays"] == 512 * 512
    # untimed (rt_render_set_timing 0: no events, no queue bound -- bench.py's
    # kernel clock): 40 back-to-back frames, none timed, all complete
    r.set_timing(False)
    try:
        for _ in range(40):
            r.start()
        r.wait()
        ms2, nt2, n2 = r.run_totals()
        assert n2 - n1 == 40 and nt2 == nt1 and ms2 == ms1
        assert np.array_equal(r.framebuffer(), ref)
    finally:
        r.set_timing(True)
    r.render()
    assert r.run_totals()[1] == nt2 + 1      # timed again (a start on an idle queue)


def test_rtapp_cli_against_golden():
    exe = os.path.join(_lib.LIB_DIR, "rtapp")
    out = subprocess.run([exe, "-t", scene_path("triangle"), "-w", "64", "-h", "64", "-o",
                          "/tmp/rtapp_tri64.png", "-r", f"{GOLDEN}/draw3d/triangle_ref_64.png"],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "PASSED!" in out.stdout


@pytest.mark.parametrize("flags", [["-B", "sah"], ["-B", "lbvh"], ["-H"], ["-B", "sah", "-H"]])
def test_rtapp_cli_device_build_and_host_setup(flags):
    """rtapp -B sah|lbvh (device BVH build) and -H (host-loop setup) render
    draw3d's tekkaman golden exactly (primary rays are raster-exact)."""
    exe = os.path.join(_lib.LIB_DIR, "rtapp")
    out = subprocess.run([exe, "-t", scene_path("tekkaman"), "-w", "128", "-h", "128", "-o",
                          "/tmp/rtapp_tek128.png", "-r", f"{GOLDEN}/draw3d/tekkaman_ref_128.png"] + flags,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "PASSED!" in out.stdout
    assert ("Setup (host)" if "-H" in flags else "Setup (device)") in out.stdout
    if "-B" in flags:
        assert f"Device BVH ({flags[1]})" in out.stdout


def test_counters_off_writes_no_counter_rows():
    """The timed product configuration (counters=False) writes no per-block
    counter rows: the user counters read 0 and MINSTRET is the launch's
    declared task count; with counters on they are the real counts."""
    _, r = renderer("tekkaman")
    r.configure(256, 256, shadows=True, counters=True)
    r.render()
    on = r.stats()
    fb_on = r.framebuffer()
    r.configure(256, 256, shadows=True, counters=False)
    r.render()
    off = r.stats()
    assert on["primary_rays"] == 256 * 256 and on["shadow_rays"] > 0
    assert off["primary_rays"] == 0 and off["shadow_rays"] == 0
    assert off["tasks"] == off["num_tasks"] == on["tasks"]
    assert np.array_equal(r.framebuffer(), fb_on)
