"""CPU-side tests of the native product (no GPU calls): the C-ABI libraries
load and export every declared symbol, the C++ scene reader agrees with the
oracle's independent reader, host-side fixed-point setup matches the oracle,
the BVH is well formed and its traversal (restated by the oracle) returns the
brute-force closest hits bit for bit."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT, scene_path

os.environ.setdefault("SKYBOX_RT_NO_TORCH", "1")

from skybox_rt_amd import _lib, rt, vortex  # noqa: E402

SCENES = ["triangle", "tekkaman", "box", "carnival", "scene", "vase", "mouse"]


def _declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(\w+)\s*\(", txt, flags=re.M)
    return sorted({n for n in names if n.startswith(("vx_", "rt_")) and not n.endswith("_t")})


@pytest.fixture(scope="session", autouse=True)
def native_built():
    if _lib.missing():
        _lib.build()
    assert not _lib.missing()


@pytest.mark.parametrize("header,lib", [("vortex.h", "libvortex.so"), ("vx_rt.h", "librtapp.so"),
                                        ("vx_tex.h", "librtapp.so"),
                                        ("rt_shard.h", "librt_shard.so")])
def test_c_abi_exports_every_declared_symbol(header, lib):
    h = C.CDLL(os.path.join(_lib.LIB_DIR, lib))
    names = _declared(header)
    assert len(names) >= {"vortex.h": 22, "vx_rt.h": 15, "vx_tex.h": 7, "rt_shard.h": 1}[header]
    for n in names:
        assert hasattr(h, n), f"{lib} does not export {n} declared in include/{header}"


def test_driver_exports_vx_dev_init_and_extensions():
    h = C.CDLL(os.path.join(_lib.LIB_DIR, "libvortex-hip.so"))
    for n in ("vx_dev_init", "vx_hip_mem_ptr", "vx_hip_stream", "vx_hip_last_run", "vx_hip_device_id",
              "vx_hip_run_totals", "vx_hip_mpm_rows", "vx_hip_set_counters", "vx_hip_set_timing",
              "vx_hip_launch_group", "vx_hip_copy_to_dev_async", "vx_hip_set_launch_tag",
              "vx_hip_set_launch_words", "vx_hip_timing_source"):
        assert hasattr(h, n)


def test_driver_fills_all_16_callbacks():
    h = C.CDLL(os.path.join(_lib.LIB_DIR, "libvortex-hip.so"))
    cb = (C.c_void_p * 16)()
    assert h.vx_dev_init(None) == -1
    assert h.vx_dev_init(C.byref(cb)) == 0
    assert all(cb[i] for i in range(16))


def test_vortex_api_rejects_calls_without_device():
    lib = vortex.lib()
    assert lib.vx_mem_free(None) == 0           # callbacks.inc:100-102: null buffer is a no-op
    assert lib.vx_dev_open(None) != 0


def test_kernel_images_have_vxbin_header():
    for name, vma in (("rt_kernel.vxbin", 0x80000000), ("rt_kernel_stats.vxbin", 0x90000000)):
        data = open(os.path.join(_lib.LIB_DIR, name), "rb").read()
        lo, hi = np.frombuffer(data[:16], np.uint64)
        assert lo == vma and hi - lo >= len(data) - 16 and (hi - lo) % 4096 == 0
        assert data[16:20] == b"\x7fELF"             # gfx950 code object


@pytest.mark.parametrize("name", SCENES)
def test_scene_reader_matches_oracle_reader(oracle_lib, name):
    s = rt.Scene.load(scene_path(name))
    ref = oracle_lib.cgltrace.load(scene_path(name))
    assert np.array_equal(s.prims().view(np.uint32), ref.prim_verts.view(np.uint32))
    info = s.info()
    assert info["num_drawcalls"] == len(ref.drawcalls)
    assert info["num_textures"] == len(ref.textures)


@pytest.mark.parametrize("name,size", [("tekkaman", 128), ("tekkaman", 1024), ("vase", 256),
                                       ("triangle", 64), ("mouse", 4096)])
def test_fixed_point_setup_matches_oracle(oracle_lib, name, size):
    s = rt.Scene.load(scene_path(name))
    ref = oracle_lib.cgltrace.load(scene_path(name))
    got = s.setup_prims(size, size)
    lib = oracle_lib.lib()
    for dci, dc in enumerate(ref.drawcalls):
        for g in range(dc.prim_offset, dc.prim_offset + dc.prim_count):
            out = np.zeros(30, np.int32)
            bb = np.zeros(4, np.int32)
            v = np.ascontiguousarray(ref.prim_verts[g])
            lib.orc_setup_prim(v.ctypes.data, size, size, C.c_float(dc.viewport["near"]),
                               C.c_float(dc.viewport["far"]), out.ctypes.data, bb.ctypes.data)
            assert np.array_equal(out, got[g, :30]), g
            assert got[g, 30] == dci


def _check_bvh(nodes, tris, npids):
    seen = []

    def walk(ref, lo, hi, depth):
        if ref >= 0:
            n = nodes[ref]
            for ch in range(2):
                c = int(n[12:14].view(np.int32)[ch])
                if c == -1:
                    continue
                clo = n[[0 + 2 * ch, 4 + 2 * ch, 8 + 2 * ch]]
                chi = n[[1 + 2 * ch, 5 + 2 * ch, 9 + 2 * ch]]
                assert np.all(clo <= chi)
                walk(c, clo, chi, depth + 1)
        else:
            u = ref & 0xFFFFFFFF
            first, count = (u >> 4) & 0x7FFFFFF, (u & 15) + 1
            for k in range(first, first + count):
                t = tris[k]
                v0, e1, e2 = t[0:3], t[4:7], t[8:11]
                for p in (v0, v0 + e1, v0 + e2):   # vertices inside the padded box
                    assert np.all(p >= lo - 1e-3) and np.all(p <= hi + 1e-3)
                seen.append(int(t[3:4].view(np.int32)[0]))
    walk(0, None, None, 0)
    assert sorted(seen) == sorted(npids)


@pytest.mark.parametrize("name", ["tekkaman", "scene", "box", "vase"])
def test_bvh_structure(name):
    s = rt.Scene.load(scene_path(name))
    info = s.info()
    nodes, tris = s.bvh()
    assert info["bvh_depth"] <= 24
    assert info["bvh_tris"] == info["num_geometry"]
    geom = [g for g in range(info["num_prims"])]
    ref_pids = sorted(int(x) for x in tris[:, 3].view(np.int32))
    assert len(set(ref_pids)) == len(ref_pids)
    _check_bvh(nodes, tris, ref_pids)
    assert set(ref_pids) <= set(geom)


@pytest.mark.parametrize("name,size,shadows", [("tekkaman", 256, True), ("tekkaman", 1024, True),
                                               ("scene", 256, False), ("box", 128, True)])
def test_bvh_traversal_equals_bruteforce(oracle_lib, name, size, shadows):
    po = oracle_lib
    s = rt.Scene.load(scene_path(name))
    osc = po.OracleScene(po.cgltrace.load(scene_path(name)))
    p = po.rt_params(size, size, shadows=shadows, nthreads=8)
    cb, pb, tb, kb = po.rt_render(osc, p)
    cv, pv, tv, kv = po.rt_render(osc, p, bvh=s.bvh())
    assert np.array_equal(cb, cv) and np.array_equal(pb, pv)
    assert np.array_equal(tb.view(np.uint32), tv.view(np.uint32))
    assert kb["occluded"] == kv["occluded"] and kb["geometry_hits"] == kv["geometry_hits"]
    assert kv["tri_tests"] < kb["tri_tests"]


def _check_bvh4(nodes4, nodes, tris, stack_bound):
    """The 4-wide BVH holds exactly the BVH2's leaves, under the same padded
    boxes, and the host's stack bound covers every root-to-leaf walk."""
    leaves4, leaves2 = [], []

    def walk2(ref):
        if ref >= 0:
            for ch in range(2):
                c = int(nodes[ref][12:14].view(np.int32)[ch])
                if c != -1:
                    walk2(c)
        else:
            leaves2.append(ref)

    def walk4(ref, lo, hi):
        n = nodes4[ref]
        refs = n[24:28].view(np.int32)
        used = [i for i in range(4) if refs[i] != -1]
        assert used == list(range(len(used))) and (len(used) >= 2 or ref == 0)
        need = 0
        for i in used:
            clo = n[[i, 8 + i, 16 + i]]
            chi = n[[4 + i, 12 + i, 20 + i]]
            assert np.all(clo <= chi)
            if lo is not None:                      # BVH2 nesting: child box inside parent's
                assert np.all(clo >= lo - 1e-3) and np.all(chi <= hi + 1e-3)
            c = int(refs[i])
            if c >= 0:
                need = max(need, walk4(c, clo, chi))
            else:
                leaves4.append(c)
        return len(used) - 1 + need

    walk2(0)
    st = walk4(0, None, None)
    assert sorted(leaves4) == sorted(leaves2)
    assert st == stack_bound


@pytest.mark.parametrize("name", ["tekkaman", "scene", "box", "carnival"])
def test_bvh4_collapse_structure(name):
    s = rt.Scene.load(scene_path(name))
    info = s.info()
    nodes, tris = s.bvh()
    nodes4 = s.bvh4()
    assert info["bvh4_nodes"] == len(nodes4) and 0 < len(nodes4) <= len(nodes)
    assert info["bvh4_depth"] <= info["bvh_depth"]
    if len(nodes) > 100:
        # each BVH4 node absorbs up to 3 BVH2 nodes (about half of them in practice)
        assert len(nodes4) <= 0.6 * len(nodes) and info["bvh4_depth"] < info["bvh_depth"]
    _check_bvh4(nodes4, nodes, tris, info["bvh4_stack"])
    assert info["bvh4_stack"] <= 32


@pytest.mark.parametrize("name", ["tekkaman", "scene", "box", "carnival"])
def test_bvh4_binary16_boxes_are_outward(name, monkeypatch):
    """rt_node4h_t (the kernel's 64-B node): every BVH4 box plane is a
    binary16 value (so the kernel's exact f16->f32 conversion reproduces the
    exported fp32 planes the oracle traverses), each rounded box contains the
    unrounded one (RT_BVH_F16=0), and the tree is otherwise the same."""
    s = rt.Scene.load(scene_path(name))
    assert s.info()["bvh4_f16"] == 1
    n16 = s.bvh4()
    monkeypatch.setenv("RT_BVH_F16", "0")
    s32 = rt.Scene.load(scene_path(name))
    assert s32.info()["bvh4_f16"] == 0
    n32 = s32.bvh4()
    assert n16.shape == n32.shape
    planes = n16[:, :24]
    assert np.array_equal(planes.astype(np.float16).astype(np.float32), planes)
    assert np.array_equal(n16[:, 24:].view(np.int32), n32[:, 24:].view(np.int32))
    for k in range(3):
        assert np.all(n16[:, 8 * k:8 * k + 4] <= n32[:, 8 * k:8 * k + 4])
        assert np.all(n16[:, 8 * k + 4:8 * k + 8] >= n32[:, 8 * k + 4:8 * k + 8])
        # outward by at most one binary16 quantum (2^-10 relative, 2^-24 absolute)
        for sl in (slice(8 * k, 8 * k + 4), slice(8 * k + 4, 8 * k + 8)):
            d = np.abs(n16[:, sl].astype(np.float64) - n32[:, sl])
            assert np.all(d <= np.maximum(np.abs(n32[:, sl]) * 2.0 ** -10, 2.0 ** -24))


@pytest.mark.parametrize("name,size,shadows,path", [
    ("tekkaman", 256, True, False), ("tekkaman", 1024, True, False), ("scene", 256, False, False),
    ("box", 128, True, False), ("carnival", 200, True, False), ("tekkaman", 128, False, True)])
def test_bvh4_traversal_equals_bvh2(oracle_lib, name, size, shadows, path):
    """Any traversal order gives the same closest hit (t, then the depth
    test's pid tie rule) and the same any-hit verdict: the BVH4 restatement
    reproduces the BVH2 renders exactly, with fewer node visits."""
    po = oracle_lib
    s = rt.Scene.load(scene_path(name))
    osc = po.OracleScene(po.cgltrace.load(scene_path(name)))
    # the primary walk too (not the block lists): this compares tree traversals
    p = po.rt_params(size, size, shadows=shadows, nthreads=8, path=path, bounces=3, vis_lists=False)
    nodes, tris = s.bvh()
    c2, p2, t2, k2 = po.rt_render(osc, p, bvh=(nodes, tris))
    c4, p4, t4, k4 = po.rt_render(osc, p, bvh=(nodes, tris, s.bvh4()))
    assert np.array_equal(c2, c4) and np.array_equal(p2, p4)
    assert np.array_equal(t2.view(np.uint32), t4.view(np.uint32))
    for key in ("occluded", "geometry_hits", "shadow_rays", "bounce_rays"):
        assert k2[key] == k4[key], key
    assert k4["node_visits"] < k2["node_visits"] or len(nodes) == 1


def test_rtapp_cli_usage():
    out = subprocess.run([os.path.join(_lib.LIB_DIR, "rtapp"), "-?"], capture_output=True, text=True)
    assert out.returncode == 0 and "Usage" in out.stdout


def lbvh_inputs(s):
    """The GPU builder's inputs for a scene: the depth-tested triangles in
    ascending pid order as clip (x, y, w) corners and as rt_tri_t records."""
    _, tris = s.bvh()
    pids = np.sort(tris[:, 3].copy().view(np.int32))
    P = s.prims()[pids]
    verts = np.ascontiguousarray(P[:, :, [0, 1, 3]], np.float32)
    geom = np.zeros((len(pids), 12), np.float32)
    geom[:, 0:3] = verts[:, 0]
    geom[:, 3] = pids.view(np.float32)
    geom[:, 4:7] = verts[:, 1] - verts[:, 0]
    geom[:, 8:11] = verts[:, 2] - verts[:, 0]
    return verts, geom, pids


@pytest.mark.parametrize("name", ["tekkaman", "scene", "box", "carnival"])
def test_lbvh_collapse4_oracle_structure_and_traversal(oracle_lib, name):
    """The device BVH4 collapse restated (oracle/lbvh.c orc_lbvh_collapse4):
    every leaf of the LBVH exactly once under nested boxes, >= 2 children per
    node, the reported stack bound equal to the worst root-to-leaf push count,
    and BVH4 traversal over it reproduces the BVH2 frames bit for bit."""
    po = oracle_lib
    s = rt.Scene.load(scene_path(name))
    verts, geom, _ = lbvh_inputs(s)
    nodes, tris, depth = po.lbvh_build(verts, geom)
    nodes4, stack = po.lbvh_collapse4(nodes)
    _check_bvh4(nodes4, nodes, tris, stack)
    assert stack <= 3 * ((depth + 1) // 2)
    osc = po.OracleScene(po.cgltrace.load(scene_path(name)))
    p = po.rt_params(160, 160, shadows=True, nthreads=8)
    c2, p2, t2, k2 = po.rt_render(osc, p, bvh=(nodes, tris))
    c4, p4, t4, k4 = po.rt_render(osc, p, bvh=(nodes, tris, nodes4))
    assert np.array_equal(c2, c4) and np.array_equal(p2, p4)
    assert np.array_equal(t2.view(np.uint32), t4.view(np.uint32))
    assert k4["occluded"] == k2["occluded"] and k4["node_visits"] <= k2["node_visits"]


@pytest.mark.parametrize("name", ["tekkaman", "scene", "box", "carnival"])
def test_lbvh_oracle_structure_and_traversal(oracle_lib, name):
    """The linear-BVH restatement (oracle/lbvh.c) builds a valid tree -- every
    triangle in exactly one leaf, inside its padded boxes, depth within the
    deep traversal stack -- and tracing over it reproduces brute force."""
    po = oracle_lib
    s = rt.Scene.load(scene_path(name))
    verts, geom, pids = lbvh_inputs(s)
    nodes, tris, depth = po.lbvh_build(verts, geom)
    assert 1 <= depth <= 32
    _check_bvh(nodes, tris, sorted(int(p) for p in pids))
    osc = po.OracleScene(po.cgltrace.load(scene_path(name)))
    p = po.rt_params(160, 160, shadows=True, nthreads=8)
    cb, pb, tb, _ = po.rt_render(osc, p)
    cv, pv, tv, kv = po.rt_render(osc, p, bvh=(nodes, tris))
    assert np.array_equal(cb, cv) and np.array_equal(pb, pv)
    assert np.array_equal(tb.view(np.uint32), tv.view(np.uint32))


@pytest.mark.parametrize("name", ["tekkaman", "scene", "carnival"])
def test_oracle_half4_restates_host_rounding(name, oracle_lib):
    """The host tree's fp32 BVH4 planes are already rounded outward to
    binary16 values (bvh.cpp HalfRound), so the oracle's restatement
    (orc_half4, which the device tree's BVHB_HALF phase is checked against)
    must leave them unchanged, and its half records must decode to them."""
    po = oracle_lib
    s = rt.Scene.load(scene_path(name))
    n4 = s.bvh4()
    r4, h = po.half4(n4)
    assert np.array_equal(r4.view(np.uint32), n4.view(np.uint32))
    halves = h[:, :48].copy().view(np.float16).astype(np.float32)
    assert np.array_equal(halves, n4[:, :24])
    assert np.array_equal(h[:, 48:].copy().view(np.int32), n4[:, 24:28].view(np.int32))
