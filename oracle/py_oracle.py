"""ctypes front-end of liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module (see oracle/oracle.h).  It never touches the product.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from . import cgltrace  # noqa: F401  (re-exported for callers)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")

CLEAR_COLOR = 0xFF000000  # draw3d/main.cpp:47
CLEAR_DEPTH = 0xFFFFFFFF  # draw3d/main.cpp:48
RT_SHADOWS = 0x1
RT_PATH = 0x8
PT_SEED = 0x5EED


class DrawcallC(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("prim_offset", "prim_count", "tex_slot")] + [
        ("znear", C.c_float), ("zfar", C.c_float), ("color_enabled", C.c_int32),
        ("color_writemask", C.c_uint32)] + [(n, C.c_int32) for n in (
            "depth_test", "depth_writemask", "depth_func", "stencil_test",
            "stencil_func", "stencil_zpass", "stencil_zfail", "stencil_fail",
            "stencil_ref", "stencil_mask", "stencil_writemask", "texture_enabled",
            "texture_envmode", "texture_minfilter", "texture_magfilter",
            "texture_addressU", "texture_addressV", "blend_enabled", "blend_src",
            "blend_dst")]


class TextureC(C.Structure):
    _fields_ = [("format", C.c_int32), ("width", C.c_int32), ("height", C.c_int32),
                ("pad", C.c_int32), ("offset", C.c_int64)]


class SceneC(C.Structure):
    _fields_ = [("num_drawcalls", C.c_int32), ("drawcalls", C.POINTER(DrawcallC)),
                ("num_prims", C.c_int32), ("prim_verts", C.POINTER(C.c_float)),
                ("num_textures", C.c_int32), ("textures", C.POINTER(TextureC)),
                ("texels", C.POINTER(C.c_uint8))]


class RtParamsC(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("flags", C.c_uint32),
                ("light", C.c_float * 3), ("clear_color", C.c_uint32),
                ("bounces", C.c_uint32), ("seed", C.c_uint32), ("nthreads", C.c_uint32),
                ("row_begin", C.c_uint32), ("row_end", C.c_uint32), ("row_step", C.c_uint32),
                ("vis_per_lane", C.c_uint32), ("vis_lists", C.c_uint32),
                ("shadow_lists", C.c_uint32), ("path_queue", C.c_uint32), ("split_log", C.c_uint32)]


class RtCountersC(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "primary_rays", "shadow_rays", "geometry_hits", "occluded", "node_visits",
        "tri_tests", "layer_tests", "shaded", "texel_bytes", "bounce_rays")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


class BvhC(C.Structure):
    _fields_ = [("num_nodes", C.c_int32), ("nodes", C.POINTER(C.c_float)),
                ("num_tris", C.c_int32), ("tris", C.POINTER(C.c_float)),
                ("num_nodes4", C.c_int32), ("nodes4", C.POINTER(C.c_float)),
                ("num_vis_nodes", C.c_int32), ("vis_refs", C.POINTER(C.c_int32)),
                ("num_vis_leaves", C.c_int32), ("vis_pids", C.POINTER(C.c_int32))]


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _lib.orc_raster_render.argtypes = [C.POINTER(SceneC), C.c_uint32, C.c_uint32, C.c_uint32,
                                           C.c_void_p, C.c_void_p, C.c_void_p]
        for fn in (_lib.orc_rt_render_bruteforce,):
            fn.argtypes = [C.POINTER(SceneC), C.POINTER(RtParamsC), C.c_void_p, C.c_void_p,
                           C.c_void_p, C.POINTER(RtCountersC)]
        _lib.orc_rt_render_bvh.argtypes = [C.POINTER(SceneC), C.POINTER(BvhC), C.POINTER(RtParamsC),
                                           C.c_void_p, C.c_void_p, C.c_void_p,
                                           C.POINTER(RtCountersC)]
        _lib.orc_setup_prim.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_float, C.c_float,
                                        C.c_void_p, C.c_void_p]
        _lib.orc_mt.argtypes = [C.c_void_p] * 5 + [C.c_float, C.POINTER(C.c_float)]
        _lib.orc_vis_prims.argtypes = [C.POINTER(SceneC), C.c_uint32, C.c_uint32, C.c_void_p]
        _lib.orc_vis_block_lists.argtypes = [C.POINTER(SceneC)] + [C.c_uint32] * 4 + [
            C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)]
        _lib.orc_lbvh_build.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                        C.POINTER(C.c_uint32)]
        _lib.orc_lbvh_collapse4.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p,
                                            C.POINTER(C.c_uint32)]
        _lib.orc_half4.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
        _lib.orc_tex_encode.argtypes = [C.c_uint32, C.c_uint32]
        _lib.orc_tex_encode.restype = C.c_uint32
        _lib.orc_tex_build.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p,
                                       C.c_void_p, C.c_void_p]
        _lib.orc_tex_build.restype = C.c_size_t
        _lib.orc_tex_lod.argtypes = [C.c_uint32] * 4 + [C.POINTER(C.c_uint32)] * 2
        _lib.orc_tex_render.argtypes = [C.c_void_p, C.c_void_p] + [C.c_uint32] * 8 + [C.c_void_p]
    return _lib


def _ptr(a, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


class OracleScene:
    """Keeps the numpy buffers alive for the C structs."""

    def __init__(self, scene):
        self.scene = scene
        tex_ids = sorted(scene.textures)
        slot = {tid: i for i, tid in enumerate(tex_ids)}
        blobs, texs, off = [], [], 0
        for tid in tex_ids:
            fmt, w, h, data = scene.textures[tid]
            texs.append(TextureC(fmt, w, h, 0, off))
            blobs.append(np.frombuffer(data, np.uint8))
            off += len(data)
        self.texels = np.concatenate(blobs) if blobs else np.zeros(1, np.uint8)
        self.tex_arr = (TextureC * max(1, len(texs)))(*texs)
        dcs = []
        for dc in scene.drawcalls:
            s = dc.states
            dcs.append(DrawcallC(
                prim_offset=dc.prim_offset, prim_count=dc.prim_count,
                tex_slot=slot.get(dc.texture_id, -1) if s["texture_enabled"] else -1,
                znear=dc.viewport["near"], zfar=dc.viewport["far"],
                color_enabled=s["color_enabled"], color_writemask=s["color_writemask"] & 0xFFFFFFFF,
                **{k: s[k] for k in (
                    "depth_test", "depth_writemask", "depth_func", "stencil_test",
                    "stencil_func", "stencil_zpass", "stencil_zfail", "stencil_fail",
                    "stencil_ref", "stencil_mask", "stencil_writemask", "texture_enabled",
                    "texture_envmode", "texture_minfilter", "texture_magfilter",
                    "texture_addressU", "texture_addressV", "blend_enabled", "blend_src",
                    "blend_dst")}))
        self.dc_arr = (DrawcallC * max(1, len(dcs)))(*dcs)
        self.verts = np.ascontiguousarray(scene.prim_verts, dtype=np.float32).reshape(-1)
        if self.verts.size == 0:
            self.verts = np.zeros(30, np.float32)
        self.c = SceneC(len(dcs), self.dc_arr, scene.num_prims, _ptr(self.verts, C.c_float),
                        len(texs), self.tex_arr, _ptr(self.texels, C.c_uint8))


def raster_render(oscene: OracleScene, width: int, height: int, tile_logsize: int = 5):
    color = np.full(width * height, CLEAR_COLOR, np.uint32)
    depth = np.full(width * height, CLEAR_DEPTH, np.uint32)
    pid = np.empty(width * height, np.int32)
    rc = lib().orc_raster_render(C.byref(oscene.c), width, height, tile_logsize,
                                 color.ctypes.data, depth.ctypes.data, pid.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"orc_raster_render failed: {rc}")
    return (color.reshape(height, width), depth.reshape(height, width),
            pid.reshape(height, width))


def raster_coverage(oscene: OracleScene, width: int, height: int, tile_logsize: int = 5):
    """The raster regression app's image (ARGB, row 0 = bottom): covered
    pixels 0xffffffff over the 0xff000000 clear."""
    L = lib()
    L.orc_raster_coverage.argtypes = [C.POINTER(SceneC), C.c_uint32, C.c_uint32, C.c_uint32,
                                      C.c_void_p]
    color = np.full(width * height, CLEAR_COLOR, np.uint32)
    if L.orc_raster_coverage(C.byref(oscene.c), width, height, tile_logsize, color.ctypes.data):
        raise RuntimeError("orc_raster_coverage failed")
    return color.reshape(height, width)


def edge_cover(edges, x0: int, y0: int, w: int, h: int) -> np.ndarray:
    """orc_edge_cover: the rasterizer's coverage of one primitive, (a, b, c)
    per edge, over the w x h window at (x0, y0) -> uint8 [h, w]."""
    L = lib()
    L.orc_edge_cover.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p]
    L.orc_edge_cover.restype = None
    e = np.ascontiguousarray(np.asarray(edges, np.int64).reshape(9).astype(np.int32))
    m = np.zeros(w * h, np.uint8)
    L.orc_edge_cover(e.ctypes.data, x0, y0, w, h, m.ctypes.data)
    return m.reshape(h, w)


def vis_prims(oscene: OracleScene, width: int, height: int) -> np.ndarray:
    """uint32[P, 3]: every primitive's covered-pixel rectangle (x0|x1<<16,
    y0|y1<<16, inclusive) and depth-word lower bound, by brute force (vis.c)."""
    n = oscene.scene.num_prims
    out = np.zeros((max(n, 1), 3), np.uint32)
    rc = lib().orc_vis_prims(C.byref(oscene.c), width, height, out.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"orc_vis_prims failed: {rc}")
    return out[:n]


def vis_block_lists(oscene: OracleScene, width: int, height: int, shard_index: int = 0,
                    shard_count: int = 1):
    """The per-8x8-block candidate lists of one shard (oracle/rt.c
    orc_vis_block_lists, the product's rt_bentry_t layout) -> (idx
    uint32[nlb, 2]: first entry, count; ent uint32[total, 4]: geometry index,
    union corners lo, hi, depth bound)."""
    tot, nlb = C.c_uint64(), C.c_uint32()
    rc = lib().orc_vis_block_lists(C.byref(oscene.c), width, height, shard_index, shard_count, None,
                                   None, C.byref(tot), C.byref(nlb))
    if rc != 0:
        raise RuntimeError(f"orc_vis_block_lists failed: {rc}")
    idx = np.zeros((max(nlb.value, 1), 2), np.uint32)
    ent = np.zeros((max(tot.value, 1), 4), np.uint32)
    lib().orc_vis_block_lists(C.byref(oscene.c), width, height, shard_index, shard_count,
                              idx.ctypes.data, ent.ctypes.data, C.byref(tot), C.byref(nlb))
    return idx[:nlb.value], ent[:tot.value]


SL_N = 128  # rt.c SL_N, the kernels' RT_SLIST_N


def shadow_lists(oscene: OracleScene, light=(0.0, 60.0, 80.0)):
    """The light-space shadow lists (oracle/rt.c orc_shadow_lists) -> (idx
    uint32[6*128*128, 2]: first entry, count; ent int32[total]: geometry
    indices, ascending within a cell)."""
    L = (C.c_float * 3)(*[float(np.float32(x)) for x in light])
    tot = C.c_uint64()
    lib().orc_shadow_lists.argtypes = [C.POINTER(SceneC), C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.POINTER(C.c_uint64)]
    rc = lib().orc_shadow_lists(C.byref(oscene.c), L, None, None, C.byref(tot))
    if rc != 0:
        raise RuntimeError(f"orc_shadow_lists failed: {rc}")
    idx = np.zeros((6 * SL_N * SL_N, 2), np.uint32)
    ent = np.zeros(max(tot.value, 1), np.int32)
    lib().orc_shadow_lists(C.byref(oscene.c), L, idx.ctypes.data, ent.ctypes.data, C.byref(tot))
    return idx, ent[:tot.value]


def rt_params(width, height, shadows=True, light=(0.0, 60.0, 80.0), nthreads=1,
              clear_color=CLEAR_COLOR, row_begin=0, row_end=0, row_step=0,
              path=False, bounces=4, seed=PT_SEED, vis_per_lane=False, vis_lists=None,
              shadow_lists=None, path_queue=None, split_log=0):
    p = RtParamsC()
    p.vis_per_lane = 1 if vis_per_lane else 0
    # the product resolves primary visibility from per-block candidate lists
    # (its default, primary+shadow and path frames)
    p.vis_lists = (0 if vis_per_lane else 1) if vis_lists is None else int(bool(vis_lists))
    # the product's shadow rays (primary+shadow frames and every path vertex)
    # test the light-space lists (its default with the device setup)
    p.shadow_lists = int(bool(shadows or path) if shadow_lists is None else bool(shadow_lists))
    # path_queue: the product's two-kernel path tracer (RT_PT_QUEUE=1; the
    # primary pass counts per 8x8 block everywhere); default the one-kernel
    # pt_kernel (32-pixel waves in geometry tiles)
    p.path_queue = int(bool(path_queue))
    # path trace: pixels per wave in the geometry tiles, 2^split_log (0: 32)
    p.split_log = int(split_log)
    p.width, p.height = width, height
    p.flags = (RT_SHADOWS if shadows else 0) | (RT_PATH if path else 0)
    p.bounces, p.seed = bounces, seed
    p.light[:] = [float(np.float32(x)) for x in light]
    p.clear_color = clear_color
    p.nthreads = nthreads
    p.row_begin, p.row_end, p.row_step = row_begin, row_end, row_step
    return p


def rt_render(oscene: OracleScene, params: RtParamsC, bvh=None, vis_tree=None):
    """bvh: None (brute force), (nodes float32[N,16], tris float32[M,12]) or
    (nodes, tris, nodes4 float32[N4,32]) -- the last traverses the 4-wide BVH.
    vis_tree: the primary rays' tree (refs int32[N,4], leaf pids int32[M]) as
    the product exports it (Renderer.export_vis_tree); None = walk the BVH
    (the frame is the same either way, the traversal counters are not)."""
    n = params.width * params.height
    color = np.zeros(n, np.uint32)
    pid = np.full(n, -1, np.int32)
    t = np.zeros(n, np.float32)
    cnt = RtCountersC()
    if bvh is None:
        rc = lib().orc_rt_render_bruteforce(C.byref(oscene.c), C.byref(params), color.ctypes.data,
                                            pid.ctypes.data, t.ctypes.data, C.byref(cnt))
    else:
        nodes = np.ascontiguousarray(bvh[0], np.float32)
        tris = np.ascontiguousarray(bvh[1], np.float32)
        b = BvhC(nodes.shape[0], _ptr(nodes, C.c_float), tris.shape[0], _ptr(tris, C.c_float), 0,
                 None)
        if len(bvh) > 2 and bvh[2] is not None:
            nodes4 = np.ascontiguousarray(bvh[2], np.float32)
            b.num_nodes4, b.nodes4 = nodes4.shape[0], _ptr(nodes4, C.c_float)
        if vis_tree is not None and len(vis_tree[0]):
            vrefs = np.ascontiguousarray(vis_tree[0], np.int32)
            vpids = np.ascontiguousarray(vis_tree[1], np.int32)
            b.num_vis_nodes, b.vis_refs = vrefs.shape[0], _ptr(vrefs, C.c_int32)
            b.num_vis_leaves, b.vis_pids = vpids.shape[0], _ptr(vpids, C.c_int32)
        rc = lib().orc_rt_render_bvh(C.byref(oscene.c), C.byref(b), C.byref(params),
                                     color.ctypes.data, pid.ctypes.data, t.ctypes.data,
                                     C.byref(cnt))
    if rc != 0:
        raise RuntimeError(f"oracle rt render failed: {rc}")
    h, w = params.height, params.width
    return color.reshape(h, w), pid.reshape(h, w), t.reshape(h, w), cnt.as_dict()


def argb_to_rgba_image(fb: np.ndarray) -> np.ndarray:
    """ARGB8888 framebuffer (row 0 = bottom) -> RGBA uint8 image, top-down
    (the reference saves with a negative pitch, draw3d/main.cpp:385-386)."""
    fb = np.asarray(fb, np.uint32)[::-1]
    out = np.empty(fb.shape + (4,), np.uint8)
    out[..., 0] = (fb >> 16) & 0xFF
    out[..., 1] = (fb >> 8) & 0xFF
    out[..., 2] = fb & 0xFF
    out[..., 3] = (fb >> 24) & 0xFF
    return out


def compare_images(a: np.ndarray, b: np.ndarray, tol: int = 0) -> int:
    """Pixels whose max per-channel |difference| exceeds `tol` (the reference
    calls cocogfx CompareImages(out, ref, A8R8G8B8, tol): draw3d/main.cpp:507;
    cocogfx is not vendored, this is the documented interpretation)."""
    d = np.abs(a.astype(np.int32) - b.astype(np.int32)).max(axis=-1)
    return int((d > tol).sum())


# ---- texture regression app (tests/regression/tex; oracle/tex.c) ---------
TEX_FORMATS = ("A8R8G8B8", "R5G6B5", "A1R5G5B5", "A4R4G4B4", "A8L8", "L8", "A8")


def load_png_argb(path) -> np.ndarray:
    """PNG -> ARGB8888 uint32[h, w], row 0 = top (cocogfx LoadImage with
    FORMAT_A8R8G8B8; RGB images get alpha 0xff)."""
    from PIL import Image
    a = np.array(Image.open(path).convert("RGBA"), np.uint32)
    return (a[..., 3] << 24) | (a[..., 0] << 16) | (a[..., 1] << 8) | a[..., 2]


def argb_to_rgba_topdown(fb: np.ndarray) -> np.ndarray:
    """ARGB8888 image already top-down (tex/main.cpp saves with +pitch) -> RGBA."""
    fb = np.asarray(fb, np.uint32)
    return np.stack([(fb >> 16) & 0xFF, (fb >> 8) & 0xFF, fb & 0xFF, fb >> 24], -1).astype(np.uint8)


def tex_build(argb: np.ndarray, fmt: int):
    """-> (texels uint8[], mipoff uint32[16], levels)"""
    argb = np.ascontiguousarray(argb, np.uint32)
    h, w = argb.shape
    mip = np.zeros(16, np.uint32)
    lv = C.c_uint32()
    n = lib().orc_tex_build(argb.ctypes.data, w, h, fmt, None, mip.ctypes.data, C.byref(lv))
    out = np.zeros(max(n, 1), np.uint8)
    lib().orc_tex_build(argb.ctypes.data, w, h, fmt, out.ctypes.data, mip.ctypes.data, C.byref(lv))
    return out[:n], mip, lv.value


def tex_lod(logw, logh, dst_w, dst_h):
    lod, frac = C.c_uint32(), C.c_uint32()
    lib().orc_tex_lod(logw, logh, dst_w, dst_h, C.byref(lod), C.byref(frac))
    return lod.value, frac.value


def tex_render(argb: np.ndarray, fmt: int = 0, wrap: int = 0, filt: int = 0, scale: float = 1.0,
               num_tasks: int = 0) -> np.ndarray:
    """The whole tex app on the CPU: dst = (uint32)(src * scale) per side,
    ARGB8888 rows top-down.  num_tasks 0 = one task per row (the reference's
    min(cores x warps x threads, dst_height) on any device with at least
    dst_height hardware threads)."""
    h, w = argb.shape
    texels, mip, _ = tex_build(argb, fmt)
    dw, dh = int(np.float32(w) * np.float32(scale)), int(np.float32(h) * np.float32(scale))
    dst = np.zeros((dh, dw), np.uint32)
    nt = num_tasks or dh
    lib().orc_tex_render(texels.ctypes.data, mip.ctypes.data, int(w).bit_length() - 1,
                         int(h).bit_length() - 1, fmt, wrap, filt, dw, dh, min(nt, dh),
                         dst.ctypes.data)
    return dst


# ---- linear BVH (oracle/lbvh.c) -------------------------------------------
def lbvh_build(verts: np.ndarray, geom: np.ndarray):
    """verts float32[n, 3, 3] clip (x, y, w) corners, geom float32[n, 12] their
    rt_tri_t records -> (nodes float32[max(n-1,1), 16], tris float32[n, 12], depth)."""
    verts = np.ascontiguousarray(verts, np.float32)
    geom = np.ascontiguousarray(geom, np.float32)
    n = verts.shape[0]
    nodes = np.zeros((max(n - 1, 1), 16), np.float32)
    tris = np.zeros((n + 3, 12), np.float32)
    depth = C.c_uint32()
    rc = lib().orc_lbvh_build(verts.ctypes.data, geom.ctypes.data, n, nodes.ctypes.data,
                              tris.ctypes.data, C.byref(depth))
    if rc != 0:
        raise RuntimeError(f"orc_lbvh_build failed: {rc}")
    return nodes, tris[:n], depth.value


def lbvh_collapse4(nodes: np.ndarray):
    """BVH4 collapse of an LBVH node array (oracle/lbvh.c) -> (nodes4
    float32[nn, 32], worst-case traversal stack)."""
    nodes = np.ascontiguousarray(nodes, np.float32)
    nn = nodes.shape[0]
    nodes4 = np.zeros((nn, 32), np.float32)
    stack = C.c_uint32()
    rc = lib().orc_lbvh_collapse4(nodes.ctypes.data, nn, nodes4.ctypes.data, C.byref(stack))
    if rc != 0:
        raise RuntimeError(f"orc_lbvh_collapse4 failed: {rc}")
    return nodes4, stack.value


def half4(nodes4: np.ndarray):
    """binary16 planes of a BVH4 node array (oracle/lbvh.c orc_half4) ->
    (the fp32 nodes with every plane rounded outward, uint8[nn, 64]
    rt_node4h_t records)."""
    n4 = np.ascontiguousarray(nodes4, np.float32).copy()
    nn = n4.shape[0]
    half = np.zeros((nn, 64), np.uint8)
    lib().orc_half4(n4.ctypes.data, nn, half.ctypes.data)
    return n4, half


def om_app(width=128, height=128, num_tasks=256 * 32 * 64, color=0xFFFFFFFF, depth_enable=False,
           blend=False, backface=False):
    """The OM regression app (tests/regression/om/main.cpp:130-300 host side,
    restated: the checkerboard depth clear of :265-275 with TFixed<24>(0.0 /
    0.99), colour clear 0, the OM DCR words of :153-190) run through the
    oracle's unit (gfx.c orc_om_app).  Returns the ARGB8888 colour buffer
    [height, width], row 0 = bottom like the device buffer.  num_tasks
    defaults to the MI355X driver's cores x warps x threads (256 x 32 x 64)."""
    L = lib()
    L.orc_om_app.argtypes = [C.c_uint32] * 5 + [C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                                C.c_void_p]
    fx24 = lambda f: int(np.float32(f) * np.float32(16777216.0))   # truncating TFixed<24>
    y, x = np.mgrid[0:height, 0:width]
    zbuf = np.where((x & 1) == (y & 1), fx24(0.0), fx24(0.99)).astype(np.uint32).reshape(-1)
    cbuf = np.zeros(width * height, np.uint32)
    dcr = np.zeros(18, np.uint32)          # VX_DCR_OM_STATE_BEGIN + i
    dcr[2] = 0xF                                                  # CBUF_WRITEMASK
    dcr[5] = 2 if depth_enable else 0                             # DEPTH_FUNC LESS / ALWAYS
    dcr[6] = 1 if depth_enable else 0                             # DEPTH_WRITEMASK
    dcr[12] = 0xFF                                                # STENCIL_MASK
    dcr[14] = 0                                                   # BLEND_MODE ADD/ADD
    dcr[15] = ((7 << 24) | (7 << 16) | (1 << 8) | 1) if blend else ((1 << 8) | 1)
    rc = L.orc_om_app(width, height, num_tasks, color & 0xFFFFFFFF, 0x800000, int(backface),
                      int(blend), dcr.ctypes.data, cbuf.ctypes.data, zbuf.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"orc_om_app failed: {rc}")
    return cbuf.reshape(height, width)
