"""ctypes binding of include/vx_rt.h (librtapp.so): the RT regression app.

    scene = Scene.load("tekkaman.cgltrace")
    r = Renderer(scene)
    r.configure(1024, 1024, shadows=True)
    r.render()
    fb = r.framebuffer()          # uint32 ARGB8888 [H, W], row 0 = NDC y=-1
    stats = r.stats()

All work runs through the native library and the HIP driver; there is no
fallback.  Errors raise RtError with the library's message.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _lib

RT_RENDER_SHADOWS = 0x1
RT_RENDER_PATH = 0x8
RT_RENDER_FLAT = 0x10
RT_RENDER_RASTER = 0x20
RT_RENDER_BVH2 = 0x40
PT_SEED = 0x5EED
RT_RENDER_INSTRUMENTED = 0x100
RT_RENDER_COMPACT = 0x200
RT_RENDER_COUNTERS = 0x400
RT_RENDER_HOST_SETUP = 0x800
RT_RENDER_BVH_WALK = 0x2000
# rt_renderer_export_records arrays: name -> (id, dtype, words per record)
RECORDS = {"prims": (0, np.int32, 32), "bbox": (1, np.uint32, 2), "vis": (2, np.uint32, 4),
           "vnodes": (3, np.uint32, 16), "vtris": (4, np.int32, 16), "vlayers": (5, np.int32, 16),
           "vgeom": (6, np.int32, 16), "order": (7, np.uint32, 1), "ptris": (8, np.float32, 12),
           "geom": (9, np.float32, 12), "bidx": (10, np.uint32, 2), "blist": (11, np.uint32, 4),
           "sidx": (12, np.uint32, 2), "slist": (13, np.float32, 12)}
RT_BVH_STACK4_UNUSED = 0xFFFFFFFF
RT_BVH_BUILD_HOST = 2
CLEAR_COLOR = 0xFF000000               # draw3d/main.cpp:47
DEFAULT_LIGHT = (0.0, 60.0, 80.0)      # clip (x, y, w), SURVEY.md 8(d) config 3
TILE = 32                              # RASTER_TILE_LOGSIZE = 5


class SceneInfo(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in (
        "num_drawcalls", "num_prims", "num_geometry", "num_layer", "num_textures",
        "bvh_nodes", "bvh_tris", "bvh_leaves", "bvh_depth", "bvh4_nodes", "bvh4_depth",
        "bvh4_stack", "bvh4_f16")] + [
        ("parse_ms", C.c_double), ("bvh_ms", C.c_double)]


class BvhBuildStats(C.Structure):
    _fields_ = [("nodes", C.c_uint32), ("depth", C.c_uint32), ("launches", C.c_uint32),
                ("stack4", C.c_uint32), ("build_ms", C.c_double), ("kernel_ms", C.c_double),
                ("nodes4", C.c_uint32), ("depth4", C.c_uint32), ("method", C.c_uint32),
                ("pad", C.c_uint32)]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_ if n != "pad"}


class SetupStats(C.Structure):
    _fields_ = [("device", C.c_uint32), ("launches", C.c_uint32), ("heavy_tiles", C.c_uint32),
                ("blist_blocks", C.c_uint32), ("setup_ms", C.c_double), ("configure_ms", C.c_double),
                ("blist_entries", C.c_uint64), ("blist_max", C.c_uint32), ("slist_on", C.c_uint32),
                ("slist_entries", C.c_uint64), ("path_queue", C.c_uint32), ("slist_built", C.c_uint32),
                ("slist_stale", C.c_uint32)]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_ if n != "pad"}


class RenderParams(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("flags", C.c_uint32),
                ("light", C.c_float * 3), ("clear_color", C.c_uint32),
                ("shard_index", C.c_uint32), ("shard_count", C.c_uint32),
                ("bounces", C.c_uint32), ("seed", C.c_uint32), ("tile_logsize", C.c_uint32)]


class Stats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "primary_rays", "shadow_rays", "geometry_hits", "occluded", "node_visits",
        "tri_tests", "layer_tests", "shaded", "texel_bytes", "tasks")] + [
        ("kernel_ms", C.c_double), ("grid", C.c_uint32), ("block", C.c_uint32),
        ("num_tasks", C.c_uint32), ("local_tiles", C.c_uint32), ("bounce_rays", C.c_uint64),
        ("rect_tests", C.c_uint64), ("edge_tests", C.c_uint64)]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class RtError(RuntimeError):
    pass


_h = None


def lib():
    global _h
    if _h is None:
        h = _lib.load("librtapp.so")
        vp, u32, u64 = C.c_void_p, C.c_uint32, C.c_uint64
        sig = {
            "rt_scene_load": [C.c_char_p, C.POINTER(vp)],
            "rt_scene_free": [vp],
            "rt_scene_info": [vp, C.POINTER(SceneInfo)],
            "rt_scene_export_prims": [vp, vp, u64],
            "rt_scene_export_bvh": [vp, vp, vp],
            "rt_scene_export_bvh4": [vp, vp],
            "rt_renderer_build_bvh": [vp, C.POINTER(BvhBuildStats)],
            "rt_renderer_build_bvh_ex": [vp, u32, C.POINTER(BvhBuildStats)],
            "rt_renderer_bvh_stats": [vp, C.POINTER(BvhBuildStats)],
            "rt_renderer_export_bvh": [vp, vp, vp, C.POINTER(u32), C.POINTER(u32)],
            "rt_renderer_export_bvh4": [vp, vp, C.POINTER(u32)],
            "rt_renderer_export_bvh4h": [vp, vp, C.POINTER(u32)],
            "rt_renderer_export_vis_tree": [vp, vp, C.POINTER(u32), vp, C.POINTER(u32)],
            "rt_renderer_create": [vp, C.c_char_p, C.POINTER(vp)],
            "rt_renderer_free": [vp],
            "rt_renderer_configure": [vp, C.POINTER(RenderParams)],
            "rt_render_start": [vp],
            "rt_render_wait": [vp],
            "rt_render": [vp],
            "rt_render_stats": [vp, C.POINTER(Stats)],
            "rt_render_kernel_ms": [vp, C.POINTER(C.c_double)],
            "rt_render_run_totals": [vp, C.POINTER(C.c_double), C.POINTER(C.c_uint64),
                                     C.POINTER(C.c_uint64)],
            "rt_render_set_timing": [vp, C.c_int],
            "rt_read_framebuffer": [vp, vp, u64],
            "rt_read_depthbuffer": [vp, vp, u64],
            "rt_launch_rows": [vp, vp, u64, C.POINTER(u64)],
            "rt_scene_setup_prims": [vp, u32, u32, vp, u64],
            "rt_scene_setup_vis": [vp, u32, u32, vp, u64],
            "rt_scene_vis_tree": [vp, u32, u32, C.c_float, vp, C.POINTER(u32), vp, C.POINTER(u32),
                                  C.POINTER(u32)],
            "rt_framebuffer_device": [vp, C.POINTER(vp), C.POINTER(u64)],
            "rt_device_stream": [vp, C.POINTER(vp)],
            "rt_device_caps": [vp, C.POINTER(u64)],
            "rt_render_gather": [vp, vp, vp],
            "rt_renderer_setup_stats": [vp, C.POINTER(SetupStats)],
            "rt_renderer_set_light": [vp, C.POINTER(C.c_float)],
            "rt_renderer_set_list_policy": [vp, u32],
            "rt_renderer_export_records": [vp, u32, vp, u64, C.POINTER(u64)],
        }
        for name, argtypes in sig.items():
            fn = getattr(h, name)
            fn.argtypes = argtypes
            fn.restype = C.c_int
        h.rt_last_error.restype = C.c_char_p
        h.rt_last_error.argtypes = []
        _h = h
    return _h


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RtError(f"{what} failed ({rc}): {lib().rt_last_error().decode(errors='replace')}")


class Scene:
    def __init__(self, handle):
        self._h = handle

    @classmethod
    def load(cls, path: str) -> "Scene":
        h = C.c_void_p()
        _check(lib().rt_scene_load(str(path).encode(), C.byref(h)), f"rt_scene_load({path})")
        return cls(h)

    def info(self) -> dict:
        i = SceneInfo()
        _check(lib().rt_scene_info(self._h, C.byref(i)), "rt_scene_info")
        return {n: getattr(i, n) for n, _ in i._fields_ if n not in ("pad", "pad8")}

    def prims(self) -> np.ndarray:
        n = self.info()["num_prims"]
        out = np.zeros((max(n, 1), 3, 10), np.float32)
        _check(lib().rt_scene_export_prims(self._h, out.ctypes.data, n), "rt_scene_export_prims")
        return out[:n]

    def bvh(self):
        info = self.info()
        nodes = np.zeros((max(info["bvh_nodes"], 1), 16), np.float32)
        tris = np.zeros((max(info["bvh_tris"], 1), 12), np.float32)
        _check(lib().rt_scene_export_bvh(self._h, nodes.ctypes.data, tris.ctypes.data),
               "rt_scene_export_bvh")
        return nodes[:info["bvh_nodes"]], tris[:info["bvh_tris"]]

    def bvh4(self):
        """The 4-wide BVH nodes (float32[N4, 32], rt_node4_t); leaves index bvh()'s tris."""
        n = self.info()["bvh4_nodes"]
        nodes4 = np.zeros((max(n, 1), 32), np.float32)
        _check(lib().rt_scene_export_bvh4(self._h, nodes4.ctypes.data), "rt_scene_export_bvh4")
        return nodes4[:n]

    def setup_prims(self, width: int, height: int) -> np.ndarray:
        """rt_prim_t shading records (int32[P, 32]) at width x height."""
        n = self.info()["num_prims"]
        out = np.zeros((max(n, 1), 32), np.int32)
        _check(lib().rt_scene_setup_prims(self._h, width, height, out.ctypes.data, n),
               "rt_scene_setup_prims")
        return out[:n]

    def setup_vis(self, width: int, height: int) -> np.ndarray:
        """Primary-visibility records (uint32[P, 3]: covered-pixel rectangle
        x0|x1<<16, y0|y1<<16 inclusive, depth-word lower bound) at width x height."""
        n = self.info()["num_prims"]
        out = np.zeros((max(n, 1), 3), np.uint32)
        _check(lib().rt_scene_setup_vis(self._h, width, height, out.ctypes.data, n),
               "rt_scene_setup_vis")
        return out[:n]

    def vis_tree(self, width: int, height: int, depth_scale: float = 0.0):
        """The primary rays' screen-space BVH4 at width x height: (refs
        int32[N, 4], leaf_pids int32[M], worst-case stack)."""
        nn, nl, st = C.c_uint32(), C.c_uint32(), C.c_uint32()
        _check(lib().rt_scene_vis_tree(self._h, width, height, depth_scale, None, C.byref(nn), None,
                                       C.byref(nl), C.byref(st)), "rt_scene_vis_tree")
        refs = np.zeros((max(nn.value, 1), 4), np.int32)
        pids = np.zeros(max(nl.value, 1), np.int32)
        _check(lib().rt_scene_vis_tree(self._h, width, height, depth_scale, refs.ctypes.data,
                                       C.byref(nn), pids.ctypes.data, C.byref(nl), C.byref(st)),
               "rt_scene_vis_tree")
        return refs[:nn.value], pids[:nl.value], st.value

    def close(self) -> None:
        if self._h:
            lib().rt_scene_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Renderer:
    """One vortex device running the RT kernel for one scene."""

    def __init__(self, scene: Scene, kernel_dir: str = None):
        self.scene = scene
        h = C.c_void_p()
        _check(lib().rt_renderer_create(scene._h, kernel_dir.encode() if kernel_dir else None,
                                        C.byref(h)), "rt_renderer_create")
        self._h = h
        self.params = None
        # the tree rt_renderer_create built: on the device (binned SAH, the
        # host build's arrays) unless env RT_BVH=host
        st = self.bvh_stats()
        self.gpu_bvh = st["method"] != RT_BVH_BUILD_HOST
        self.gpu_bvh4 = self.gpu_bvh and st["stack4"] != RT_BVH_STACK4_UNUSED

    def configure(self, width: int, height: int, shadows: bool = True, light=DEFAULT_LIGHT,
                  clear_color: int = CLEAR_COLOR, shard_index: int = 0, shard_count: int = 1,
                  instrumented: bool = False, path: bool = False, bounces: int = 4,
                  seed: int = PT_SEED, flat: bool = False, raster: bool = False,
                  bvh_width: int = 0, compact: bool = False, counters: bool = True,
                  host_setup: bool = False, bvh_walk: bool = False) -> None:
        """path=True: diffuse path trace (pt_kernel; `bounces` segments per
        path, RNG `seed`) instead of primary + shadow rays.  flat=True: the
        flat triangle list without BVH (BASELINE config 2).  raster=True:
        the draw3d raster pipeline (any scene; depth/stencil/blend).
        bvh_width: 2 = traverse the binary BVH, 0 = the default (the 4-wide
        BVH unless env RT_BVH_WIDTH=2).  compact=True: the shard layout
        (tile order, as for shard_count > 1) for a single shard too.
        counters=False: no per-workgroup counter rows (the timed product
        configuration; stats() then has the task count and kernel time only).
        host_setup=True: build the per-resolution records with the host loops
        instead of on the device (kernels/rt_setup.hip).  bvh_walk=True: no
        per-block / light-space lists -- primary visibility by the BVH4 packet
        walk, shadow rays by the BVH (BASELINE config 3's full BVH traversal;
        primary+shadow frames run the rt_bvh image)."""
        p = RenderParams()
        p.width, p.height = width, height
        p.flags = ((RT_RENDER_SHADOWS if shadows else 0) | (RT_RENDER_INSTRUMENTED if instrumented else 0)
                   | (RT_RENDER_PATH if path else 0) | (RT_RENDER_FLAT if flat else 0)
                   | (RT_RENDER_RASTER if raster else 0) | (RT_RENDER_BVH2 if bvh_width == 2 else 0)
                   | (RT_RENDER_COMPACT if compact else 0) | (RT_RENDER_COUNTERS if counters else 0)
                   | (RT_RENDER_HOST_SETUP if host_setup else 0) | (RT_RENDER_BVH_WALK if bvh_walk else 0))
        p.bounces, p.seed = bounces, seed
        p.light[:] = [float(np.float32(x)) for x in light]
        p.clear_color = clear_color
        p.shard_index, p.shard_count = shard_index, shard_count
        _check(lib().rt_renderer_configure(self._h, C.byref(p)), "rt_renderer_configure")
        self.params = p
        self.bvh4 = (bvh_width != 2 and os.environ.get("RT_BVH_WIDTH", "4") != "2"
                     and (not self.gpu_bvh or self.gpu_bvh4))
        # BVH4 node steps read 64-B binary16 nodes (rt_node4h_t) when the scene has them
        self.bvh4_f16 = self.bvh4 and (self.gpu_bvh or bool(self.scene.info()["bvh4_f16"]))

    def set_light(self, light) -> None:
        """Move the point light (clip x, y, w) of the current configuration,
        queued behind the frames already started (rt_renderer_set_light: no
        host wait).  When the configuration uses light-space shadow lists
        they are rebuilt on the device -- at once, or (the default policy,
        set_list_policy) once the light has stayed for a few frames, the
        frames before tracing their shadow rays by the BVH packet walk."""
        arr = (C.c_float * 3)(*[float(np.float32(x)) for x in light])
        _check(lib().rt_renderer_set_light(self._h, arr), "rt_renderer_set_light")
        self.params.light[:] = [float(np.float32(x)) for x in light]

    def set_list_policy(self, defer_frames: int) -> None:
        """0: set_light queues the new light's shadow lists at once; n > 0:
        before the (n + 1)-th frame with that light (rt_renderer_set_list_policy)."""
        _check(lib().rt_renderer_set_list_policy(self._h, int(defer_frames)),
               "rt_renderer_set_list_policy")

    def setup_stats(self) -> dict:
        """How the last configure built its records (device / host, launches,
        heavy tiles, setup and configure wall ms)."""
        st = SetupStats()
        _check(lib().rt_renderer_setup_stats(self._h, C.byref(st)), "rt_renderer_setup_stats")
        return st.as_dict()

    def records(self, name: str) -> np.ndarray:
        """One per-resolution record array of the current configuration
        (RECORDS: prims, bbox, vis, vnodes, vtris, vlayers, vgeom, order,
        ptris, geom, bidx, blist -- the per-block candidate lists, blist with
        its 3 padding entries), as [count, words]."""
        which, dt, words = RECORDS[name]
        n = C.c_uint64()
        _check(lib().rt_renderer_export_records(self._h, which, None, 0, C.byref(n)),
               f"rt_renderer_export_records({name})")
        out = np.zeros(max(n.value // 4, 1), dt)
        _check(lib().rt_renderer_export_records(self._h, which, out.ctypes.data, out.nbytes, C.byref(n)),
               f"rt_renderer_export_records({name})")
        return out[:n.value // 4].reshape(-1, words)

    def bvh_stats(self) -> dict:
        """How the current tree was built (method: 0 LBVH, 1 SAH on the
        device, 2 the host build; nodes, depth, stack4, build_ms, ...)."""
        st = BvhBuildStats()
        _check(lib().rt_renderer_bvh_stats(self._h, C.byref(st)), "rt_renderer_bvh_stats")
        return st.as_dict()

    def build_bvh(self, method: str = "lbvh") -> dict:
        """Build the BVH on the device and trace over it from now on; returns
        the build statistics.  method "lbvh": Morton codes + radix tree
        (kernels/bvh_build.hip); "sah": the host builder's binned-SAH tree
        restated on the device (kernels/bvh_sah.hip), equal to the scene's
        host-built arrays."""
        st = BvhBuildStats()
        m = {"lbvh": 0, "sah": 1}[method]
        _check(lib().rt_renderer_build_bvh_ex(self._h, m, C.byref(st)), "rt_renderer_build_bvh_ex")
        self.gpu_bvh = True
        self.gpu_bvh4 = st.stack4 != RT_BVH_STACK4_UNUSED
        if self.params is not None:
            self.bvh4 = self.gpu_bvh4 and not self.params.flags & RT_RENDER_BVH2
            self.bvh4_f16 = self.bvh4  # the device tree carries binary16 records (BVHB_HALF)
        return st.as_dict()

    def export_bvh4(self):
        """The renderer's current BVH4 nodes (float32[N4, 32], rt_node4_t)."""
        n = C.c_uint32()
        _check(lib().rt_renderer_export_bvh4(self._h, None, C.byref(n)), "rt_renderer_export_bvh4")
        nodes4 = np.zeros((max(n.value, 1), 32), np.float32)
        _check(lib().rt_renderer_export_bvh4(self._h, nodes4.ctypes.data, C.byref(n)),
               "rt_renderer_export_bvh4")
        return nodes4[:n.value]

    def export_bvh4h(self):
        """The same nodes as rt_node4h_t records (uint8[N4, 64]: 24 binary16
        planes, 4 child refs) -- what the kernels read."""
        n = C.c_uint32()
        _check(lib().rt_renderer_export_bvh4h(self._h, None, C.byref(n)), "rt_renderer_export_bvh4h")
        out = np.zeros((max(n.value, 1), 64), np.uint8)
        _check(lib().rt_renderer_export_bvh4h(self._h, out.ctypes.data, C.byref(n)),
               "rt_renderer_export_bvh4h")
        return out[:n.value]

    def export_vis_tree(self):
        """The primary rays' tree of the current configuration: (refs
        int32[N, 4] child references, leaf_pids int32[M])."""
        nn, nl = C.c_uint32(), C.c_uint32()
        _check(lib().rt_renderer_export_vis_tree(self._h, None, C.byref(nn), None, C.byref(nl)),
               "rt_renderer_export_vis_tree")
        refs = np.zeros((max(nn.value, 1), 4), np.int32)
        pids = np.zeros(max(nl.value, 1), np.int32)
        _check(lib().rt_renderer_export_vis_tree(self._h, refs.ctypes.data, C.byref(nn),
                                                 pids.ctypes.data, C.byref(nl)),
               "rt_renderer_export_vis_tree")
        return refs[:nn.value], pids[:nl.value]

    def export_bvh(self):
        """The renderer's current BVH: (nodes float32[N, 16], tris float32[M, 12])."""
        nn, nt = C.c_uint32(), C.c_uint32()
        _check(lib().rt_renderer_export_bvh(self._h, None, None, C.byref(nn), C.byref(nt)),
               "rt_renderer_export_bvh")
        nodes = np.zeros((max(nn.value, 1), 16), np.float32)
        tris = np.zeros((max(nt.value, 1), 12), np.float32)
        _check(lib().rt_renderer_export_bvh(self._h, nodes.ctypes.data, tris.ctypes.data,
                                            C.byref(nn), C.byref(nt)), "rt_renderer_export_bvh")
        return nodes[:nn.value], tris[:nt.value]

    def render(self) -> None:
        _check(lib().rt_render(self._h), "rt_render")

    def start(self) -> None:
        _check(lib().rt_render_start(self._h), "rt_render_start")

    def wait(self) -> None:
        _check(lib().rt_render_wait(self._h), "rt_render_wait")

    def stats(self) -> dict:
        s = Stats()
        _check(lib().rt_render_stats(self._h, C.byref(s)), "rt_render_stats")
        return s.as_dict()

    def kernel_ms(self) -> float:
        """HIP-event duration of the last launch (cheap: no counter read-back)."""
        ms = C.c_double()
        _check(lib().rt_render_kernel_ms(self._h, C.byref(ms)), "rt_render_kernel_ms")
        return ms.value

    def run_totals(self):
        """(summed kernel ms of the timed launches, timed launches, all
        launches) since the device opened; waits for every queued frame."""
        ms, nt, n = C.c_double(), C.c_uint64(), C.c_uint64()
        _check(lib().rt_render_run_totals(self._h, C.byref(ms), C.byref(nt), C.byref(n)),
               "rt_render_run_totals")
        return ms.value, nt.value, n.value

    def set_timing(self, timed: bool) -> None:
        """Events on the launches (True, the default) or none (False: no queue
        bound either, back-to-back frames for a host clock); waits for the
        in-flight frames."""
        _check(lib().rt_render_set_timing(self._h, 1 if timed else 0), "rt_render_set_timing")

    def framebuffer(self) -> np.ndarray:
        p = self.params
        if p.shard_count > 1 or p.flags & RT_RENDER_COMPACT:
            n = self.stats()["local_tiles"] * TILE * TILE
            out = np.zeros(max(n, 1), np.uint32)
            _check(lib().rt_read_framebuffer(self._h, out.ctypes.data, n), "rt_read_framebuffer")
            return out[:n]
        out = np.zeros((p.height, p.width), np.uint32)
        _check(lib().rt_read_framebuffer(self._h, out.ctypes.data, out.size), "rt_read_framebuffer")
        return out

    def launch_rows(self) -> np.ndarray:
        """uint32 [grid, 16]: the last launch's per-workgroup counter rows."""
        n = C.c_uint64()
        _check(lib().rt_launch_rows(self._h, None, 0, C.byref(n)), "rt_launch_rows")
        out = np.zeros((max(n.value, 1), 16), np.uint32)
        _check(lib().rt_launch_rows(self._h, out.ctypes.data, n.value, C.byref(n)), "rt_launch_rows")
        return out[:n.value]

    def gather(self, comm) -> np.ndarray:
        """rt_render_gather over a shard.ShardComm: this rank's compact tiles
        to rank 0 (RCCL), assembled there; rank 0 gets the uint32 [H, W]
        frame, other ranks None."""
        p = self.params
        rank, _ = comm.info()
        out = np.zeros((p.height, p.width), np.uint32) if rank == 0 else None
        _check(lib().rt_render_gather(self._h, comm.handle, out.ctypes.data if out is not None else None),
               "rt_render_gather")
        return out

    def depthbuffer(self) -> np.ndarray:
        """RT_RENDER_RASTER: uint32 [H, W] depth/stencil words (stencil << 24 | depth)."""
        p = self.params
        out = np.zeros((p.height, p.width), np.uint32)
        _check(lib().rt_read_depthbuffer(self._h, out.ctypes.data, out.size), "rt_read_depthbuffer")
        return out

    def framebuffer_device(self):
        ptr, nbytes = C.c_void_p(), C.c_uint64()
        _check(lib().rt_framebuffer_device(self._h, C.byref(ptr), C.byref(nbytes)),
               "rt_framebuffer_device")
        return ptr.value, nbytes.value

    def device_stream(self) -> int:
        s = C.c_void_p()
        _check(lib().rt_device_stream(self._h, C.byref(s)), "rt_device_stream")
        return s.value

    def caps(self):
        c = (C.c_uint64 * 8)()
        _check(lib().rt_device_caps(self._h, c), "rt_device_caps")
        return list(c)

    def close(self) -> None:
        if self._h:
            lib().rt_renderer_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def deinterleave_tiles(shards, width: int, height: int) -> np.ndarray:
    """Assemble per-rank compact tile buffers (rank r holds tiles t with
    t % G == r, each 32x32 in 8x8-block/lane task order) into a W x H image."""
    from .shard import deinterleave_tiles as _d
    return _d(shards, width, height)
