"""Multi-GPU frame sharding: 32x32 tiles dealt round-robin,
tile t -> rank t % G (the reference's raster-unit striding,
sim/simx/raster_unit.cpp:109-111, 224-227); every rank renders its tiles into
a compact buffer of its local tiles (local tile lt = global tile
rank + lt * G, each tile row-major: slot = lt * 1024 + 32 * (y % 32) + x % 32,
the RT kernels' store_pixel); one gather to rank 0 -- over RCCL (backend
"nccl") on the GPUs, gloo in the CPU tests -- and the frame assembly there
(on the GPU the HIP kernel runtime/frame_assemble.hip behind
include/rt_shard.h, on the CPU rehearsal a numpy/torch index gather).  That gather is the only exchange of the path: the frame shards with
no data-path collective.

    g = FrameGather(dist, width, height, device)
    image = g(local)   # rank 0: int32[H*W] image, other ranks: None
"""
from __future__ import annotations

import ctypes

import numpy as np

TILE = 32


def tiles_of(width: int, height: int):
    return (width + TILE - 1) // TILE, (height + TILE - 1) // TILE


def local_tiles(width: int, height: int, rank: int, world: int) -> int:
    tx, ty = tiles_of(width, height)
    n = tx * ty
    return (n - rank + world - 1) // world if n > rank else 0


def task_pixel_index(width: int, height: int, rank: int, world: int) -> np.ndarray:
    """Image index (y * W + x) of every slot of rank's compact buffer, -1 for
    the slots of edge tiles that overhang the image.  Restates the kernels'
    store_pixel compact index (kernels/rt_trace.h)."""
    tx, _ = tiles_of(width, height)
    n = local_tiles(width, height, rank, world)
    t = np.arange(n * TILE * TILE, dtype=np.int64)
    lt, row, col = t >> 10, (t >> 5) & 31, t & 31
    gt = rank + lt * world
    x = (gt % tx) * TILE + col
    y = (gt // tx) * TILE + row
    return np.where((x < width) & (y < height), y * width + x, -1)


def deinterleave_tiles(shards, width: int, height: int) -> np.ndarray:
    """Host form: assemble per-rank compact buffers into a W x H uint32 image."""
    G = len(shards)
    img = np.zeros(width * height, np.uint32)
    for r, buf in enumerate(shards):
        idx = task_pixel_index(width, height, r, G)
        buf = np.asarray(buf, np.uint32)[:idx.size]
        ok = idx >= 0
        img[idx[ok]] = buf[ok]
    return img.reshape(height, width)


class FrameGather:
    """Gather the ranks' compact tile buffers to rank 0 and assemble the
    frame there.  Buffers are padded to the largest rank's size so one
    dist.gather moves them, straight into views of one receive buffer (on
    RCCL a gather to one root is point-to-point sends to it, each peer over
    its own xGMI link -- no ring all-gather); the frame is then assembled by
    ONE HIP kernel (rt_frame_assemble: arithmetic tile -> rank mapping,
    coalesced 128-B tile rows; 8 B of HBM traffic per pixel, no index array).

    Synchronous:  image = g(local)
    Pipelined:    g.start(slot[, stream]) after filling g.locals[slot] --
    the gather (and on rank 0 the frame assembly) is enqueued (async_op) so
    it overlaps the next frames' renders.  Every slot has its own send and
    receive buffers, so frames in flight never share memory; before a slot
    is refilled, g.reclaim(slot) waits ON THE HOST until that slot's
    previous gather and assembly have completed -- normally long done, so
    the frame loop puts no cross-stream waits on the render stream.  On
    GPUs the gather follows `stream` (the stream that filled the slot) and
    the assembly runs on a stream of its own.  g.finish(slot) = reclaim."""

    def __init__(self, dist, width: int, height: int, device, slots: int = 2):
        import torch
        self.dist = dist
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.width, self.height = width, height
        self.device = device
        self.cuda = getattr(device, "type", str(device)) == "cuda"
        self.max_local = local_tiles(width, height, 0, self.world) * TILE * TILE
        self.locals = [torch.zeros(self.max_local, dtype=torch.int32, device=device)
                       for _ in range(slots)]
        self.local = self.locals[0]
        self.works = [None] * slots
        self.asm_done = [None] * slots
        self.recvs = self.parts_s = None
        self.recv = self.parts = self.perm = self.image = None
        self.asm_stream = torch.cuda.Stream(device) if self.cuda and self.rank == 0 else None
        if self.rank == 0:
            self.recvs = [torch.empty(self.world * self.max_local, dtype=torch.int32, device=device)
                          for _ in range(slots)]
            self.parts_s = [list(r.split(self.max_local)) for r in self.recvs]
            self.recv, self.parts = self.recvs[0], self.parts_s[0]
            self.image = torch.zeros(width * height, dtype=torch.int32, device=device)
            if self.cuda:
                # the HIP assembly kernel (include/rt_shard.h); no torch fallback
                from . import _lib
                self._asm = _lib.load("librt_shard.so").rt_frame_assemble
                self._asm.restype = ctypes.c_int
                self._asm.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                      ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64,
                                      ctypes.c_void_p]
            else:
                # host-staged rehearsal (gloo): one index gather through the
                # permutation frame pixel i <- slot perm[i]
                perm = np.empty(width * height, np.int64)
                for r in range(self.world):
                    idx = task_pixel_index(width, height, r, self.world)
                    ok = np.nonzero(idx >= 0)[0]
                    perm[idx[ok]] = ok + r * self.max_local
                self.perm = torch.from_numpy(perm)

    def _assemble(self, slot: int = 0):
        import torch
        if self.cuda:
            rc = self._asm(self.image.data_ptr(), self.recvs[slot].data_ptr(), self.width,
                           self.height, self.world, self.max_local,
                           torch.cuda.current_stream(self.device).cuda_stream)
            if rc != 0:
                raise RuntimeError(f"rt_frame_assemble failed ({rc})")
        else:
            torch.index_select(self.recvs[slot], 0, self.perm, out=self.image)

    def __call__(self, local=None):
        """local: this rank's compact buffer (int32 tensor); None = use
        self.local (filled by the caller, e.g. by a device copy)."""
        self.reclaim(0)
        if local is not None:
            self.local[:local.numel()].copy_(local.reshape(-1))
        self.dist.gather(self.local, self.parts, dst=0)
        if self.rank != 0:
            return None
        self._assemble(0)
        return self.image

    def start(self, slot: int, stream=None) -> None:
        """Enqueue the gather of self.locals[slot] (+ the assembly on rank 0).
        stream: the CUDA stream that filled the slot (default: current)."""
        import contextlib
        import torch
        self.reclaim(slot)
        parts = self.parts_s[slot] if self.rank == 0 else None
        ctx = torch.cuda.stream(stream) if (self.cuda and stream is not None) else contextlib.nullcontext()
        with ctx:
            w = self.dist.gather(self.locals[slot], parts, dst=0, async_op=True)
        if self.rank == 0:
            if self.asm_stream is not None:
                with torch.cuda.stream(self.asm_stream):
                    w.wait()  # the assembly stream waits for the gather (the host does not)
                    self._assemble(slot)
                    ev = torch.cuda.Event()
                    ev.record(self.asm_stream)
                    self.asm_done[slot] = ev
            else:
                w.wait()
                self._assemble(slot)
        self.works[slot] = w

    def reclaim(self, slot: int) -> None:
        """Host wait until the slot's previous gather (and assembly) are done."""
        import time
        w, ev = self.works[slot], self.asm_done[slot]
        if w is not None:
            if self.cuda:
                while not w.is_completed():
                    time.sleep(0)
            else:
                w.wait()
            self.works[slot] = None
        if ev is not None:
            ev.synchronize()
            self.asm_done[slot] = None

    finish = reclaim


class ShardComm:
    """ctypes binding of include/rt_shard.h's RCCL communicator
    (librt_shard.so): the C-ABI frame exchange a C host uses without torch
    (rtapp -G rank,ranks).  Renderer.gather(comm) runs rt_render_gather."""
    ID_BYTES = 128

    @staticmethod
    def _lib():
        from . import _lib
        h = _lib.load("librt_shard.so")
        h.rt_shard_unique_id.argtypes = [ctypes.c_char_p]
        h.rt_shard_comm_init.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_char_p,
                                         ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int]
        h.rt_shard_comm_free.argtypes = [ctypes.c_void_p]
        h.rt_shard_comm_info.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32),
                                         ctypes.POINTER(ctypes.c_uint32)]
        h.rt_shard_local_words.argtypes = [ctypes.c_uint32] * 4
        h.rt_shard_local_words.restype = ctypes.c_uint64
        return h

    @classmethod
    def unique_id(cls) -> bytes:
        buf = ctypes.create_string_buffer(cls.ID_BYTES)
        if cls._lib().rt_shard_unique_id(buf) != 0:
            raise RuntimeError("rt_shard_unique_id failed")
        return buf.raw

    def __init__(self, uid: bytes, rank: int, world: int, device: int = 0):
        self.handle = ctypes.c_void_p()
        if self._lib().rt_shard_comm_init(ctypes.byref(self.handle), uid, rank, world, device) != 0:
            raise RuntimeError("rt_shard_comm_init failed")

    def info(self):
        r, w = ctypes.c_uint32(), ctypes.c_uint32()
        if self._lib().rt_shard_comm_info(self.handle, ctypes.byref(r), ctypes.byref(w)) != 0:
            raise RuntimeError("rt_shard_comm_info failed")
        return r.value, w.value

    def close(self):
        if self.handle:
            self._lib().rt_shard_comm_free(self.handle)
            self.handle = None

