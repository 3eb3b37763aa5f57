"""Multi-GPU frame sharding: 32x32 tiles dealt round-robin,
tile t -> rank t % G (the reference's raster-unit striding,
sim/simx/raster_unit.cpp:109-111, 224-227); every rank renders its tiles into
a compact buffer in task order (the RT kernels' task_pixel mapping: tile,
then 8x8 block, then lane); one gather to rank 0 -- over RCCL (backend
"nccl") on the GPUs, gloo in the CPU tests -- and a de-interleave scatter
there.  That gather is the only exchange of the path: the frame shards with
no data-path collective.

    g = FrameGather(dist, width, height, device)
    image = g(local)   # rank 0: int32[H*W] image, other ranks: None
"""
from __future__ import annotations

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
    task_pixel (kernels/rt_trace.h)."""
    tx, _ = tiles_of(width, height)
    n = local_tiles(width, height, rank, world)
    t = np.arange(n * TILE * TILE, dtype=np.int64)
    lt, blk, ln = t >> 10, (t >> 6) & 15, t & 63
    gt = rank + lt * world
    x = (gt % tx) * TILE + (blk & 3) * 8 + (ln & 7)
    y = (gt // tx) * TILE + (blk >> 2) * 8 + (ln >> 3)
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
    its own xGMI link -- no ring all-gather); the frame is then ONE index
    gather through a precomputed permutation (frame pixel i <- slot perm[i]).

    Synchronous:  image = g(local)
    Pipelined:    g.start(slot) after filling g.locals[slot] -- the gather
    and the frame assembly are enqueued (async_op) so they overlap the next
    frame's render; g.finish(slot) (or the next start on the same slot)
    waits for them before the buffer is reused.  Two slots."""

    def __init__(self, dist, width: int, height: int, device, slots: int = 2):
        import torch
        self.dist = dist
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.width, self.height = width, height
        self.device = device
        self.max_local = local_tiles(width, height, 0, self.world) * TILE * TILE
        self.locals = [torch.zeros(self.max_local, dtype=torch.int32, device=device)
                       for _ in range(slots)]
        self.local = self.locals[0]
        self.works = [None] * slots
        self.recv = self.parts = self.perm = self.image = None
        if self.rank == 0:
            self.recv = torch.empty(self.world * self.max_local, dtype=torch.int32, device=device)
            self.parts = list(self.recv.split(self.max_local))
            perm = np.empty(width * height, np.int64)
            for r in range(self.world):
                idx = task_pixel_index(width, height, r, self.world)
                ok = np.nonzero(idx >= 0)[0]
                perm[idx[ok]] = ok + r * self.max_local
            self.perm = torch.from_numpy(perm).to(device)
            self.image = torch.zeros(width * height, dtype=torch.int32, device=device)

    def _assemble(self):
        import torch
        torch.index_select(self.recv, 0, self.perm, out=self.image)

    def __call__(self, local=None):
        """local: this rank's compact buffer (int32 tensor); None = use
        self.local (filled by the caller, e.g. by a device copy)."""
        if local is not None:
            self.local[:local.numel()].copy_(local.reshape(-1))
        self.dist.gather(self.local, self.parts, dst=0)
        if self.rank != 0:
            return None
        self._assemble()
        return self.image

    def start(self, slot: int) -> None:
        """Enqueue the gather of self.locals[slot] (+ the assembly on rank 0)."""
        self.finish(slot)
        w = self.dist.gather(self.locals[slot], self.parts, dst=0, async_op=True)
        if self.rank == 0:
            w.wait()          # the current stream waits for the gather (the host does not)
            self._assemble()
        self.works[slot] = w

    def finish(self, slot: int) -> None:
        """Block until the gather from self.locals[slot] has completed."""
        import torch
        w = self.works[slot]
        if w is not None:
            w.wait()
            if self.device.type == "cuda":
                torch.cuda.current_stream().synchronize()
            self.works[slot] = None
