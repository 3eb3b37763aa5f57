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
    """Gather the ranks' compact tile buffers to rank 0 and scatter them into
    the frame.  Buffers are padded to the largest rank's size so one
    dist.gather moves them; on RCCL a gather to one root is point-to-point
    sends to it, each peer over its own xGMI link (no ring all-gather)."""

    def __init__(self, dist, width: int, height: int, device):
        import torch
        self.dist = dist
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.width, self.height = width, height
        self.max_local = local_tiles(width, height, 0, self.world) * TILE * TILE
        self.local = torch.zeros(self.max_local, dtype=torch.int32, device=device)
        self.parts = None
        if self.rank == 0:
            self.parts = [torch.empty_like(self.local) for _ in range(self.world)]
            src, dst = [], []
            for r in range(self.world):
                idx = task_pixel_index(width, height, r, self.world)
                ok = np.nonzero(idx >= 0)[0]
                src.append(ok + r * self.max_local)
                dst.append(idx[ok])
            self.src = torch.from_numpy(np.concatenate(src)).to(device)
            self.dst = torch.from_numpy(np.concatenate(dst)).to(device)
            self.image = torch.zeros(width * height, dtype=torch.int32, device=device)

    def __call__(self, local=None):
        """local: this rank's compact buffer (int32 tensor); None = use
        self.local (filled by the caller, e.g. by a device copy)."""
        if local is not None:
            self.local[:local.numel()].copy_(local.reshape(-1))
        self.dist.gather(self.local, self.parts, dst=0)
        if self.rank != 0:
            return None
        import torch
        self.image[self.dst] = torch.cat(self.parts)[self.src]
        return self.image
