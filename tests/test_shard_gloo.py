"""Multi-rank frame sharding on CPU (gloo, world_size 2 and 3): every rank
builds its compact tile buffer from a synthetic frame with the kernels'
task -> pixel mapping (shard.task_pixel_index, the mapping the GPU sharding
tests check against real renders), skybox_rt_amd.shard.FrameGather gathers
them to rank 0 -- the same code bench.py runs over RCCL -- and rank 0 must
rebuild the frame exactly."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from skybox_rt_amd import shard


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _frame(w, h):
    rng = np.random.default_rng(w * 7919 + h)
    return rng.integers(0, 2**31 - 1, w * h, dtype=np.int64).astype(np.int32)


def _worker(rank, world, port, w, h, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        frame = _frame(w, h)
        idx = shard.task_pixel_index(w, h, rank, world)
        local = np.where(idx >= 0, frame[np.maximum(idx, 0)], 0).astype(np.int32)
        g = FrameGatherCPU(w, h)
        img = g(torch.from_numpy(local))
        ok = rank != 0 or bool(np.array_equal(img.numpy(), frame))
        # the pipelined form bench.py runs: two slots in flight
        for step in range(3):
            slot = step % 2
            g.locals[slot][:local.size].copy_(torch.from_numpy(local))
            g.start(slot)
        g.finish(0)
        g.finish(1)
        if rank == 0:
            q.put(ok and bool(np.array_equal(g.image.numpy(), frame)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def FrameGatherCPU(w, h):
    return shard.FrameGather(dist, w, h, torch.device("cpu"))


@pytest.mark.parametrize("world,w,h", [(2, 256, 256), (2, 1000, 1000), (3, 333, 200),
                                       (3, 64, 64)])
def test_frame_gather_gloo(world, w, h):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, w, h, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert q.get(timeout=10) is True


def test_task_pixel_index_is_a_partition():
    for world in (1, 2, 3, 8):
        for w, h in ((1024, 1024), (333, 200), (32, 32), (40, 1)):
            seen = np.concatenate([shard.task_pixel_index(w, h, r, world) for r in range(world)])
            seen = seen[seen >= 0]
            assert seen.size == w * h and np.array_equal(np.sort(seen), np.arange(w * h))
