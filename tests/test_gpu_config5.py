"""BASELINE config 5 at full size on one GPU: a 4096x4096 tekkaman frame
(primary + shadow rays) rendered as the 8 tile shards of an 8-GPU node
(32x32 tile t -> shard t % 8, sim/simx/raster_unit.cpp:109-111 striding),
the shards' compact buffers laid side by side as the RCCL gather leaves them
in rank 0's receive buffer and assembled by rt_frame_assemble -- which must
give the full single-launch 4096^2 render, which must equal the oracle bit
for bit.  Also the FrameGather path itself at world size 1 (RCCL to self):
compact render -> gather -> assembly == the full render.  Exercises the
arena addressing and compact-tile indexing at config 5's 64 MiB framebuffer."""
import ctypes
import os
import socket

import numpy as np
import pytest

from conftest import scene_path

pytestmark = pytest.mark.gpu

from skybox_rt_amd import _lib, rt, shard  # noqa: E402

W = H = 4096
SHARDS = 8


@pytest.fixture(scope="module")
def tek():
    s = rt.Scene.load(scene_path("tekkaman"))
    r = rt.Renderer(s)
    r.configure(W, H, shadows=True)
    r.render()
    full = r.framebuffer().copy()
    yield s, r, full
    r.close()
    s.close()


def test_config5_full_frame_equals_oracle(tek, oracle_lib):
    po = oracle_lib
    _, _, full = tek
    c, _, _, k = po.rt_render(po.OracleScene(po.cgltrace.load(scene_path("tekkaman"))),
                              po.rt_params(W, H, shadows=True, nthreads=min(16, os.cpu_count() or 1)))
    bad = int((full != c).sum())
    assert bad == 0, f"{bad} of {W * H} pixels differ from the oracle at 4096^2"
    assert k["primary_rays"] == W * H


def test_config5_eight_shards_assemble_to_the_full_frame(tek):
    import torch
    _, r, full = tek
    per = shard.local_tiles(W, H, 0, SHARDS) * 1024
    recv = torch.zeros(SHARDS * per, dtype=torch.int32, device="cuda")
    rays = 0
    for i in range(SHARDS):
        r.configure(W, H, shadows=True, shard_index=i, shard_count=SHARDS)
        r.render()
        part = r.framebuffer()
        assert part.size == shard.local_tiles(W, H, i, SHARDS) * 1024
        recv[i * per:i * per + part.size] = torch.from_numpy(part.view(np.int32)).cuda()
        rays += r.stats()["primary_rays"]
    assert rays == W * H
    f = _lib.load("librt_shard.so").rt_frame_assemble
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                  ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p]
    img = torch.full((W * H,), -1, dtype=torch.int32, device="cuda")
    assert f(img.data_ptr(), recv.data_ptr(), W, H, SHARDS, per,
             torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    got = img.cpu().numpy().view(np.uint32).reshape(H, W)
    assert np.array_equal(got, full)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_config5_frame_gather_world_size_1(tek):
    """The bench's exchange code (FrameGather over RCCL) at world size 1."""
    import torch
    import torch.distributed as dist
    from skybox_rt_amd.shard import FrameGather
    _, r, full = tek
    dev = torch.device("cuda", torch.cuda.current_device())
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1, device_id=dev)
    try:
        r.configure(W, H, shadows=True, compact=True)
        r.render()
        local = torch.from_numpy(r.framebuffer().view(np.int32)).to(dev)
        fg = FrameGather(dist, W, H, dev)
        image = fg(local)
        torch.cuda.synchronize()
        assert np.array_equal(image.cpu().numpy().view(np.uint32).reshape(H, W), full)
    finally:
        dist.destroy_process_group()


def test_c_abi_gather_world_size_1(tek):
    """The C-ABI exchange (include/rt_shard.h over RCCL, no torch):
    rt_render_gather at world size 1 == the full frame, at 4096^2."""
    from skybox_rt_amd.shard import ShardComm
    _, r, full = tek
    comm = ShardComm(ShardComm.unique_id(), 0, 1, 0)
    try:
        assert comm.info() == (0, 1)
        r.configure(W, H, shadows=True, shard_index=0, shard_count=1, compact=True)
        r.render()
        assert np.array_equal(r.gather(comm), full)
    finally:
        comm.close()


def test_rtapp_rank_mode_world_size_1(tmp_path):
    """rtapp -G 0,1: the C host's multi-GPU mode (render its shard, RCCL
    gather, assemble on rank 0) reproduces the reference's golden image."""
    import subprocess
    from conftest import GOLDEN
    exe = os.path.join(_lib.LIB_DIR, "rtapp")
    out = subprocess.run([exe, "-t", scene_path("tekkaman"), "-w", "128", "-h", "128", "-G", "0,1",
                          "-I", str(tmp_path / "id"), "-o", str(tmp_path / "o.png"), "-r",
                          f"{GOLDEN}/draw3d/tekkaman_ref_128.png"],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "communicator: 1 ranks" in out.stdout and "PASSED!" in out.stdout


def test_torch_and_c_abi_exchanges_give_identical_frames():
    """The two bindings of the frame exchange -- bench.py's torch FrameGather
    and the C-ABI rt_render_gather C hosts use (librt_shard.so) -- return the
    same frame, frame after frame (three lights, so the frames differ), at
    world size 1 over RCCL, and each equals the full render."""
    import torch
    import torch.distributed as dist
    from skybox_rt_amd.shard import FrameGather, ShardComm
    s = rt.Scene.load(scene_path("tekkaman"))
    r = rt.Renderer(s)
    side = 512
    dev = torch.device("cuda", torch.cuda.current_device())
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1, device_id=dev)
    comm = ShardComm(ShardComm.unique_id(), 0, 1, 0)
    try:
        fg = FrameGather(dist, side, side, dev)
        for light in ((0.0, 60.0, 80.0), (-40.0, 30.0, 60.0), (25.0, -10.0, 120.0)):
            r.configure(side, side, shadows=True, light=light)
            r.render()
            full = r.framebuffer().copy()
            r.configure(side, side, shadows=True, light=light, shard_index=0, shard_count=1,
                        compact=True)
            r.render()
            c_img = r.gather(comm)
            t_img = fg(torch.from_numpy(r.framebuffer().view(np.int32)).to(dev))
            torch.cuda.synchronize()
            t_img = t_img.cpu().numpy().view(np.uint32).reshape(side, side)
            assert np.array_equal(c_img, t_img), light
            assert np.array_equal(c_img, full), light
    finally:
        comm.close()
        dist.destroy_process_group()
        r.close()
        s.close()
