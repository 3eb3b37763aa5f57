"""Rank 0's frame assembly kernel (include/rt_shard.h rt_frame_assemble,
runtime/frame_assemble.hip) against the host restatement of the compact
tile layout (shard.deinterleave_tiles / task_pixel_index), bit for bit, on
random shard contents: image sizes with edge tiles and widths that are not a
multiple of 4, 1..8 ranks, and the receive-buffer stride FrameGather uses."""
import ctypes

import numpy as np
import pytest

from skybox_rt_amd import _lib, shard

pytestmark = pytest.mark.gpu


def _assemble_fn():
    f = _lib.load("librt_shard.so").rt_frame_assemble
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                  ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p]
    return f


@pytest.mark.parametrize("w,h,world", [(64, 64, 1), (1024, 1024, 2), (1000, 520, 3),
                                       (333, 97, 4), (2896, 2896, 8), (130, 66, 8),
                                       (4096, 4096, 8)])
def test_frame_assemble_equals_host_deinterleave(w, h, world):
    import torch
    f = _assemble_fn()
    per = shard.local_tiles(w, h, 0, world) * 1024
    rng = np.random.default_rng(w * 7 + h * 3 + world)
    recv = rng.integers(0, 2**32, size=world * per, dtype=np.uint64).astype(np.uint32)
    want = shard.deinterleave_tiles([recv[r * per:(r + 1) * per] for r in range(world)], w, h)
    d_recv = torch.from_numpy(recv.view(np.int32)).cuda()
    d_img = torch.full((w * h,), -1, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    assert f(d_img.data_ptr(), d_recv.data_ptr(), w, h, world, per, s.cuda_stream) == 0
    torch.cuda.synchronize()
    got = d_img.cpu().numpy().view(np.uint32).reshape(h, w)
    assert np.array_equal(got, want)


def test_frame_assemble_rejects_bad_arguments():
    import torch
    f = _assemble_fn()
    buf = torch.zeros(4096, dtype=torch.int32, device="cuda")
    p = buf.data_ptr()
    assert f(None, p, 64, 64, 1, 4096, None) == -1
    assert f(p, p, 0, 64, 1, 4096, None) == -1
    assert f(p, p, 64, 64, 0, 4096, None) == -1
    assert f(p, p, 64, 64, 1, 1000, None) == -1       # stride not a multiple of 1024
    assert f(p, p, 64, 64, 1, 3072, None) == -1       # stride below rank 0's 4 tiles
