#!/usr/bin/env python3
"""Rank 0's frame assembly at the multi-GPU frame sizes: the HIP kernel
(rt_frame_assemble) vs the earlier form, torch.index_select through an int64
permutation.  HIP-event timed on one stream; one JSON line per size/world."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from skybox_rt_amd import _lib, shard
    f = _lib.load("librt_shard.so").rt_frame_assemble
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                  ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p]
    for side, world in ((1024, 1), (1448, 2), (2048, 4), (2896, 8), (4096, 8)):
        per = shard.local_tiles(side, side, 0, world) * 1024
        recv = torch.randint(-2**31, 2**31 - 1, (world * per,), dtype=torch.int32, device="cuda")
        img = torch.empty(side * side, dtype=torch.int32, device="cuda")
        perm = np.empty(side * side, np.int64)
        for r in range(world):
            idx = shard.task_pixel_index(side, side, r, world)
            ok = np.nonzero(idx >= 0)[0]
            perm[idx[ok]] = ok + r * per
        dperm = torch.from_numpy(perm).cuda()
        s = torch.cuda.current_stream()
        out = {"side": side, "world": world, "pixels": side * side}
        for name, fn in (("hip", lambda: f(img.data_ptr(), recv.data_ptr(), side, side, world, per,
                                            s.cuda_stream)),
                         ("index_select", lambda: torch.index_select(recv, 0, dperm, out=img))):
            for _ in range(5):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 50
            e0.record()
            for _ in range(n):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / n
            out[name + "_ms"] = round(ms, 5)
            out[name + "_GBps"] = round(8 * side * side / ms / 1e6, 1)  # 4 B read + 4 B written
        ref = torch.index_select(recv, 0, dperm)
        f(img.data_ptr(), recv.data_ptr(), side, side, world, per, s.cuda_stream)
        torch.cuda.synchronize()
        out["identical"] = bool(torch.equal(ref, img))
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
