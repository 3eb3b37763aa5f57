"""The GPU's coverage predicate (gfx::covers: raster_kernel.hip and the RT
kernels' primary tests) on the RTL raster slice's known-answer vector
(hw/unit_tests/raster_unit/raster_slice/testbench.cpp:53-66,
golden_data/test_data.txt; tests/test_raster_slice_kat.py has the oracle
side) and on random edges -- int32 wrap included -- against the oracle's
orc_edge_cover.  Runs the edge_kat image through the Vortex C ABI."""
import os
import struct

import numpy as np
import pytest

from test_raster_slice_kat import absolute_edges, golden_mask, kat

pytestmark = pytest.mark.gpu

from skybox_rt_amd import _lib, vortex  # noqa: E402


def gpu_cover(edges, x0, y0, w, h):
    d = vortex.Device()
    try:
        k = d.upload_kernel_file(os.path.join(_lib.LIB_DIR, "edge_kat.vxbin"))
        out = d.mem_alloc(4 * w * h)
        vals = d.mem_alloc(12 * w * h)
        e = np.asarray(edges, np.int64).reshape(9).astype(np.int32)
        args = d.upload_bytes(struct.pack("<9i5IQQ", *e.tolist(), x0, y0, w, h, 0, out.address,
                                          vals.address))
        d.start(k, args)
        d.ready_wait()
        o = np.frombuffer(out.read(), np.uint32).reshape(h, w)
        v = np.frombuffer(vals.read(), np.int32).reshape(h, w, 3)
        return o, v
    finally:
        d.close()


def test_gpu_covers_equals_raster_slice_golden():
    k = kat()
    t = k["tile"]
    o, v = gpu_cover(absolute_edges(k), k["x_loc"], k["y_loc"], t, t)
    assert np.array_equal((o >> 31).astype(np.uint8), golden_mask(k))
    # the slice's own stepping: origin value + a*dx + b*dy
    dy, dx = np.mgrid[0:t, 0:t]
    for i, ((a, b, _), e0) in enumerate(zip(k["edges"], k["edge_func_val"])):
        assert np.array_equal(v[:, :, i], (e0 + a * dx + b * dy).astype(np.int32))


@pytest.mark.parametrize("seed", range(4))
def test_gpu_covers_equals_oracle_random_edges(oracle_lib, seed):
    rng = np.random.default_rng(seed)
    # Q15.16-sized coefficients; large offsets wrap int32 as on the host
    e = rng.integers(-(1 << 20), 1 << 20, size=(3, 3)).astype(np.int64)
    e[:, 2] = rng.integers(-(1 << 31), (1 << 31) - 1, size=3)
    x0, y0 = int(rng.integers(0, 4000)), int(rng.integers(0, 4000))
    o, _ = gpu_cover(e, x0, y0, 64, 48)
    m = oracle_lib.edge_cover(e, x0, y0, 64, 48)
    assert np.array_equal((o >> 31).astype(np.uint8), m)
