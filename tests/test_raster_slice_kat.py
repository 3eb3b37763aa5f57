"""The RTL raster slice's known-answer test pins the rasterizer's coverage
predicate.

hw/unit_tests/raster_unit/raster_slice/testbench.cpp:53-66 feeds one 16x16
tile at (0, 256) with three edges and their values at the tile origin;
golden_data/test_data.txt lists the pixels the slice covers (compare.py:
same set).  The fixture (tests/golden/raster_slice_kat.json,
scripts/make_raster_slice_kat.py) holds both.  The slice steps each edge
from its origin value, v + a*dx + b*dy, so the absolute edge the primitive
records hold is (a, b, v - a*x_loc - b*y_loc); the oracle's orc_edge_cover
(the predicate of raster.c / vis.c / rt.c) over the tile must give exactly
the golden set.  The GPU's gfx::covers runs the same vector in
tests/test_gpu_edge_kat.py."""
import json
import os

import numpy as np

from conftest import GOLDEN


def kat():
    with open(os.path.join(GOLDEN, "raster_slice_kat.json")) as f:
        return json.load(f)


def absolute_edges(k):
    x0, y0 = k["x_loc"], k["y_loc"]
    return [[a, b, v - a * x0 - b * y0] for (a, b, _), v in zip(k["edges"], k["edge_func_val"])]


def golden_mask(k):
    t = k["tile"]
    m = np.zeros((t, t), np.uint8)
    for x, y in k["covered"]:
        m[y - k["y_loc"], x - k["x_loc"]] = 1
    return m


def test_fixture_is_the_reference_vector():
    k = kat()
    assert k["tile"] == 16 and (k["x_loc"], k["y_loc"]) == (0, 256)
    assert len(k["covered"]) == 64 and len(set(map(tuple, k["covered"]))) == 64
    # every golden pixel lies in the tile
    assert all(0 <= x < 16 and 256 <= y < 272 for x, y in k["covered"])


def test_oracle_edge_cover_equals_raster_slice_golden(oracle_lib):
    k = kat()
    t = k["tile"]
    m = oracle_lib.edge_cover(absolute_edges(k), k["x_loc"], k["y_loc"], t, t)
    assert np.array_equal(m, golden_mask(k))


def test_extents_bound_the_block_steps():
    """The slice's extents (per edge, the largest step over a block it adds
    before rejecting one): with them no covered block is rejected --
    origin value + extent >= 0 for every 8x8 block holding a golden pixel."""
    k = kat()
    g = golden_mask(k)
    for by in range(2):
        for bx in range(2):
            if not g[8 * by:8 * by + 8, 8 * bx:8 * bx + 8].any():
                continue
            for (a, b, _), v, ext in zip(k["edges"], k["edge_func_val"], k["extents"]):
                assert v + a * 8 * bx + b * 8 * by + ext >= 0
