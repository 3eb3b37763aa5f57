#!/usr/bin/env python3
"""Writes tests/golden/raster_slice_kat.json: the RTL raster slice's
known-answer vector (run once, here, where /root/reference exists).

Inputs: hw/unit_tests/raster_unit/raster_slice/testbench.cpp:53-66 (config
#1, tile 16, block 8): tile origin (x_loc, y_loc) = (0, 256), the three edges
(a, b, c), the edge values at the tile origin (edge_func_val) and the
extents.  Expected output: golden_data/test_data.txt, one covered pixel
"x y" per line (compare.py checks the slice's output set against it).

The slice steps each edge from its value at the tile origin
(v + a*dx + b*dy); its `c` column is not used for that.  The equivalent
absolute-coordinate edge -- what the primitive records and
orc_edge_cover / gfx::covers evaluate -- is (a, b, v - a*x_loc - b*y_loc)."""
import json
import os
import sys

REF = "/root/reference/hw/unit_tests/raster_unit/raster_slice"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "tests", "golden", "raster_slice_kat.json")


def main():
    x_loc, y_loc = 0, 256
    edges = [[-73, -36, 65456], [5, -89, 65440], [0, 255, -65280]]
    edge_func_val = [518, 42976, 0]
    extents = [0, 320, 16320]
    with open(os.path.join(REF, "golden_data", "test_data.txt")) as f:
        pix = [tuple(int(v) for v in ln.split()) for ln in f if ln.strip()]
    doc = {
        "source": "hw/unit_tests/raster_unit/raster_slice/testbench.cpp:53-66 + golden_data/test_data.txt",
        "tile": 16, "block": 8, "x_loc": x_loc, "y_loc": y_loc,
        "edges": edges, "edge_func_val": edge_func_val, "extents": extents,
        "covered": sorted(pix),
    }
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
    print(f"{OUT}: {len(pix)} covered pixels", file=sys.stderr)


if __name__ == "__main__":
    main()
