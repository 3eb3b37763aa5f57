"""Pin the oracle's restatement of the render-output regression app
(tests/regression/om: main.cpp:130-300 host state, kernel.cpp:16-40, the OM
unit sim/simx/om_unit.cpp:28-160) against the reference's own goldens
om/whitebox_{8..128}.png (copied as data to tests/golden/om/; the CI runs the
app with default flags, ci/regression.sh.in:165-174), plus the properties the
other flags imply (the goldens cover only the default state)."""
import numpy as np
import pytest

from conftest import GOLDEN

SIZES = (8, 16, 32, 64, 128)


@pytest.mark.parametrize("size", SIZES)
def test_om_oracle_matches_whitebox_golden(oracle_lib, size):
    po = oracle_lib
    fb = po.om_app(size, size)
    ref = po.load_png_argb(f"{GOLDEN}/om/whitebox_{size}.png")
    assert np.array_equal(fb[::-1], ref)      # the app saves row 0 = bottom flipped


def test_om_oracle_depth_test_is_the_checkerboard(oracle_lib):
    # -d: LESS against the 0.0 / 0.99 checkerboard: 0.5 < 0.99 passes off the
    # equal-parity diagonal only; colour stays at the clear (0) elsewhere
    fb = oracle_lib.om_app(32, 32, depth_enable=True)
    y, x = np.mgrid[0:32, 0:32]
    assert np.array_equal(fb, np.where((x & 1) == (y & 1), 0, 0xFFFFFFFF).astype(np.uint32))


def test_om_oracle_blend_alpha_ramp(oracle_lib):
    # -b: ONE / ONE_MINUS_SRC_A over a 0 buffer = the source; alpha = task x
    # 255 / rows_per_task, tasks of ceil(H / num_tasks) rows (kernel.cpp:17-23)
    fb = oracle_lib.om_app(16, 16, num_tasks=4, blend=True)
    alphas = [int(t * np.float32(255.0 / 4)) & 0xFF for t in range(4)]
    assert [int(v >> 24) for v in fb[::4, 0]] == alphas
    assert np.all((fb & 0xFFFFFF) == 0xFFFFFF)
    # the MI355X task count: one row per task, alpha = (task * 255) mod 256
    fb = oracle_lib.om_app(8, 8, blend=True)
    assert [int(v >> 24) for v in fb[:, 0]] == [(t * 255) & 0xFF for t in range(8)]


def test_om_oracle_colour_and_face(oracle_lib):
    fb = oracle_lib.om_app(8, 8, color=12345)
    assert np.all(fb == (0xFF000000 | 12345))
    # stencil is ALWAYS/KEEP on both faces, so -f changes nothing
    assert np.array_equal(oracle_lib.om_app(8, 8, backface=True), oracle_lib.om_app(8, 8))
