"""GPU tests of the render-output regression app (tests/regression/om) on the
MI355X: `omapp` (app/om_main.cpp, vortex.h only) with the om.vxbin kernel
image, run with the reference CI's flags against the reference goldens
om/whitebox_{8..128}.png, and with every other flag against the oracle's
restatement (oracle/gfx.c orc_om_app) bit for bit."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

from skybox_rt_amd import _lib  # noqa: E402

EXE = os.path.join(_lib.LIB_DIR, "omapp")


def _run(args, tmp_path, name="om.png"):
    out = os.path.join(tmp_path, name)
    p = subprocess.run([EXE, "-o", out] + args, capture_output=True, text=True, timeout=120)
    return p, out


@pytest.mark.parametrize("size", (8, 16, 32, 64, 128))
def test_omapp_whitebox_golden(tmp_path, size):
    # ci/regression.sh.in:165-174 run `--app=om --args="-rwhitebox_128.png"`
    args = [f"-r{GOLDEN}/om/whitebox_{size}.png"]
    if size != 128:
        args += [f"-w{size}", f"-h{size}"]
    p, _ = _run(args, tmp_path)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "PASSED!" in p.stdout


@pytest.mark.parametrize("flags,kw", [
    (["-d"], dict(depth_enable=True)),
    (["-b"], dict(blend=True)),
    (["-f"], dict(backface=True)),
    (["-c", "12345"], dict(color=12345)),
    (["-d", "-b", "-f"], dict(depth_enable=True, blend=True, backface=True)),
    (["-w", "100", "-h", "37", "-d"], dict(depth_enable=True)),
])
def test_omapp_flags_equal_oracle(tmp_path, oracle_lib, flags, kw):
    p, out = _run(flags, tmp_path)
    assert p.returncode == 0, p.stdout + p.stderr
    tasks = int(re.search(r"number of tasks: (\d+)", p.stdout).group(1))
    w = int(flags[flags.index("-w") + 1]) if "-w" in flags else 128
    h = int(flags[flags.index("-h") + 1]) if "-h" in flags else 128
    ref = oracle_lib.om_app(w, h, num_tasks=tasks, **kw)
    img = oracle_lib.load_png_argb(out)
    assert np.array_equal(img[::-1], ref)
