"""GPU parity of the texture regression app (tex_kernel.hip behind
include/vx_tex.h): every invocation of the
reference's CI (ci/regression.sh.in:131-156) against its golden images, and
scaled renders (magnification, minification with lod/trilinear blend, all
formats and wrap modes) bit-exact against the oracle (oracle/tex.c)."""
import os
import subprocess

import numpy as np
import pytest
from PIL import Image

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

from skybox_rt_amd import _lib, tex  # noqa: E402

TEX = f"{GOLDEN}/tex"
_app = {}


def app():
    if "a" not in _app:
        _app["a"] = tex.TexApp()
    return _app["a"]


CASES = ([("toad", f, 0, f"toad_ref_f{f}") for f in range(7)] +
         [(n, 0, g, f"{n}_ref_g{g}") for n in ("soccer", "palette4", "palette16", "palette64")
          for g in range(3)])


@pytest.mark.parametrize("name,fmt,filt,ref", CASES)
def test_tex_kernel_matches_reference_goldens(oracle_lib, name, fmt, filt, ref):
    po = oracle_lib
    a = app()
    a.configure(po.load_png_argb(f"{TEX}/{name}.png"), fmt=fmt, filt=filt)
    a.render()
    golden = np.array(Image.open(f"{TEX}/{ref}.png").convert("RGBA"))
    assert po.compare_images(po.argb_to_rgba_topdown(a.image()), golden, tol=0) == 0
    st = a.stats()
    assert st["pixels"] == golden.shape[0] * golden.shape[1]


SCALED = [("toad", 0, 1, 0, 1.37), ("toad", 1, 2, 1, 0.5), ("toad", 3, 1, 2, 2.0),
          ("rainbow", 0, 2, 0, 0.3), ("rainbow", 1, 2, 1, 0.77), ("rainbow", 5, 0, 2, 1.9),
          ("soccer", 2, 1, 1, 3.3), ("soccer", 4, 2, 2, 0.45), ("palette64", 6, 1, 0, 5.01),
          ("palette4", 0, 1, 1, 33.0), ("rainbow", 0, 2, 2, 16.0), ("rainbow", 1, 2, 0, 0.01)]


@pytest.mark.parametrize("name,fmt,filt,wrap,scale", SCALED)
def test_tex_kernel_scaled_bit_exact_vs_oracle(oracle_lib, name, fmt, filt, wrap, scale):
    po = oracle_lib
    src = po.load_png_argb(f"{TEX}/{name}.png")
    a = app()
    a.configure(src, fmt=fmt, filt=filt, wrap=wrap, scale=scale)
    a.render()
    st = a.stats()
    ref = po.tex_render(src, fmt=fmt, wrap=wrap, filt=filt, scale=scale,
                        num_tasks=st["num_tasks"])
    assert ref.shape == (st["dst_height"], st["dst_width"])
    got = a.image()
    assert np.array_equal(got, ref), f"{int((got != ref).sum())} pixels differ"
    assert (st["lod"], st["frac"]) == po.tex_lod(int(src.shape[1]).bit_length() - 1,
                                                 int(src.shape[0]).bit_length() - 1,
                                                 st["dst_width"], st["dst_height"])


def test_tex_kernel_task_partition_matches_oracle(oracle_lib):
    """Fewer tasks than rows: each task walks tile_height rows accumulating
    fv (kernel.cpp:79-127) -- the per-row coordinates depend on the
    partition on non-dyadic sizes, and the kernel replays it exactly."""
    po = oracle_lib
    src = po.load_png_argb(f"{TEX}/rainbow.png")
    a = app()
    for nt in (1, 7, 64):
        a.configure(src, fmt=0, filt=1, scale=0.77, num_tasks=nt)
        a.render()
        ref = po.tex_render(src, fmt=0, filt=1, scale=0.77, num_tasks=nt)
        assert np.array_equal(a.image(), ref), nt


def test_texapp_cli_against_golden(tmp_path):
    exe = os.path.join(_lib.LIB_DIR, "texapp")
    for args in (["-i", f"{TEX}/toad.png", "-r", f"{TEX}/toad_ref_f1.png", "-f1", "-g0"],
                 ["-i", f"{TEX}/soccer.png", "-r", f"{TEX}/soccer_ref_g2.png", "-g2"]):
        out = subprocess.run([exe, "-o", str(tmp_path / "out.png")] + args, capture_output=True,
                             text=True, timeout=300)
        assert out.returncode == 0, out.stdout + out.stderr
        assert "PASSED!" in out.stdout
