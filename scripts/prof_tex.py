#!/usr/bin/env python3
"""Runs one texture-app case for profiler passes (rocprofv3 --pmc): `frames`
launches of tex_kernel_f<filter> on a fixed input.  Cases as bench_tex.py."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="bilinear")
    ap.add_argument("--frames", type=int, default=10)
    args = ap.parse_args()
    import torch  # noqa: F401
    from conftest import GOLDEN
    from oracle import py_oracle as po
    from skybox_rt_amd import tex
    if args.case == "point":
        rng = np.random.default_rng(7)
        src = rng.integers(0, 2 ** 32, size=(4096, 4096), dtype=np.uint64).astype(np.uint32)
        cfg = dict(fmt=0, filt=0, wrap=0, scale=1.0)
    elif args.case == "trilinear":
        src = po.load_png_argb(f"{GOLDEN}/tex/rainbow.png")
        cfg = dict(fmt=0, filt=2, wrap=0, scale=16.0)
    else:
        src = po.load_png_argb(f"{GOLDEN}/tex/rainbow.png")
        cfg = dict(fmt=1, filt=1, wrap=2, scale=8.0)
    a = tex.TexApp()
    a.configure(src, **cfg)
    for _ in range(args.frames):
        a.render()
    print(args.case, a.stats())


if __name__ == "__main__":
    main()
