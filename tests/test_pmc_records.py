"""The committed rocprofv3 PMC records (profiles/pmc_<mode>.json, written by
scripts/pmc_profile.sh on the GPU box) must describe the kernel images this
tree builds: bench.py reports roofline.traffic and the issue roofline from
them only when the image MD5 matches, so a stale record would silently drop
the measured numbers.  CPU test: hashes the built images, no GPU."""
import hashlib
import json
import os

import pytest

from skybox_rt_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
IMAGES = {"shadow": ("rt_kernel.co",), "path": ("pt_kernel.co",),
          "flat": ("rt_flat.co",), "bvh": ("rt_bvh.co",)}


@pytest.mark.parametrize("mode", sorted(IMAGES))
def test_pmc_record_matches_built_image(mode):
    if _lib.missing():
        _lib.build()
    rec_path = os.path.join(ROOT, "profiles", f"pmc_{mode}.json")
    assert os.path.exists(rec_path), f"no PMC record for {mode}: run scripts/pmc_profile.sh"
    rec = json.load(open(rec_path))
    h = hashlib.md5()  # the frame's images concatenated (scripts/pmc_profile.py)
    for co in IMAGES[mode]:
        h.update(open(os.path.join(_lib.LIB_DIR, co), "rb").read())
    md5 = h.hexdigest()
    assert rec["kernel_md5"] == md5, (
        f"profiles/pmc_{mode}.json was taken on another {IMAGES[mode]} "
        f"({rec['kernel_md5']} != {md5}): regenerate it with scripts/pmc_profile.sh")
    assert rec["traffic_bytes"] > 0 and rec["sq"].get("SQ_INSTS_VALU", 0) > 0
    assert rec["width"] == rec["height"] == (256 if mode == "flat" else 1024)
