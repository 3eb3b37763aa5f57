"""CPU tests of the path-trace oracle (BASELINE
config 4).  No reference implementation exists for this row (SURVEY.md
section 0.1: parity unpinned); these tests pin the oracle's own invariants:
BVH traversal == brute force, thread-count invariance, agreement with the
primary+shadow render wherever no path starts, the bounce/shadow ray
bookkeeping, and a committed digest of its output (tests/golden/pt/, made by
tests/golden/pt/make_pt_digests.py) so the oracle cannot drift silently."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, scene_path

os.environ.setdefault("SKYBOX_RT_NO_TORCH", "1")

from skybox_rt_amd import rt  # noqa: E402


@pytest.fixture(scope="module")
def scenes(oracle_lib):
    po = oracle_lib
    out = {}
    for name in ("tekkaman", "box", "scene"):
        s = rt.Scene.load(scene_path(name))
        out[name] = (po.OracleScene(po.cgltrace.load(scene_path(name))), s.bvh())
    return out


@pytest.mark.parametrize("name,size", [("tekkaman", 96), ("box", 64), ("scene", 64)])
def test_pt_bvh_equals_bruteforce(oracle_lib, scenes, name, size):
    po = oracle_lib
    osc, bvh = scenes[name]
    p = po.rt_params(size, size, path=True, nthreads=8)
    cb, pb, _, kb = po.rt_render(osc, p)
    cv, pv, _, kv = po.rt_render(osc, p, bvh=bvh)
    assert np.array_equal(cb, cv) and np.array_equal(pb, pv)
    for key in ("primary_rays", "shadow_rays", "geometry_hits", "occluded", "bounce_rays",
                "shaded", "texel_bytes"):
        assert kb[key] == kv[key], key


def test_pt_thread_invariance(oracle_lib, scenes):
    po = oracle_lib
    osc, bvh = scenes["tekkaman"]
    a = po.rt_render(osc, po.rt_params(128, 128, path=True, nthreads=1), bvh=bvh)
    b = po.rt_render(osc, po.rt_params(128, 128, path=True, nthreads=7), bvh=bvh)
    assert np.array_equal(a[0], b[0]) and a[3] == b[3]


@pytest.mark.parametrize("bounces", (0, 1, 4))
def test_pt_bookkeeping(oracle_lib, scenes, bounces):
    po = oracle_lib
    osc, bvh = scenes["tekkaman"]
    c, pid, _, k = po.rt_render(osc, po.rt_params(128, 128, path=True, bounces=bounces,
                                                  nthreads=8), bvh=bvh)
    ref, rpid, _, rk = po.rt_render(osc, po.rt_params(128, 128, shadows=False, nthreads=8), bvh=bvh)
    assert np.array_equal(pid, rpid)                       # same primary visibility
    hit = k["geometry_hits"]
    assert hit == rk["geometry_hits"] > 0
    # one shadow ray per path vertex: primary hits + surviving bounce hits
    assert k["shadow_rays"] >= hit
    assert k["bounce_rays"] <= bounces * hit
    if bounces == 0:
        assert k["bounce_rays"] == 0 and k["shadow_rays"] == hit
    else:
        assert k["bounce_rays"] >= hit                     # every path bounces once
        assert k["shadow_rays"] - hit <= k["bounce_rays"]
    # pixels where no path starts keep the primary render's colour; path
    # pixels keep its alpha
    assert not np.any((c != ref) & ~_geometry_mask(osc, rpid))
    assert np.array_equal(c >> 24, ref >> 24)


def _geometry_mask(osc, pid):
    geom = np.zeros(max(osc.scene.num_prims, 1), bool)
    for dc in osc.scene.drawcalls:
        if dc.states["depth_test"]:
            geom[dc.prim_offset:dc.prim_offset + dc.prim_count] = True
    return (pid >= 0) & geom[np.maximum(pid, 0)]


def test_pt_seed_changes_only_bounced_light(oracle_lib, scenes):
    po = oracle_lib
    osc, bvh = scenes["tekkaman"]
    a, _, _, ka = po.rt_render(osc, po.rt_params(96, 96, path=True, nthreads=8), bvh=bvh)
    b, _, _, kb = po.rt_render(osc, po.rt_params(96, 96, path=True, seed=1234, nthreads=8), bvh=bvh)
    assert ka["geometry_hits"] == kb["geometry_hits"]
    assert not np.array_equal(a, b)
    z, _, _, _ = po.rt_render(osc, po.rt_params(96, 96, path=True, bounces=0, nthreads=8), bvh=bvh)
    z2, _, _, _ = po.rt_render(osc, po.rt_params(96, 96, path=True, bounces=0, seed=1234,
                                                 nthreads=8), bvh=bvh)
    assert np.array_equal(z, z2)                           # direct light is seed independent


def test_pt_oracle_digest(oracle_lib, scenes):
    po = oracle_lib
    with open(os.path.join(GOLDEN, "pt", "pt_digests.json")) as fh:
        want = json.load(fh)
    for case in want:
        osc, bvh = scenes[case["scene"]]
        c, _, _, k = po.rt_render(osc, po.rt_params(case["size"], case["size"], path=True,
                                                    bounces=case["bounces"], seed=case["seed"],
                                                    nthreads=8), bvh=bvh)
        assert hashlib.sha256(np.ascontiguousarray(c).tobytes()).hexdigest() == case["sha256"]
        assert {key: k[key] for key in case["counters"]} == case["counters"]
