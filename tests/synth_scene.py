"""Synthetic .cgltrace scenes for tests that need more triangles than the
reference's scenes hold (the GPU BVH builder's multi-block radix sort).
Same XML layout as the reference's traces (tests/golden/scenes/triangle.
cgltrace: boost_serialization v15); one depth-tested (LESS) drawcall of n
random triangles in clip space, w in [90, 110] like tekkaman's model."""
import gzip
import os

import numpy as np

from conftest import scene_path

_ITEM0 = ('<item class_id="6" tracking_level="0" version="0"><first>{i}</first>'
          '<second class_id="7" tracking_level="0" version="0">'
          '<pos class_id="8" tracking_level="0" version="0"><x>{x:.9e}</x><y>{y:.9e}</y>'
          '<z>{z:.9e}</z><w>{w:.9e}</w></pos><color><r>{r:.9e}</r><g>{g:.9e}</g><b>{b:.9e}</b>'
          '<a>1.000000000e+00</a></color><texcoord class_id="9" tracking_level="0" version="0">'
          '<u>0.000000000e+00</u><v>0.000000000e+00</v></texcoord></second></item>')
_ITEM = ('<item><first>{i}</first><second><pos><x>{x:.9e}</x><y>{y:.9e}</y><z>{z:.9e}</z>'
         '<w>{w:.9e}</w></pos><color><r>{r:.9e}</r><g>{g:.9e}</g><b>{b:.9e}</b>'
         '<a>1.000000000e+00</a></color><texcoord><u>0.000000000e+00</u><v>0.000000000e+00</v>'
         '</texcoord></second></item>')


def make_scene(path: str, n: int, seed: int = 1, size: float = 0.03, w_range=(90.0, 110.0),
               spread: float = 0.8, w_jitter: float = 0.5, degenerate: int = 0) -> str:
    """Writes a gzip'd trace of n triangles to `path` (returned): centres
    uniform in +-spread (NDC), corners +-size around them, w in w_range,
    each corner's w jittered by +-w_jitter (w_jitter > w_range[0] puts some
    corners behind the eye); the first `degenerate` triangles repeat their
    first corner as their last (zero area: the setup's det == 0 exactly)."""
    rng = np.random.default_rng(seed)
    w = rng.uniform(w_range[0], w_range[1], n)
    cx, cy = rng.uniform(-spread, spread, n) * w, rng.uniform(-spread, spread, n) * w
    verts = []
    for k in range(3):
        ox, oy = rng.uniform(-size, size, n) * w, rng.uniform(-size, size, n) * w
        dw = rng.uniform(-w_jitter, w_jitter, n)
        verts.append((cx + ox, cy + oy, (w + dw) * 0.5, w + dw))
    if degenerate:
        verts[2] = tuple(np.concatenate([v0[:degenerate], v2[degenerate:]])
                         for v0, v2 in zip(verts[0], verts[2]))
    col = rng.uniform(0.2, 1.0, (n, 3))
    return _write(path, verts, col)


def make_chain_scene(path: str, n: int, ratio: float = 1.6, base: float = 1e-3) -> str:
    """n small triangles whose x centres grow geometrically (base * ratio^k,
    NDC): every binned-SAH split peels a few off the far end, so the tree is
    about n / 5 levels deep -- deeper than the device build's level budget
    (log2 n + 4) for n = 96."""
    k = np.arange(n, dtype=np.float64)
    w = np.full(n, 100.0)
    cx = base * ratio ** k * w
    verts = [(cx + dx * w, np.full(n, dy) * w, w * 0.5, w) for dx, dy in ((0.0, 0.0), (0.01, 0.0), (0.0, 0.01))]
    return _write(path, verts, np.full((n, 3), 0.5))


def _write(path, verts, col):
    n = len(col)
    items = []
    for t in range(n):
        for k in range(3):
            x, y, z, ww = (float(a[t]) for a in verts[k])
            fmt = _ITEM0 if not items else _ITEM
            items.append(fmt.format(i=3 * t + k, x=x, y=y, z=z, w=ww, r=col[t, 0], g=col[t, 1],
                                    b=col[t, 2]))
    prims = ['<item class_id="11" tracking_level="0" version="0"><i0>0</i0><i1>1</i1><i2>2</i2></item>']
    prims += [f"<item><i0>{3 * t}</i0><i1>{3 * t + 1}</i1><i2>{3 * t + 2}</i2></item>"
              for t in range(1, n)]
    tmpl = open(scene_path("triangle")).read()
    head, rest = tmpl.split('<vertices class_id="5"', 1)
    head = head.replace("<depth_test>0</depth_test>", "<depth_test>1</depth_test>")
    head = head.replace("<depth_func>0</depth_func>", "<depth_func>1</depth_func>")
    head = head.replace("<depth_writemask>0</depth_writemask>", "<depth_writemask>1</depth_writemask>")
    tail = rest.split("</primitives>", 1)[1]
    xml = (head + f'<vertices class_id="5" tracking_level="0" version="0"><count>{3 * n}</count>'
           f'<bucket_count>{3 * n}</bucket_count><item_version>0</item_version>' + "".join(items) +
           '</vertices><primitives class_id="10" tracking_level="0" version="0">'
           f'<count>{n}</count><item_version>0</item_version>' + "".join(prims) + "</primitives>" + tail)
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with gzip.open(path, "wt") as f:
        f.write(xml)
    return path
