"""Independent `.cgltrace` reader -- TEST INFRASTRUCTURE (oracle side).

This module is part of the oracle: only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import it. The product parses scenes with its
own C++ reader (skybox_rt_amd/csrc/app/cgltrace.cpp); tests cross-check the two.

Format (restated from the reference's scene input, a boost_serialization XML
archive, version 15 -- see tests/regression/draw3d/triangle.cgltrace:1-136):

  cgltrace/drawcalls/item*
      states/{color_enabled, color_writemask, depth_test, depth_writemask,
              depth_func, stencil_*, texture_enabled, texture_envmode,
              texture_minfilter, texture_magfilter, texture_addressU/V,
              blend_enabled, blend_src, blend_dst, ...}
      texture_id
      vertices  = unordered_map<id, {pos{x,y,z,w}, color{r,g,b,a}, texcoord{u,v}}>
      primitives = vector<{i0,i1,i2}>      (ids into `vertices`)
      viewport{left,right,top,bottom,near,far}
  cgltrace/textures = unordered_map<id, {format,width,height,size,pixels(base64)}>

The reference loads this with cocogfx `CGLTrace::load` (draw3d/main.cpp:428-430;
cocogfx is an un-vendored submodule, .gitmodules:10-12).

The flattened form below is the interchange format the oracle C code consumes:
  prim_verts  float32[P, 3, 10]  (x,y,z,w, r,g,b,a, u,v) per primitive corner
  drawcalls   list of dicts (prim_offset, prim_count, states..., near, far)
  textures    dict id -> (format, width, height, bytes)
"""
from __future__ import annotations

import base64
import gzip
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field

import numpy as np

STATE_KEYS = (
    "color_enabled", "color_format", "color_writemask", "depth_test",
    "depth_writemask", "depth_format", "depth_func", "stencil_test",
    "stencil_func", "stencil_zpass", "stencil_zfail", "stencil_fail",
    "stencil_ref", "stencil_mask", "stencil_writemask", "texture_enabled",
    "texture_envmode", "texture_minfilter", "texture_magfilter",
    "texture_addressU", "texture_addressV", "blend_enabled", "blend_src",
    "blend_dst",
)


@dataclass
class DrawCall:
    states: dict
    texture_id: int
    prim_offset: int
    prim_count: int
    viewport: dict


@dataclass
class Scene:
    drawcalls: list = field(default_factory=list)
    prim_verts: np.ndarray = None          # float32 [P,3,10]
    textures: dict = field(default_factory=dict)  # id -> (fmt, w, h, bytes)

    @property
    def num_prims(self) -> int:
        return 0 if self.prim_verts is None else int(self.prim_verts.shape[0])


def _f32(text: str) -> np.float32:
    # decimal -> nearest float32 (same as strtof), via float64 then exact-round
    return np.float32(float(text))


def _vertex(el) -> np.ndarray:
    pos, col, tc = el.find("pos"), el.find("color"), el.find("texcoord")
    vals = [pos.find(k).text for k in "xyzw"]
    vals += [col.find(k).text for k in "rgba"]
    vals += [tc.find(k).text for k in "uv"]
    return np.array([_f32(v) for v in vals], dtype=np.float32)


def load(path: str) -> Scene:
    opener = gzip.open if str(path).endswith(".gz") else open
    with opener(path, "rb") as f:
        root = ET.parse(f).getroot()
    cgl = root.find("cgltrace")
    scene = Scene()
    all_prims = []
    for item in cgl.find("drawcalls").findall("item"):
        st = item.find("states")
        states = {}
        for k in STATE_KEYS:
            e = st.find(k)
            states[k] = int(e.text) if e is not None else 0
        verts = {}
        for vi in item.find("vertices").findall("item"):
            verts[int(vi.find("first").text)] = _vertex(vi.find("second"))
        prims = []
        for pi in item.find("primitives").findall("item"):
            ids = [int(pi.find(k).text) for k in ("i0", "i1", "i2")]
            prims.append(np.stack([verts[i] for i in ids]))
        vp = item.find("viewport")
        viewport = {k: float(_f32(vp.find(k).text)) for k in
                    ("left", "right", "top", "bottom", "near", "far")}
        scene.drawcalls.append(DrawCall(
            states=states,
            texture_id=int(item.find("texture_id").text),
            prim_offset=len(all_prims), prim_count=len(prims),
            viewport=viewport))
        all_prims.extend(prims)
    scene.prim_verts = (np.stack(all_prims).astype(np.float32) if all_prims
                        else np.zeros((0, 3, 10), np.float32))
    tex = cgl.find("textures")
    if tex is not None:
        for ti in tex.findall("item"):
            tid = int(ti.find("first").text)
            s = ti.find("second")
            fmt = int(s.find("format").text)
            w = int(s.find("width").text)
            h = int(s.find("height").text)
            data = base64.b64decode("".join(s.find("pixels").text.split()))
            size = int(s.find("size").text)
            assert len(data) == size, (len(data), size)
            scene.textures[tid] = (fmt, w, h, data)
    return scene


def select_drawcalls(scene: Scene, keep) -> Scene:
    """The scene with only drawcalls `keep` (ascending indices), in order:
    draw3d's -s / -e draw range (tests/regression/draw3d/main.cpp:179-181)."""
    out = Scene(textures=scene.textures)
    verts = []
    for d in keep:
        dc = scene.drawcalls[d]
        verts.append(scene.prim_verts[dc.prim_offset:dc.prim_offset + dc.prim_count])
        out.drawcalls.append(DrawCall(dc.states, dc.texture_id, sum(len(v) for v in verts[:-1]),
                                      dc.prim_count, dc.viewport))
    out.prim_verts = (np.concatenate(verts).astype(np.float32) if verts
                      else np.zeros((0, 3, 10), np.float32))
    return out
