// vis.h -- per-resolution primary-visibility records (rt_vtri_t, rt_vnode_t;
// see kernels/rt_common.h): what makes the RT kernels' primary rays
// raster-exact.
//
// Coverage is draw3d's: a pixel (x, y) is covered by a primitive iff its
// three Q15.16 edge values (a*x + b*y + c, int32 wrap; graphics.cpp:640-642)
// are all >= 0 (inclusive, no top-left rule, graphics.cpp:813-825) and the
// pixel lies in a 32x32 tile the primitive's screen box was binned to
// (gfxutil.cpp:237-271; pixels outside the viewport are never covered).
// VisPrim is that set's exact bounding rectangle, computed row by row with
// exact integer arithmetic (a row whose edge values could wrap int32 is
// scanned pixel by pixel), plus a lower bound of the primitive's masked
// 24-bit depth word over its covered pixels (the draw3d shader's z
// interpolation, draw3d/kernel.cpp:37-59, as bounded in vis.cpp).
// NO REFERENCE for the records themselves (the reference rasterizes); the
// oracle restates them by brute force (oracle/vis.c) and the GPU tests check
// the frames against the pinned raster restatement and the golden images.
#pragma once

#include <array>
#include <cstdint>
#include <vector>

#include "../kernels/rt_common.h"

namespace rt {

struct VisPrim {
  uint32_t rx = RT_VIS_EMPTY_RECT, ry = RT_VIS_EMPTY_RECT;  // inclusive pixel rectangle
  uint32_t zmin = RT_VIS_ZMIN_NONE;                          // depth-word lower bound
  bool any = false;                                          // covers at least one pixel
};

// `ok`: the primitive survived setup (not degenerate, screen box not empty);
// bbox: its screen box (PrimBBox) at width x height.
VisPrim ComputeVisPrim(const rt_prim_t& p, bool ok, const rt_bbox_t& bbox, uint32_t width,
                       uint32_t height);

// the 64-B leaf / layer record of primitive `pid`
rt_vtri_t MakeVisTri(const rt_prim_t& p, const VisPrim& v, int32_t pid);

// rt_vnode_t for every node of a tree given by its child references (4 per
// node; a BVH2 uses slots 0-1, RT_EMPTY_REF elsewhere; leaf references
// index `leaf_pids`, the pid of every leaf triangle record in tris order).
// Unreachable node slots are left empty.  Returns 0, -1 on a malformed tree.
int BuildVisNodes(const std::vector<std::array<int32_t, 4>>& refs,
                  const std::vector<int32_t>& leaf_pids, const std::vector<VisPrim>& by_pid,
                  std::vector<rt_vnode_t>* out);

// The primary rays' own tree, per resolution: a 4-wide BVH over the
// geometry primitives' covered-pixel rectangles (binned SAH on screen area,
// optionally with the depth bound as a third axis scaled by depth_scale
// pixels per 2^24; primitives covering no pixel are left out), in the
// layout BuildVisNodes takes.  stack4 = its worst-case traversal stack.
int BuildScreenTree(const std::vector<VisPrim>& by_pid, const std::vector<int32_t>& geometry,
                    float depth_scale, std::vector<std::array<int32_t, 4>>* refs,
                    std::vector<int32_t>* leaf_pids, uint32_t* stack4);

}  // namespace rt
