// setup.h -- host-side scene preparation for the RT kernel.
//
//  * PrimSetup: the per-primitive part of graphics::Binning
//    (sim/common/gfxutil.cpp:131-251): clip -> 2D-homogeneous device
//    coordinates, edge equations, half-pixel offset, Q15.16 edges, Q7.24
//    attribute deltas -> rt_prim_t (the fixed-point shading record).
//  * DrawcallState: the draw3d host state setup (draw3d/main.cpp:286-344)
//    reduced to what shading needs -> rt_dcstate_t.
//  * cocogfx CGLTrace enum mapping (inferred; pinned by the golden images
//    through the oracle, see oracle/gfx.h).
#pragma once

#include <cstdint>

#include "VX_types.h"
#include "../kernels/rt_common.h"
#include "cgltrace.h"

namespace rt {

// CGLTrace -> VX enum mapping (gfxutil.cpp:280-346 case order)
uint32_t ToVXCompare(int32_t cgl_compare);
int32_t ToVXFormat(int32_t cgl_format);
uint32_t FormatStride(int32_t vx_format);

constexpr int32_t kCglFilterNearest = 1;
constexpr int32_t kCglAddressWrap = 0;
constexpr int32_t kCglEnvModeModulate = 3;

enum SetupStatus { kSetupOk = 0, kSetupDegenerate = 1, kSetupCulled = 2 };

// Fills `out` (edges/attribs) for one triangle at width x height.
int PrimSetup(const std::array<Vertex, 3>& v, uint32_t width, uint32_t height, float znear,
              float zfar, rt_prim_t* out);

// Shading state of a drawcall (texture address filled by the caller).
rt_dcstate_t DrawcallState(const DrawCall& dc, const Scene& scene);

// Screen bounding box of a triangle at width x height (gfxutil.cpp:168-192);
// returns kSetupCulled (and an empty box) when it misses the viewport.
int PrimBBox(const std::array<Vertex, 3>& v, uint32_t width, uint32_t height, rt_bbox_t* out);

// Output-merger state of a drawcall (raster pipeline).
rt_omstate_t OmState(const DrawCall& dc);

}  // namespace rt
