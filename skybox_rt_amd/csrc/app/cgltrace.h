// cgltrace.h -- .cgltrace scene reader (the north star's scene input).
//
// The reference loads scenes with cocogfx CGLTrace::load (draw3d/main.cpp:
// 428-430), a boost_serialization XML archive (v15) whose layout is visible in
// tests/regression/draw3d/triangle.cgltrace:1-136.  cocogfx is an un-vendored
// submodule (.gitmodules:10-12) and boost is absent here, so this is a
// self-contained reader for exactly that archive layout (plain or gzip).
#pragma once

#include <array>
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace rt {

struct Vertex {
  float pos[4];    // clip-space x, y, z, w
  float color[4];  // r, g, b, a
  float uv[2];
};

struct States {   // CGLTrace::states_t (field order of the archive)
  int32_t color_enabled = 0, color_format = 0;
  uint32_t color_writemask = 0xffffffffu;
  int32_t depth_test = 0, depth_writemask = 0, depth_format = 0, depth_func = 0;
  int32_t stencil_test = 0, stencil_func = 0, stencil_zpass = 0, stencil_zfail = 0;
  int32_t stencil_fail = 0, stencil_ref = 0, stencil_mask = 0, stencil_writemask = 0;
  int32_t texture_enabled = 0, texture_envmode = 0, texture_minfilter = 0;
  int32_t texture_magfilter = 0, texture_addressU = 0, texture_addressV = 0;
  int32_t blend_enabled = 0, blend_src = 0, blend_dst = 0;
};

struct DrawCall {
  States states;
  int32_t texture_id = 0;
  uint32_t prim_offset = 0, prim_count = 0;  // into Scene::prims
  float viewport[6] = {0, 0, 0, 0, 0, 1};    // left, right, top, bottom, near, far
};

struct Texture {
  int32_t format = 0, width = 0, height = 0;
  std::vector<uint8_t> pixels;
};

struct Scene {
  std::vector<DrawCall> drawcalls;
  std::vector<std::array<Vertex, 3>> prims;  // all drawcalls' triangles, in order
  std::map<int32_t, Texture> textures;
};

// Returns 0 on success; on failure returns -1 and sets *error.
int LoadCGLTrace(const std::string& path, Scene* scene, std::string* error);

}  // namespace rt
