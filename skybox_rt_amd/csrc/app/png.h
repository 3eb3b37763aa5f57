// png.h -- minimal PNG I/O for the rtapp CLI (8-bit RGB/RGBA, non-interlaced).
// The reference uses cocogfx SaveImage/CompareImages (draw3d/main.cpp:386,
// 505-514); cocogfx is not vendored, so this is a small zlib-based stand-in.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace rt {

// Writes an ARGB8888 framebuffer (row 0 = bottom, like the reference's
// negative-pitch SaveImage) as a top-down RGBA PNG.
int SavePngARGB(const std::string& path, const uint32_t* argb, uint32_t width, uint32_t height);

// Reads a PNG into ARGB8888, top-down rows.
int LoadPngARGB(const std::string& path, std::vector<uint32_t>* argb, uint32_t* width,
                uint32_t* height);

// Pixels whose max per-channel difference exceeds `tol` (CompareImages).
int64_t CompareARGB(const uint32_t* a, const uint32_t* b, uint64_t count, int tol);

}  // namespace rt
