/*
 * vx_tex.h -- C-ABI of the texture regression app (librtapp.so, texapp CLI).
 *
 * The host side of the reference's tests/regression/tex (main.cpp: image
 * load + format conversion, mip chain, TEX DCR setup, vx_start/vx_ready_wait,
 * read-back) on the public vortex.h API, with its kernel (kernel.cpp) as
 * tex_kernel.vxbin.  The texapp executable takes the reference's flags
 * (-i -o -r -s -w -f -g -z -k).  Errors: negative return, message from
 * rt_last_error() (vx_rt.h).
 */
#ifndef VX_TEX_H
#define VX_TEX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rt_tex* rt_tex_h;

typedef struct {
  uint32_t format;     /* VX_TEX_FORMAT_* (-f), default A8R8G8B8 */
  uint32_t filter;     /* -g: 0 point, 1 bilinear, 2 bilinear + lod blend */
  uint32_t wrap;       /* VX_TEX_WRAP_* (-w), both axes */
  float scale;         /* -s: dst = (uint32_t)(src * scale) per side */
  uint32_t num_tasks;  /* 0 = the reference's min(cores x warps x threads, dst_height) */
} rt_tex_params_t;

typedef struct {
  uint32_t dst_width, dst_height, lod, frac, levels, num_tasks;
  uint64_t texture_bytes;      /* the converted mip chain */
  uint64_t pixels;             /* written by the kernel (counter) */
  double kernel_ms;            /* HIP-event time of the last launch */
  uint32_t grid, block;
} rt_tex_stats_t;

/* tex/main.cpp:173-183 (cocogfx LoadImage + GenerateMipmaps): the A8R8G8B8
 * image (top-down rows) converted to `format` with its mip chain.  out NULL
 * = size query (*size); mipoff[16] byte offsets (0 past the chain). */
int rt_tex_build_image(const uint32_t* argb, uint32_t width, uint32_t height, uint32_t format,
                       uint8_t* out, uint64_t* size, uint32_t mipoff[16], uint32_t* levels);

/* kernel_dir: directory holding tex_kernel_f{0,1,2}.vxbin (NULL = next to librtapp.so) */
int rt_tex_create(const char* kernel_dir, rt_tex_h* out);
int rt_tex_free(rt_tex_h t);
/* source: A8R8G8B8, power-of-two sides, rows top-down */
int rt_tex_configure(rt_tex_h t, const uint32_t* argb, uint32_t width, uint32_t height,
                     const rt_tex_params_t* p);
int rt_tex_render(rt_tex_h t);                         /* vx_start + vx_ready_wait */
int rt_tex_stats(rt_tex_h t, rt_tex_stats_t* st);
/* dst_width x dst_height ARGB8888, row 0 = top (main.cpp saves with +pitch) */
int rt_tex_read(rt_tex_h t, uint32_t* out, uint64_t count);

#ifdef __cplusplus
}
#endif

#endif /* VX_TEX_H */
