// tex_common.h -- kernel argument of the texture regression app's kernel
// (tex_kernel.hip), shared by the host (app/tex_app.cpp).  The reference
// passes the same information as kernel_arg_t + the TEX DCRs
// (tests/regression/tex/common.h:14-24, main.cpp:233-246) and derives
// lod/frac and the per-pixel coordinates in kernel.cpp:63-128; here the host
// replays those float steps once per column/row (utab/vtab) so the kernel is
// pure integer sampling.
#pragma once

#include <stdint.h>

#define TEX_BLOCK_THREADS 256
// Work decomposition: a row is cut into groups of 64 * TEX_PPT(filter)
// pixels; a group is 64 consecutive tasks (one wave chunk), and task `lane`
// of a group owns the group's pixels lane, lane + 64, lane + 128, ... -- so
// every load and store instruction of a wave covers 64 consecutive pixels
// (coalesced), and a lane has TEX_PPT independent samples in flight
#define TEX_PPT(filter) ((filter) == 0 ? 8u : 4u)
#define TEX_GROUP(filter) (64u * TEX_PPT(filter))

typedef struct {
  uint64_t dst_addr;     // ARGB8888 dst_width x dst_height, row 0 = top, pitch dst_width*4
  uint64_t utab_addr;    // int32 TFixed<23> u per column (padded to whole groups)
  uint64_t vtab_addr;    // int32 TFixed<23> v per row
  uint64_t tex_addr;     // the texture's mip chain (VX_DCR_TEX_ADDR << 6)
  uint32_t dst_width, dst_height;
  uint32_t filter;       // tex/main.cpp -g: 0 point, 1 bilinear, 2 bilinear + lod blend
  uint32_t lod, frac;    // kernel.cpp:111-118
  uint32_t logw, logh;   // VX_DCR_TEX_LOGDIM
  uint32_t format;       // VX_DCR_TEX_FORMAT
  uint32_t wrap;         // VX_DCR_TEX_WRAP (same for u and v, main.cpp:236)
  uint32_t num_tasks;    // dst_height * groups per row * 64
  uint32_t mipoff[16];   // VX_DCR_TEX_MIPOFF(0..15), bytes from tex_addr
} tex_kernel_arg_t;

// counter slots (vx_mpm rows) written by the kernel
#define TEX_MPM_USER 3   // = RT_MPM_USER: vx_mpm_query(VX_CSR_MPM_BASE + 3 + slot)
#define TEX_STAT_PIXELS 0
#define TEX_STAT_TEXEL_FETCHES 1
