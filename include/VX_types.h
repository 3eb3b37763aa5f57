/*
 * VX_types.h -- device configuration register map and graphics constants.
 *
 * The numbering is the reference's (hw/rtl/VX_types.vh:22-28, 304-458, which
 * hw/scripts/gen_config.py turns into a C header there); it is restated here
 * because apps write these DCR addresses directly (draw3d/main.cpp:216-331).
 * Used by host code and by HIP kernel programs.
 */
#ifndef VX_TYPES_H
#define VX_TYPES_H

/* ---- base DCRs ---- */
#define VX_DCR_BASE_STARTUP_ADDR0 0x001
#define VX_DCR_BASE_STARTUP_ADDR1 0x002
#define VX_DCR_BASE_STARTUP_ARG0  0x003
#define VX_DCR_BASE_STARTUP_ARG1  0x004
#define VX_DCR_BASE_MPM_CLASS     0x005
#define VX_DCR_BASE_STATE_END     0x006

#define VX_DCR_MPM_CLASS_NONE   0
#define VX_DCR_MPM_CLASS_CORE   1
#define VX_DCR_MPM_CLASS_MEM    2
#define VX_DCR_MPM_CLASS_TEX    3
#define VX_DCR_MPM_CLASS_RASTER 4
#define VX_DCR_MPM_CLASS_OM     5

/* ---- texture unit ---- */
#define VX_TEX_STAGE_COUNT    2
#define VX_TEX_SUBPIXEL_BITS  8
#define VX_TEX_DIM_BITS       15
#define VX_TEX_LOD_MAX        VX_TEX_DIM_BITS
#define VX_TEX_FXD_FRAC       (VX_TEX_DIM_BITS + VX_TEX_SUBPIXEL_BITS) /* 23 */
#define VX_TEX_FILTER_POINT    0
#define VX_TEX_FILTER_BILINEAR 1
#define VX_TEX_WRAP_CLAMP  0
#define VX_TEX_WRAP_REPEAT 1
#define VX_TEX_WRAP_MIRROR 2
#define VX_TEX_FORMAT_A8R8G8B8 0
#define VX_TEX_FORMAT_R5G6B5   1
#define VX_TEX_FORMAT_A1R5G5B5 2
#define VX_TEX_FORMAT_A4R4G4B4 3
#define VX_TEX_FORMAT_A8L8     4
#define VX_TEX_FORMAT_L8       5
#define VX_TEX_FORMAT_A8       6

#define VX_DCR_TEX_STATE_BEGIN VX_DCR_BASE_STATE_END          /* 0x006 */
#define VX_DCR_TEX_STAGE       (VX_DCR_TEX_STATE_BEGIN + 0)
#define VX_DCR_TEX_ADDR        (VX_DCR_TEX_STATE_BEGIN + 1)
#define VX_DCR_TEX_LOGDIM      (VX_DCR_TEX_STATE_BEGIN + 2)
#define VX_DCR_TEX_FORMAT      (VX_DCR_TEX_STATE_BEGIN + 3)
#define VX_DCR_TEX_FILTER      (VX_DCR_TEX_STATE_BEGIN + 4)
#define VX_DCR_TEX_WRAP        (VX_DCR_TEX_STATE_BEGIN + 5)
#define VX_DCR_TEX_MIPOFF(lod) (VX_DCR_TEX_STATE_BEGIN + 6 + (lod))
#define VX_DCR_TEX_STATE_END   (VX_DCR_TEX_MIPOFF(VX_TEX_LOD_MAX) + 1) /* 0x01C */

/* ---- raster unit ---- */
#define VX_RASTER_DIM_BITS        15
#define VX_DCR_RASTER_STATE_BEGIN VX_DCR_TEX_STATE_END          /* 0x01C */
#define VX_DCR_RASTER_TBUF_ADDR   (VX_DCR_RASTER_STATE_BEGIN + 0)
#define VX_DCR_RASTER_TILE_COUNT  (VX_DCR_RASTER_STATE_BEGIN + 1)
#define VX_DCR_RASTER_PBUF_ADDR   (VX_DCR_RASTER_STATE_BEGIN + 2)
#define VX_DCR_RASTER_PBUF_STRIDE (VX_DCR_RASTER_STATE_BEGIN + 3)
#define VX_DCR_RASTER_SCISSOR_X   (VX_DCR_RASTER_STATE_BEGIN + 4)
#define VX_DCR_RASTER_SCISSOR_Y   (VX_DCR_RASTER_STATE_BEGIN + 5)
#define VX_DCR_RASTER_STATE_END   (VX_DCR_RASTER_STATE_BEGIN + 6) /* 0x022 */

/* ---- output merger ---- */
#define VX_OM_DEPTH_BITS   24
#define VX_OM_DEPTH_MASK   ((1u << VX_OM_DEPTH_BITS) - 1)
#define VX_OM_STENCIL_BITS 8
#define VX_OM_STENCIL_MASK ((1u << VX_OM_STENCIL_BITS) - 1)
#define VX_OM_DEPTH_FUNC_ALWAYS   0
#define VX_OM_DEPTH_FUNC_NEVER    1
#define VX_OM_DEPTH_FUNC_LESS     2
#define VX_OM_DEPTH_FUNC_LEQUAL   3
#define VX_OM_DEPTH_FUNC_EQUAL    4
#define VX_OM_DEPTH_FUNC_GEQUAL   5
#define VX_OM_DEPTH_FUNC_GREATER  6
#define VX_OM_DEPTH_FUNC_NOTEQUAL 7
#define VX_OM_STENCIL_OP_KEEP      0
#define VX_OM_STENCIL_OP_ZERO      1
#define VX_OM_STENCIL_OP_REPLACE   2
#define VX_OM_STENCIL_OP_INCR      3
#define VX_OM_STENCIL_OP_DECR      4
#define VX_OM_STENCIL_OP_INVERT    5
#define VX_OM_STENCIL_OP_INCR_WRAP 6
#define VX_OM_STENCIL_OP_DECR_WRAP 7
#define VX_OM_BLEND_MODE_ADD     0
#define VX_OM_BLEND_MODE_SUB     1
#define VX_OM_BLEND_MODE_REV_SUB 2
#define VX_OM_BLEND_MODE_MIN     3
#define VX_OM_BLEND_MODE_MAX     4
#define VX_OM_BLEND_MODE_LOGICOP 5
#define VX_OM_BLEND_FUNC_ZERO                0
#define VX_OM_BLEND_FUNC_ONE                 1
#define VX_OM_BLEND_FUNC_SRC_RGB             2
#define VX_OM_BLEND_FUNC_ONE_MINUS_SRC_RGB   3
#define VX_OM_BLEND_FUNC_DST_RGB             4
#define VX_OM_BLEND_FUNC_ONE_MINUS_DST_RGB   5
#define VX_OM_BLEND_FUNC_SRC_A               6
#define VX_OM_BLEND_FUNC_ONE_MINUS_SRC_A     7
#define VX_OM_BLEND_FUNC_DST_A               8
#define VX_OM_BLEND_FUNC_ONE_MINUS_DST_A     9
#define VX_OM_BLEND_FUNC_CONST_RGB           10
#define VX_OM_BLEND_FUNC_ONE_MINUS_CONST_RGB 11
#define VX_OM_BLEND_FUNC_CONST_A             12
#define VX_OM_BLEND_FUNC_ONE_MINUS_CONST_A   13
#define VX_OM_BLEND_FUNC_ALPHA_SAT           14

#define VX_DCR_OM_STATE_BEGIN       VX_DCR_RASTER_STATE_END       /* 0x022 */
#define VX_DCR_OM_CBUF_ADDR         (VX_DCR_OM_STATE_BEGIN + 0)
#define VX_DCR_OM_CBUF_PITCH        (VX_DCR_OM_STATE_BEGIN + 1)
#define VX_DCR_OM_CBUF_WRITEMASK    (VX_DCR_OM_STATE_BEGIN + 2)
#define VX_DCR_OM_ZBUF_ADDR         (VX_DCR_OM_STATE_BEGIN + 3)
#define VX_DCR_OM_ZBUF_PITCH        (VX_DCR_OM_STATE_BEGIN + 4)
#define VX_DCR_OM_DEPTH_FUNC        (VX_DCR_OM_STATE_BEGIN + 5)
#define VX_DCR_OM_DEPTH_WRITEMASK   (VX_DCR_OM_STATE_BEGIN + 6)
#define VX_DCR_OM_STENCIL_FUNC      (VX_DCR_OM_STATE_BEGIN + 7)
#define VX_DCR_OM_STENCIL_ZPASS     (VX_DCR_OM_STATE_BEGIN + 8)
#define VX_DCR_OM_STENCIL_ZFAIL     (VX_DCR_OM_STATE_BEGIN + 9)
#define VX_DCR_OM_STENCIL_FAIL      (VX_DCR_OM_STATE_BEGIN + 10)
#define VX_DCR_OM_STENCIL_REF       (VX_DCR_OM_STATE_BEGIN + 11)
#define VX_DCR_OM_STENCIL_MASK      (VX_DCR_OM_STATE_BEGIN + 12)
#define VX_DCR_OM_STENCIL_WRITEMASK (VX_DCR_OM_STATE_BEGIN + 13)
#define VX_DCR_OM_BLEND_MODE        (VX_DCR_OM_STATE_BEGIN + 14)
#define VX_DCR_OM_BLEND_FUNC        (VX_DCR_OM_STATE_BEGIN + 15)
#define VX_DCR_OM_BLEND_CONST       (VX_DCR_OM_STATE_BEGIN + 16)
#define VX_DCR_OM_LOGIC_OP          (VX_DCR_OM_STATE_BEGIN + 17)
#define VX_DCR_OM_STATE_END         (VX_DCR_OM_STATE_BEGIN + 18)  /* 0x034 */

/* DCR mirror size shipped to every launch (covers 0x000..0x03F) */
#define VX_DCR_MIRROR_SIZE 64
/* HIP-driver word of the device DCR mirror (beyond the reference's DCRs):
 * nonzero = kernels write their per-block counter rows (vx_spawn.h) */
#define VX_DCR_HIP_MPM_ROWS 0x03F

/* ---- performance counters (VX_types.vh:71-77) ---- */
#define VX_CSR_MPM_BASE  0xB00
#define VX_CSR_MCYCLE    0xB00
#define VX_CSR_MINSTRET  0xB02
#define VX_MPM_COUNT     32

/* ---- memory map (VX_config.vh:166-189) ---- */
#define STARTUP_ADDR   0x080000000ull
#define USER_BASE_ADDR 0x000010000ull

/* ---- raster tiling (VX_config.vh:477-484) ---- */
#define RASTER_TILE_LOGSIZE  5
#define RASTER_BLOCK_LOGSIZE 2

#endif /* VX_TYPES_H */
