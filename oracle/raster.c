/*
 * raster.c -- oracle restatement of the draw3d software path:
 * graphics::Binning (sim/common/gfxutil.cpp:103-276) + Rasterizer::render
 * (tests/regression/draw3d/gpu_sw.h:34-62, sim/common/graphics.cpp:715-843)
 * + shader_function_sw_rast_cb (draw3d/kernel.cpp:232-279) + OutputMerger.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 */
#include <stdlib.h>
#include <string.h>

#include "gfx.h"

/* coverage != 0: the raster regression app instead of draw3d
 * (tests/regression/raster/kernel.cpp:35-45: every covered pixel of every
 * drawcall written 0xffffffff, no shader, no output-merger state) */
static int raster_render(const orc_scene_t* scene, uint32_t width, uint32_t height,
                         uint32_t tile_logsize, int coverage, uint32_t* color, uint32_t* depth,
                         int32_t* pid_out) {
  if (!scene || !color || !depth || width == 0 || height == 0) return -1;
  if (pid_out)
    for (uint64_t i = 0; i < (uint64_t)width * height; ++i) pid_out[i] = -1;
  const uint32_t ts = 1u << tile_logsize;
  const uint32_t ntx = (width + ts - 1) >> tile_logsize;
  const uint32_t nty = (height + ts - 1) >> tile_logsize;
  const uint32_t ntiles = ntx * nty;
  uint32_t* tile_cnt = (uint32_t*)calloc(ntiles + 1, sizeof(uint32_t));
  uint32_t* tile_off = (uint32_t*)calloc(ntiles + 1, sizeof(uint32_t));
  for (int d = 0; d < scene->num_drawcalls; ++d) {
    const orc_drawcall_t* dc = &scene->drawcalls[d];
    orc_dcstate_t st;
    orc_dcstate_init(&st, scene, dc);
    const int n = dc->prim_count;
    orc_rast_prim_t* rp = (orc_rast_prim_t*)malloc(sizeof(orc_rast_prim_t) * (n ? n : 1));
    int32_t* bb = (int32_t*)malloc(sizeof(int32_t) * 4 * (n ? n : 1));
    int* ok = (int*)malloc(sizeof(int) * (n ? n : 1));
    memset(tile_cnt, 0, sizeof(uint32_t) * (ntiles + 1));
    /* Binning: per primitive bbox -> tile range (gfxutil.cpp:237-250) */
    for (int i = 0; i < n; ++i) {
      const float* v = scene->prim_verts + (size_t)(dc->prim_offset + i) * 30;
      ok[i] = orc_setup_prim(v, width, height, dc->znear, dc->zfar, &rp[i], &bb[4 * i]) == 0;
      if (!ok[i]) continue;
      const uint32_t tx0 = (uint32_t)bb[4 * i + 0] >> tile_logsize;
      const uint32_t tx1 = ((uint32_t)bb[4 * i + 1] + ts - 1) >> tile_logsize;
      const uint32_t ty0 = (uint32_t)bb[4 * i + 2] >> tile_logsize;
      const uint32_t ty1 = ((uint32_t)bb[4 * i + 3] + ts - 1) >> tile_logsize;
      for (uint32_t ty = ty0; ty < ty1; ++ty)
        for (uint32_t tx = tx0; tx < tx1; ++tx) tile_cnt[ty * ntx + tx]++;
    }
    uint32_t total = 0;
    for (uint32_t t = 0; t < ntiles; ++t) { tile_off[t] = total; total += tile_cnt[t]; }
    uint32_t* pids = (uint32_t*)malloc(sizeof(uint32_t) * (total ? total : 1));
    memset(tile_cnt, 0, sizeof(uint32_t) * (ntiles + 1));
    for (int i = 0; i < n; ++i) {
      if (!ok[i]) continue;
      const uint32_t tx0 = (uint32_t)bb[4 * i + 0] >> tile_logsize;
      const uint32_t tx1 = ((uint32_t)bb[4 * i + 1] + ts - 1) >> tile_logsize;
      const uint32_t ty0 = (uint32_t)bb[4 * i + 2] >> tile_logsize;
      const uint32_t ty1 = ((uint32_t)bb[4 * i + 3] + ts - 1) >> tile_logsize;
      for (uint32_t ty = ty0; ty < ty1; ++ty)
        for (uint32_t tx = tx0; tx < tx1; ++tx) {
          const uint32_t t = ty * ntx + tx;
          pids[tile_off[t] + tile_cnt[t]++] = (uint32_t)i;
        }
    }
    /* Rasterizer::render per tile, pids in binning order (gpu_sw.h:38-61).
     * renderTile/renderQuad's hierarchical rejection is conservative, so the
     * covered set is exactly {pixel : all three edge values >= 0} inside the
     * scissor (graphics.cpp:813-825: inclusive, no top-left rule). */
    for (uint32_t t = 0; t < ntiles; ++t) {
      const uint32_t x0 = (t % ntx) << tile_logsize, y0 = (t / ntx) << tile_logsize;
      for (uint32_t k = 0; k < tile_cnt[t]; ++k) {
        const uint32_t i = pids[tile_off[t] + k];
        const orc_rast_prim_t* p = &rp[i];
        for (uint32_t y = y0; y < y0 + ts && y < height; ++y) {
          for (uint32_t x = x0; x < x0 + ts && x < width; ++x) {
            const int32_t e0 = orc_edge_eval(p->edges[0], x, y);
            const int32_t e1 = orc_edge_eval(p->edges[1], x, y);
            const int32_t e2 = orc_edge_eval(p->edges[2], x, y);
            if (e0 < 0 || e1 < 0 || e2 < 0) continue;
            if (coverage) {
              color[(uint64_t)y * width + x] = 0xffffffffu;
              continue;
            }
            uint32_t z;
            const uint32_t c = orc_shade(&st, p, e0, e1, e2, &z);
            const uint64_t px = (uint64_t)y * width + x;
            if (orc_om_write(&st, &color[px], &depth[px], c, z) && pid_out && st.color_write)
              pid_out[px] = dc->prim_offset + (int32_t)i;
          }
        }
      }
    }
    free(pids); free(ok); free(bb); free(rp);
  }
  free(tile_cnt); free(tile_off);
  return 0;
}

int orc_raster_render(const orc_scene_t* scene, uint32_t width, uint32_t height,
                      uint32_t tile_logsize, uint32_t* color, uint32_t* depth,
                      int32_t* pid_out) {
  return raster_render(scene, width, height, tile_logsize, 0, color, depth, pid_out);
}

void orc_edge_cover(const int32_t edges[9], uint32_t x0, uint32_t y0, uint32_t w, uint32_t h,
                    uint8_t* mask) {
  for (uint32_t j = 0; j < h; ++j)
    for (uint32_t i = 0; i < w; ++i) {
      const uint32_t x = x0 + i, y = y0 + j;
      mask[j * w + i] = orc_edge_eval(&edges[0], x, y) >= 0 && orc_edge_eval(&edges[3], x, y) >= 0 &&
                        orc_edge_eval(&edges[6], x, y) >= 0;
    }
}

int orc_raster_coverage(const orc_scene_t* scene, uint32_t width, uint32_t height,
                        uint32_t tile_logsize, uint32_t* color) {
  uint32_t dummy = 0;
  if (!color) return -1;
  return raster_render(scene, width, height, tile_logsize, 1, color, &dummy, NULL);
}
