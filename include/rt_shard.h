/* rt_shard.h -- multi-GPU frame exchange of the RT path:
 * rank 0's assembly of the frame from the per-rank compact tile buffers that
 * one gather (RCCL over xGMI) placed side by side in its receive buffer.
 *
 * NO REFERENCE: the reference renders on one device; its tile striding over
 * raster units (sim/simx/raster_unit.cpp:109-111,224-227) is the partition
 * this follows -- 32x32 tile t (row-major over the frame) belongs to rank
 * t mod world and is that rank's local tile lt = t div world; a rank's
 * compact buffer holds its local tiles in order, each tile row-major
 * (slot = lt * 1024 + 32 * (y mod 32) + x mod 32; the RT kernels' store_pixel
 * with RT_FLAG_COMPACT, restated by skybox_rt_amd/shard.py task_pixel_index).
 * Library: skybox_rt_amd/lib/libframe_assemble.so. */
#ifndef RT_SHARD_H
#define RT_SHARD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* image[y * width + x] = recv[r * slots_per_rank + slot(x, y)] for every pixel
 * of the width x height frame.  image, recv: device pointers (ARGB8888
 * words); slots_per_rank: the receive buffer's per-rank stride (a multiple
 * of 1024, at least rank 0's local tiles x 1024); stream: a hipStream_t (NULL
 * = the default stream).  Asynchronous: enqueues ONE kernel on `stream`.
 * Returns 0, -1 for bad arguments, or the HIP error code of the launch. */
int rt_frame_assemble(uint32_t* image, const uint32_t* recv, uint32_t width, uint32_t height,
                      uint32_t world, uint64_t slots_per_rank, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* RT_SHARD_H */
