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
 * Library: skybox_rt_amd/lib/librt_shard.so (HIP + RCCL, no torch): the
 * assembly kernel and the RCCL gather, so a C host runs the multi-GPU path
 * without Python (rtapp --rank/--ranks). */
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

/* ---- the frame exchange over RCCL (one process per GPU) ---------------- */
typedef struct rt_shard_comm* rt_shard_comm_h;
#define RT_SHARD_ID_BYTES 128
/* communicator id: made once (rank 0) and handed to every rank by the host's
 * own means (a file, a socket, an MPI broadcast...) */
int rt_shard_unique_id(uint8_t id[RT_SHARD_ID_BYTES]);
/* join the `world`-rank communicator as `rank` on HIP device `device`
 * (collective: every rank calls it) */
int rt_shard_comm_init(rt_shard_comm_h* comm, const uint8_t id[RT_SHARD_ID_BYTES], uint32_t rank,
                       uint32_t world, int device);
int rt_shard_comm_free(rt_shard_comm_h comm);
/* the communicator's view: this rank and the number of ranks it connects */
int rt_shard_comm_info(rt_shard_comm_h comm, uint32_t* rank, uint32_t* world);
/* HIP devices visible to this process; wait for every operation on a stream */
int rt_shard_device_count(void);
int rt_shard_stream_sync(void* stream);
/* words of `rank`'s compact tile buffer for a width x height frame */
uint64_t rt_shard_local_words(uint32_t width, uint32_t height, uint32_t rank, uint32_t world);
/* One frame's exchange, enqueued on `stream` (a hipStream_t; NULL = default):
 * every rank's compact tile buffer `local` (rt_shard_local_words words, the
 * RT kernels' RT_FLAG_COMPACT output) goes to rank 0 -- ncclSend to / ncclRecv
 * from rank 0 in one group, each peer over its own link -- into `recv`
 * (rank r at r * slots_per_rank; slots_per_rank a multiple of 1024 holding
 * rank 0's buffer), then rank 0 assembles the frame into `image` (W*H words,
 * rt_frame_assemble).  recv / image are used on rank 0 only.  Collective:
 * every rank calls it for every frame.  Returns 0 or -1. */
int rt_frame_gather(rt_shard_comm_h comm, const uint32_t* local, uint32_t* recv,
                    uint64_t slots_per_rank, uint32_t* image, uint32_t width, uint32_t height,
                    void* stream);

#ifdef __cplusplus
}
#endif

#endif /* RT_SHARD_H */
