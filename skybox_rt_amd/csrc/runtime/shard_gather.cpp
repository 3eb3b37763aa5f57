// shard_gather.cpp -- the multi-GPU frame exchange of the RT path as a C
// library over RCCL (include/rt_shard.h), for C hosts: no torch, no Python.
//
// One process per GPU, one communicator; every step ends with ONE gather of
// the ranks' compact tile buffers to rank 0 -- point-to-point ncclSend /
// ncclRecv pairs inside a group, so each peer's buffer crosses its own xGMI
// link to rank 0 (no ring all-gather, which would move the whole frame over
// every link) -- and rank 0's frame assembly (rt_frame_assemble), all
// enqueued on the caller's stream behind the render that filled the buffers.
// NO REFERENCE: the reference renders on one device; the
// tile -> rank partition follows sim/simx/raster_unit.cpp:109-111.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstring>

#include "rt_shard.h"

struct rt_shard_comm {
  ncclComm_t comm = nullptr;
  uint32_t rank = 0, world = 1;
  int device = 0;
};

static_assert(sizeof(ncclUniqueId) <= RT_SHARD_ID_BYTES, "ncclUniqueId does not fit");

namespace {

uint64_t local_tiles(uint32_t width, uint32_t height, uint32_t rank, uint32_t world) {
  const uint64_t n = (uint64_t)((width + 31u) / 32u) * ((height + 31u) / 32u);
  return n > rank ? (n - rank + world - 1) / world : 0;
}

}  // namespace

extern "C" {

int rt_shard_unique_id(uint8_t id[RT_SHARD_ID_BYTES]) {
  if (!id) return -1;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return -1;
  std::memset(id, 0, RT_SHARD_ID_BYTES);
  std::memcpy(id, &u, sizeof(u));
  return 0;
}

int rt_shard_comm_init(rt_shard_comm_h* out, const uint8_t id[RT_SHARD_ID_BYTES], uint32_t rank,
                       uint32_t world, int device) {
  if (!out || !id || world == 0 || rank >= world) return -1;
  if (hipSetDevice(device) != hipSuccess) return -1;
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  auto* c = new rt_shard_comm();
  c->rank = rank;
  c->world = world;
  c->device = device;
  if (ncclCommInitRank(&c->comm, (int)world, u, (int)rank) != ncclSuccess) {
    delete c;
    return -1;
  }
  *out = c;
  return 0;
}

int rt_shard_comm_free(rt_shard_comm_h c) {
  if (!c) return 0;
  const ncclResult_t e = ncclCommDestroy(c->comm);
  delete c;
  return e == ncclSuccess ? 0 : -1;
}

int rt_shard_comm_info(rt_shard_comm_h c, uint32_t* rank, uint32_t* world) {
  if (!c) return -1;
  int n = 0, r = 0;
  if (ncclCommCount(c->comm, &n) != ncclSuccess || ncclCommUserRank(c->comm, &r) != ncclSuccess)
    return -1;
  if (rank) *rank = (uint32_t)r;
  if (world) *world = (uint32_t)n;
  return 0;
}

int rt_shard_device_count(void) {
  int n = 0;
  return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

int rt_shard_stream_sync(void* stream) {
  return hipStreamSynchronize((hipStream_t)stream) == hipSuccess ? 0 : -1;
}

uint64_t rt_shard_local_words(uint32_t width, uint32_t height, uint32_t rank, uint32_t world) {
  return world == 0 ? 0 : local_tiles(width, height, rank, world) * 1024u;
}

int rt_frame_gather(rt_shard_comm_h c, const uint32_t* local, uint32_t* recv,
                    uint64_t slots_per_rank, uint32_t* image, uint32_t width, uint32_t height,
                    void* stream) {
  if (!c || !local || width == 0 || height == 0) return -1;
  const hipStream_t s = (hipStream_t)stream;
  const uint64_t mine = local_tiles(width, height, c->rank, c->world) * 1024u;
  if (c->rank == 0) {
    if (!recv || !image || slots_per_rank % 1024u ||
        slots_per_rank < local_tiles(width, height, 0, c->world) * 1024u)
      return -1;
    // rank 0's own tiles: a device copy into its slot of the receive buffer
    if (mine && hipMemcpyAsync(recv, local, mine * 4, hipMemcpyDeviceToDevice, s) != hipSuccess)
      return -1;
  }
  if (c->world > 1) {
    if (ncclGroupStart() != ncclSuccess) return -1;
    if (c->rank == 0) {
      for (uint32_t r = 1; r < c->world; ++r) {
        const uint64_t n = local_tiles(width, height, r, c->world) * 1024u;
        if (n && ncclRecv(recv + (uint64_t)r * slots_per_rank, n, ncclUint32, (int)r, c->comm, s) !=
                     ncclSuccess) {
          ncclGroupEnd();
          return -1;
        }
      }
    } else if (mine && ncclSend(local, mine, ncclUint32, 0, c->comm, s) != ncclSuccess) {
      ncclGroupEnd();
      return -1;
    }
    if (ncclGroupEnd() != ncclSuccess) return -1;
  }
  if (c->rank == 0) return rt_frame_assemble(image, recv, width, height, c->world, slots_per_rank, stream);
  return 0;
}

}  // extern "C"
