// spawn_test.hip -- launch-surface test program (the analog of the reference's
// tests/regression/demo and basic apps, which exercise vx_spawn_threads +
// kernel_body).  Every task writes its decomposed blockIdx and bumps a
// per-task counter, so the host can check the task -> blockIdx mapping of
// vx_spawn.c:75-80 and that each task ran exactly once.
#include <hip/hip_runtime.h>

#include "vx_spawn.h"

typedef struct {
  uint32_t dim;
  uint32_t grid[3];
  uint64_t out_addr;   // uint32 [num_tasks]: x | y << 10 | z << 20
  uint64_t hits_addr;  // uint32 [num_tasks]: times the task ran
} spawn_arg_t;

static __device__ __forceinline__ void kernel_body(const vx_task_t& task, spawn_arg_t* a) {
  const uint32_t id = task.task_id;
  vx_ptr<uint32_t>(a->out_addr)[id] =
      task.blockIdx.x | (task.blockIdx.y << 10) | (task.blockIdx.z << 20);
  atomicAdd(&vx_ptr<uint32_t>(a->hits_addr)[id], 1u);
}

VX_MAIN(spawn_arg_t, arg, 256) {
  return vx_spawn_threads(arg->dim, arg->grid, (const uint32_t*)nullptr,
                          [](const vx_task_t& t, spawn_arg_t* a) { kernel_body(t, a); }, arg);
}
