/*
 * vx_spawn.h -- device-side launch surface for HIP kernel programs run by the
 * MI355X driver (libvortex-hip.so).  Replaces kernel/include/vx_spawn.h:24-59
 * and kernel/src/vx_spawn.c:157-322.
 *
 * A kernel program is one HIP translation unit compiled for gfx950 into a
 * code object, wrapped in the reference's 16-byte vxbin header
 * (kernel/scripts/vxbin.py:54-78) and uploaded with vx_upload_kernel_file().
 * vx_start() launches its `vx_main` entry over the whole device.  Like the
 * reference's main(), VX_MAIN's body reads its argument pointer from the
 * STARTUP_ARG DCRs (the reference reads MSCRATCH, draw3d/kernel.cpp:287) and
 * calls vx_spawn_threads()/vx_spawn_tasks(), which call the per-task
 * callback `kernel_body` once per task.
 *
 * Differences forced by the hardware (documented in DESIGN.md):
 *  - A GPU has no thread-local storage and HIP reserves the name `blockIdx`,
 *    so the task coordinates (the reference's __thread blockIdx/threadIdx,
 *    vx_spawn.c:26-27,75-80) reach the callback as an explicit `vx_task_t`.
 *  - VX_MAIN's body runs SPMD on every hardware thread (64-lane wave
 *    granularity); the reference runs main() per core and wspawns warps.
 *  - Tasks are dealt to hardware threads round-robin (task = k*T + tid,
 *    T = resident hardware threads), so the 64 lanes of a wave always take 64
 *    consecutive task ids (coalesced, and an 8x8 pixel tile for the RT app);
 *    the reference deals contiguous per-core chunks.  Every task still runs
 *    exactly once with blockIdx = the vx_spawn.c:75-80 decomposition.
 *  - group_size > 1 (vx_spawn.c:187-246) is not supported yet: returns -1.
 */
#ifndef VX_SPAWN_H
#define VX_SPAWN_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "VX_types.h"

/* Filled by the driver before every launch (hip_driver.cpp, start()). */
extern "C" {
__constant__ uint32_t __vx_dcrs[VX_DCR_MIRROR_SIZE];     /* DCR mirror */
__constant__ uint64_t __vx_mem_base;                     /* arena base VA */
__device__ unsigned long long __vx_mpm[VX_MPM_COUNT];    /* perf counters */
}

#define VX_MPM_TASKS 2  /* __vx_mpm slot for VX_CSR_MINSTRET (tasks run) */

typedef struct { uint32_t x, y, z; } vx_dim3_t;

typedef struct {
  vx_dim3_t blockIdx;   /* task coordinates (vx_spawn.c:75-80) */
  vx_dim3_t threadIdx;  /* always 0 for group_size == 1 (vx_spawn.c:68-70) */
  uint32_t task_id;     /* linear task id */
} vx_task_t;

/* device address (as handed out by vx_mem_alloc) -> pointer */
template <typename T>
__device__ __forceinline__ T* vx_ptr(uint64_t addr) {
  return reinterpret_cast<T*>(__vx_mem_base + addr);
}

__device__ __forceinline__ uint32_t vx_dcr(uint32_t addr) { return __vx_dcrs[addr]; }

/* hardware identity (vx_intrinsics.h vx_core_id/vx_warp_id/vx_thread_id) */
__device__ __forceinline__ uint32_t vx_core_id() { return blockIdx.x; }
__device__ __forceinline__ uint32_t vx_num_cores() { return gridDim.x; }
__device__ __forceinline__ uint32_t vx_warp_id() { return threadIdx.x >> 6; }
__device__ __forceinline__ uint32_t vx_num_warps() { return blockDim.x >> 6; }
__device__ __forceinline__ uint32_t vx_thread_id() { return threadIdx.x & 63u; }
__device__ __forceinline__ uint32_t vx_num_threads() { return 64u; }

__device__ __forceinline__ uint32_t __vx_wave_sum(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

/* vx_spawn_threads(dimension, grid_dim, block_dim, kernel_func, arg):
 * calls kernel_func(task, arg) once per grid cell.  `kernel_func` is a
 * __device__ function (inlined); returns 0, or -1 for unsupported shapes. */
template <typename F, typename Arg>
__device__ __forceinline__ int vx_spawn_threads(uint32_t dimension, const uint32_t* grid_dim,
                                                const uint32_t* block_dim, F kernel_func,
                                                Arg* arg) {
  uint32_t gd[3], num_groups = 1, group_size = 1;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    gd[i] = (grid_dim && (uint32_t)i < dimension) ? grid_dim[i] : 1u;
    const uint32_t bd = (block_dim && (uint32_t)i < dimension) ? block_dim[i] : 1u;
    num_groups *= gd[i];
    group_size *= bd;
  }
  if (group_size != 1) return -1;
  const uint32_t T = gridDim.x * blockDim.x;
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t ran = 0;
  vx_task_t task;
  task.threadIdx.x = task.threadIdx.y = task.threadIdx.z = 0;
  for (uint32_t t = tid; t < num_groups; t += T) {
    task.task_id = t;
    task.blockIdx.x = t % gd[0];
    task.blockIdx.y = (t / gd[0]) % gd[1];
    task.blockIdx.z = t / (gd[0] * gd[1]);
    kernel_func(task, arg);
    ++ran;
  }
  const uint32_t wsum = __vx_wave_sum(ran);
  if ((threadIdx.x & 63u) == 0 && wsum)
    atomicAdd(&__vx_mpm[VX_MPM_TASKS], (unsigned long long)wsum);
  return 0;
}

/* 1-D convenience form (the north star's vx_spawn_tasks) */
template <typename F, typename Arg>
__device__ __forceinline__ int vx_spawn_tasks(uint32_t num_tasks, F kernel_func, Arg* arg) {
  return vx_spawn_threads(1u, &num_tasks, (const uint32_t*)nullptr, kernel_func, arg);
}

/* VX_MAIN(ArgT, arg, block_threads) { ... return vx_spawn_tasks(...); }
 * defines the `vx_main` entry the driver launches with `block_threads`
 * threads per workgroup (must be a multiple of 64). */
#define VX_MAIN(ArgT, argname, block_threads)                                        \
  static __device__ __forceinline__ int __vx_main_body(ArgT* argname);               \
  extern "C" __global__ void __launch_bounds__(block_threads) vx_main() {            \
    const uint64_t a = ((uint64_t)__vx_dcrs[VX_DCR_BASE_STARTUP_ARG1] << 32) |       \
                       (uint64_t)__vx_dcrs[VX_DCR_BASE_STARTUP_ARG0];                \
    (void)__vx_main_body(vx_ptr<ArgT>(a));                                           \
  }                                                                                  \
  static __device__ __forceinline__ int __vx_main_body(ArgT* argname)

#endif /* VX_SPAWN_H */
