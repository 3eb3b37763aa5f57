/*
 * vx_spawn.h -- device-side launch surface for HIP kernel programs run by the
 * MI355X driver (libvortex-hip.so).  Replaces kernel/include/vx_spawn.h:24-59
 * and kernel/src/vx_spawn.c:157-322.
 *
 * A kernel program is one HIP translation unit compiled for gfx950 into a
 * code object, wrapped in the reference's 16-byte vxbin header
 * (kernel/scripts/vxbin.py:54-78) and uploaded with vx_upload_kernel_file().
 * vx_start() launches its `vx_main` entry over a resident persistent grid.
 * Like the reference's main(), VX_MAIN's body reads its argument pointer from
 * the STARTUP_ARG DCRs (the reference reads MSCRATCH, draw3d/kernel.cpp:287)
 * and calls vx_spawn_threads()/vx_spawn_tasks(), which call the per-task
 * callback `kernel_body` once per task.
 *
 * Differences forced by the hardware (documented in DESIGN.md):
 *  - A GPU has no thread-local storage and HIP reserves the name `blockIdx`,
 *    so the task coordinates (the reference's __thread blockIdx/threadIdx,
 *    vx_spawn.c:26-27,75-80) reach the callback as an explicit `vx_task_t`.
 *  - VX_MAIN's body runs SPMD on every hardware thread (64-lane waves); the
 *    reference runs main() per core and wspawns warps.
 *  - Scheduling: tasks are handed out in chunks of 64 consecutive ids, one
 *    chunk per wave (one task per lane: coalesced, and an 8x8 pixel block in
 *    the RT app); wave w of the grid takes chunks w, w + W, w + 2W, ...  The
 *    driver launches several times more blocks than are resident, so the
 *    hardware dispatcher, which hands a CU a new block whenever one retires,
 *    is the load balancer (the reference deals static per-core ranges,
 *    vx_spawn.c:247-316).  Atomic work queues (per-XCD heads) measured 2x
 *    slower than this on the RT kernel and were dropped.  Every task runs
 *    exactly once with blockIdx = the vx_spawn.c:75-80 decomposition.
 *  - Perf counters (vx_mpm_add): LDS counters per block, written as one
 *    64-B row per block at block exit (plain stores, no global atomics, no
 *    per-launch memset) when the driver enables counters; vx_mpm_query
 *    sums the rows of the last launch.  Without counters a launch writes
 *    one word (the task count) beside its output.
 *  - group_size > 1 (vx_spawn.c:187-246) is not supported yet: returns -1.
 */
#ifndef VX_SPAWN_H
#define VX_SPAWN_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "VX_types.h"

#define VX_CHUNK 64          /* tasks per wave */
#define VX_MAX_GRID 32768    /* blocks per launch (rows of the counter slab) */

/* per-launch device state: one 64-B row of the first VX_MPM_ROW u32 mpm
 * counters per block, each written by its block at exit -- only when the
 * driver asks for counters (DCR mirror word VX_DCR_HIP_MPM_ROWS: profiling
 * requested, as VORTEX_PROFILING gates the reference's perf classes,
 * runtime/stub/utils.cpp:25-47); kernel programs count into slots <
 * VX_MPM_ROW, vx_mpm_query reads the others as 0.  `tasks` = the task count
 * the launch spawned, one word written by block 0 every launch
 * (vx_mpm_query(MINSTRET) without counter rows). */
#define VX_MPM_ROW 16
typedef struct {
  uint32_t mpm[VX_MAX_GRID][VX_MPM_ROW];
  uint32_t tasks;
  uint32_t pad;
  uint64_t t0;  /* s_memrealtime (100 MHz) when block 0 started: the launch's start
                 * for the completion kernel (VX_MAIN's <entry>_done) */
} vx_state_t;

/* Filled by the driver before every launch (hip_driver.cpp, start()). */
extern "C" {
__constant__ uint32_t __vx_dcrs[VX_DCR_MIRROR_SIZE];     /* DCR mirror */
__constant__ uint64_t __vx_mem_base;                     /* arena base VA */
__device__ vx_state_t __vx_state;
}
/* this block's counters (zeroed / written back by VX_MAIN) */
__shared__ uint32_t __vx_mpm_lds[VX_MPM_ROW];

#define VX_MPM_TASKS 2  /* mpm slot for VX_CSR_MINSTRET (tasks run) */

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

/* The arena as one buffer resource (V#): device addresses below 4 GiB are
 * 32-bit buffer offsets, so hot loops use buffer_load/store with an SGPR
 * descriptor instead of 64-bit flat addressing (flat loads also count on
 * lgkmcnt and so serialise with LDS traffic).  Out-of-range offsets read 0. */
struct vx_arena {
  __amdgpu_buffer_rsrc_t r;
  uint64_t base;
  __device__ __forceinline__ static vx_arena get() {
    const uint64_t b = __vx_mem_base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    vx_arena a;
    a.base = ((uint64_t)hi << 32) | lo;
    a.r = __builtin_amdgcn_make_buffer_rsrc((void*)a.base, 0, (int)0xffffffffu, 0x00020000);
    return a;
  }
  /* Wave-uniform loads through the scalar cache (s_load into SGPRs): one
   * instruction per record for the whole wave instead of 64 lanes' worth of
   * vector-cache data return.  `off` must be the same in every lane (it is
   * taken from the first active lane); the data must not change during the
   * launch (scene records, never the framebuffer). */
  template <typename T>
  __device__ __forceinline__ T sld(uint32_t off) const {
    const uint32_t o = __builtin_amdgcn_readfirstlane(off);
    return *(const __attribute__((address_space(4))) T*)(base + o);
  }
  __device__ __forceinline__ float4 sld_f4(uint32_t off) const { return sld<float4>(off); }
  __device__ __forceinline__ uint4 sld_u4(uint32_t off) const { return sld<uint4>(off); }
  /* N consecutive 16-B words of one record from one wave-uniform address:
   * immediate offsets off one pointer, so the loads merge into wide s_loads
   * (s_load_dwordx16 for a 64-B record) instead of one per word */
  template <int N>
  __device__ __forceinline__ void sld_u4n(uint32_t off, uint4* out) const {
    const uint32_t o = __builtin_amdgcn_readfirstlane(off);
    const __attribute__((address_space(4))) uint4* p =
        (const __attribute__((address_space(4))) uint4*)(base + o);
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = p[i];
    /* (pinning every word in SGPRs at the load, so the compiler cannot sink
     * parts of it into the branches that use them, measured slower: r06a,
     * config 3 0.0181 vs 0.0169 ms, BVH walk 0.0355 vs 0.0340) */
  }
  __device__ __forceinline__ float4 ld_f4(uint32_t off) const {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]),
                       __uint_as_float(v[3]));
  }
  __device__ __forceinline__ uint4 ld_u4(uint32_t off) const {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    return make_uint4(v[0], v[1], v[2], v[3]);
  }
  __device__ __forceinline__ uint32_t ld_u32(uint32_t off) const {
    return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
  }
  __device__ __forceinline__ uint2 ld_u2(uint32_t off) const {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
    return make_uint2(v[0], v[1]);
  }
  __device__ __forceinline__ uint32_t ld_u16(uint32_t off) const {
    return __builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0);
  }
  __device__ __forceinline__ uint32_t ld_u8(uint32_t off) const {
    return __builtin_amdgcn_raw_buffer_load_b8(r, off, 0, 0);
  }
  __device__ __forceinline__ void st_u32(uint32_t off, uint32_t v) const {
    __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, 0);
  }
  __device__ __forceinline__ void st_u4(uint32_t off, uint4 v) const {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 w = {v.x, v.y, v.z, v.w};
    __builtin_amdgcn_raw_buffer_store_b128(w, r, off, 0, 0);
  }
};

/* threads per workgroup: a compile-time constant when the kernel program
 * defines VX_BLOCK_THREADS (its VX_MAIN block size) -- blockDim.x is a
 * vector-memory load from the dispatch packet, on every wave's way to its
 * first chunk */
__device__ __forceinline__ uint32_t __vx_block_dim() {
#ifdef VX_BLOCK_THREADS
  return VX_BLOCK_THREADS;
#else
  return blockDim.x;
#endif
}

/* hardware identity (vx_intrinsics.h vx_core_id/vx_warp_id/vx_thread_id) */
__device__ __forceinline__ uint32_t vx_core_id() { return blockIdx.x; }
__device__ __forceinline__ uint32_t vx_num_cores() { return gridDim.x; }
__device__ __forceinline__ uint32_t vx_warp_id() { return threadIdx.x >> 6; }
__device__ __forceinline__ uint32_t vx_num_warps() { return __vx_block_dim() >> 6; }
__device__ __forceinline__ uint32_t vx_thread_id() { return threadIdx.x & 63u; }
__device__ __forceinline__ uint32_t vx_num_threads() { return 64u; }
__device__ __forceinline__ uint32_t vx_xcc_id() {
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 7u;
}

__device__ __forceinline__ uint32_t __vx_wave_sum(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

/* mpm counter add: wave sum, then one LDS atomic per wave into the block's
 * row (all 64 lanes must call it).  Nothing when the driver wants no counter
 * rows (a wave-uniform constant): no cross-lane sums, no LDS atomics --
 * with the block barriers of VX_MAIN also gone then, config 3 measured
 * 0.02372 -> 0.01982 ms (A/B r03r). */
#ifndef VX_ROWS_GATE
#define VX_ROWS_GATE 1  /* 0: count and meet at the block barriers regardless */
#endif
__device__ __forceinline__ void vx_mpm_add(int slot, uint32_t v) {
  if (VX_ROWS_GATE && !__vx_dcrs[VX_DCR_HIP_MPM_ROWS]) return;
  const uint32_t s = __vx_wave_sum(v);
  if ((threadIdx.x & 63u) == 0 && s && slot < VX_MPM_ROW) atomicAdd(&__vx_mpm_lds[slot], s);
}

/* block 0 records how many tasks the launch spawns (all lanes may call) */
__device__ __forceinline__ void __vx_declare_tasks(uint32_t n) {
  if (blockIdx.x == 0 && threadIdx.x == 0) __vx_state.tasks = n;
}

/* The block whose chunks this hardware block runs.  VX_XCD_GROUP = g > 0:
 * blocks are dealt round-robin over the 8 XCDs (b and b + 8 share one, each
 * XCD its own L2; MI355X_MICROARCH.md "Workgroup dispatch, XCD placement"),
 * so logical blocks are regrouped that g consecutive ones -- one 32x32 tile's
 * chunks in the RT kernels -- run on one XCD, and the next 8 groups, one per
 * XCD, start together (the work order's heaviest tiles spread over the
 * XCDs).  A placement for speed only: every logical block runs once either
 * way.  The tail of a grid that is not a multiple of 8 g keeps its ids. */
#ifndef VX_XCD_GROUP
#define VX_XCD_GROUP 0
#endif
__device__ __forceinline__ uint32_t __vx_logical_block() {
#if VX_XCD_GROUP > 0
  const uint32_t b = blockIdx.x, span = 8u * VX_XCD_GROUP;
  if (b >= gridDim.x - gridDim.x % span) return b;
  const uint32_t x = b & 7u, k = b >> 3;
  return (k / VX_XCD_GROUP) * span + x * VX_XCD_GROUP + k % VX_XCD_GROUP;
#else
  return blockIdx.x;
#endif
}

struct __vx_no_epilogue {
  template <typename Arg>
  __device__ __forceinline__ void operator()(bool, Arg*) const {}
};

/* vx_spawn_threads(dimension, grid_dim, block_dim, kernel_func, arg):
 * calls kernel_func(task, arg) once per grid cell.  `epilogue(final, arg)` is
 * called by all 64 lanes of a wave after each chunk (final = false) and once
 * when the wave runs out of work (final = true): the hook a kernel uses for
 * wave-level work such as compacted secondary rays.  Returns 0, or -1 for
 * unsupported shapes. */
template <typename F, typename E, typename Arg>
__device__ __forceinline__ int vx_spawn_threads_ex(uint32_t dimension, const uint32_t* grid_dim,
                                                   const uint32_t* block_dim, F kernel_func,
                                                   E epilogue, Arg* arg) {
  uint32_t gd[3], num_groups = 1, group_size = 1;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    gd[i] = (grid_dim && (uint32_t)i < dimension) ? grid_dim[i] : 1u;
    const uint32_t bd = (block_dim && (uint32_t)i < dimension) ? block_dim[i] : 1u;
    num_groups *= gd[i];
    group_size *= bd;
  }
  if (group_size != 1) return -1;
  __vx_declare_tasks(num_groups);
  const uint32_t nchunks = (num_groups + VX_CHUNK - 1) / VX_CHUNK;
  const uint32_t nwaves = gridDim.x * (__vx_block_dim() >> 6);
  uint32_t ran = 0;
  vx_task_t task;
  task.threadIdx.x = task.threadIdx.y = task.threadIdx.z = 0;
  for (uint32_t c = __vx_logical_block() * (__vx_block_dim() >> 6) + (threadIdx.x >> 6); c < nchunks;
       c += nwaves) {
    const uint32_t t = c * VX_CHUNK + (threadIdx.x & 63u);
    if (t < num_groups) {
      task.task_id = t;
      if (dimension <= 1) {  // t < num_groups = gd[0]: no division (vx_spawn_tasks)
        task.blockIdx.x = t;
        task.blockIdx.y = task.blockIdx.z = 0;
      } else {
        task.blockIdx.x = t % gd[0];
        task.blockIdx.y = (t / gd[0]) % gd[1];
        task.blockIdx.z = t / (gd[0] * gd[1]);
      }
      kernel_func(task, arg);
      ++ran;
    }
    epilogue(false, arg);
  }
  epilogue(true, arg);
  vx_mpm_add(VX_MPM_TASKS, ran);
  return 0;
}

template <typename F, typename Arg>
__device__ __forceinline__ int vx_spawn_threads(uint32_t dimension, const uint32_t* grid_dim,
                                                const uint32_t* block_dim, F kernel_func,
                                                Arg* arg) {
  return vx_spawn_threads_ex(dimension, grid_dim, block_dim, kernel_func, __vx_no_epilogue(), arg);
}

/* 1-D convenience forms (the north star's vx_spawn_tasks) */
template <typename F, typename Arg>
__device__ __forceinline__ int vx_spawn_tasks(uint32_t num_tasks, F kernel_func, Arg* arg) {
  return vx_spawn_threads(1u, &num_tasks, (const uint32_t*)nullptr, kernel_func, arg);
}
template <typename F, typename E, typename Arg>
__device__ __forceinline__ int vx_spawn_tasks_ex(uint32_t num_tasks, F kernel_func, E epilogue,
                                                 Arg* arg) {
  return vx_spawn_threads_ex(1u, &num_tasks, (const uint32_t*)nullptr, kernel_func, epilogue, arg);
}

/* Block-synchronous form for kernels that cooperate across the waves of a
 * workgroup (e.g. compaction queues in LDS): the block takes blockDim.x
 * consecutive tasks per step (wave w: tasks step*blockDim + 64w ..+63, the
 * same 64-task chunks as above), steps are block-uniform, and every thread
 * calls kernel_func(task, valid, arg) -- valid = false past num_tasks -- and
 * then block_epilogue(step, arg), which may use __syncthreads() (step =
 * the block step: tasks step * blockDim.x ...). */
template <typename F, typename E, typename Arg>
__device__ __forceinline__ int vx_spawn_tasks_block(uint32_t num_tasks, F kernel_func,
                                                    E block_epilogue, Arg* arg) {
  const uint32_t nsteps = (num_tasks + __vx_block_dim() - 1) / __vx_block_dim();
  __vx_declare_tasks(num_tasks);
  uint32_t ran = 0;
  vx_task_t task;
  task.threadIdx.x = task.threadIdx.y = task.threadIdx.z = 0;
  task.blockIdx.y = task.blockIdx.z = 0;
  for (uint32_t st = blockIdx.x; st < nsteps; st += gridDim.x) {
    const uint32_t t = st * __vx_block_dim() + threadIdx.x;
    task.task_id = t;
    task.blockIdx.x = t;
    const bool valid = t < num_tasks;
    kernel_func(task, valid, arg);
    ran += valid;
    block_epilogue(st, arg);
  }
  vx_mpm_add(VX_MPM_TASKS, ran);
  return 0;
}

/* Block-cooperative form: each workgroup step takes ONE 64-task chunk and
 * every wave of the workgroup sees the same 64 tasks (lane l: task
 * chunk * 64 + l), so the waves can split the work of each task among them
 * (e.g. the flat image's triangle list).  kernel_func(task, valid, arg) is
 * called by every thread; steps are block-uniform (kernel_func may use
 * __syncthreads()).  Tasks are counted once (by wave 0). */
template <typename F, typename Arg>
__device__ __forceinline__ int vx_spawn_chunks_block(uint32_t num_tasks, F kernel_func, Arg* arg) {
  const uint32_t nchunks = (num_tasks + VX_CHUNK - 1) / VX_CHUNK;
  __vx_declare_tasks(num_tasks);
  uint32_t ran = 0;
  vx_task_t task;
  task.threadIdx.x = task.threadIdx.y = task.threadIdx.z = 0;
  task.blockIdx.y = task.blockIdx.z = 0;
  for (uint32_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const uint32_t t = c * VX_CHUNK + (threadIdx.x & 63u);
    task.task_id = t;
    task.blockIdx.x = t;
    const bool valid = t < num_tasks;
    kernel_func(task, valid, arg);
    ran += valid && threadIdx.x < 64u;
  }
  vx_mpm_add(VX_MPM_TASKS, ran);
  return 0;
}

/* VX_MAIN(ArgT, arg, block_threads) { ... return vx_spawn_tasks(...); }
 * defines the entry the driver launches with `block_threads` threads per
 * workgroup (must be a multiple of 64): `vx_main`, or the image's own name
 * vx_main_<image> given by -DVX_ENTRY (the driver finds it in the code
 * object's symbol table, so profiles tell the images apart).  The body also
 * sees `vx_launch_tag`, the launch's one kernel argument: 0, or the value an
 * app set for this launch with vx_hip_set_launch_tag (vortex_hip.h) -- e.g.
 * the step of a launch sequence sharing one argument block -- and
 * `vx_launch_words`, four more u32 set with vx_hip_set_launch_words (0
 * unless set): per-launch values that travel in the dispatch packet's
 * kernel arguments instead of a copy queued between two launches. */
struct vx_launch_words_t {
  uint32_t w[4];
};
#define VX_MAIN(ArgT, argname, block_threads) \
  VX_MAIN_BOUNDS(ArgT, argname, __launch_bounds__(block_threads))
/* same, asking the compiler for `waves_per_eu` resident waves per SIMD */
#define VX_MAIN_OCC(ArgT, argname, block_threads, waves_per_eu) \
  VX_MAIN_BOUNDS(ArgT, argname, __launch_bounds__(block_threads, waves_per_eu))
#ifndef VX_ENTRY
#define VX_ENTRY vx_main
#endif
#define __VX_CAT2(a, b) a##b
#define __VX_CAT(a, b) __VX_CAT2(a, b)
/* <entry>_done(host, nonce): the completion kernel the driver queues right
 * behind a launch started on an idle queue (hip_driver.cpp start: the
 * synchronous start + wait of the reference's apps).  One lane stores the
 * launch's start stamp (block 0's, vx_state_t::t0) and its own (the launch
 * has completed: stream order), then `nonce` with a system-scope release, to
 * the driver's pinned host words; vx_ready_wait spins on that word -- no HIP
 * event or stream query between the frame and the host. */
#define __VX_DONE_KERNEL                                                             \
  extern "C" __global__ void __launch_bounds__(64) __VX_CAT(VX_ENTRY, _done)(uint64_t __vx_host, \
                                                                        uint32_t __vx_nonce) { \
    if (threadIdx.x == 0) {                                                          \
      const uint64_t t1 = __builtin_amdgcn_s_memrealtime();                          \
      const uint64_t t0 = __vx_state.t0;                                             \
      uint32_t* h = reinterpret_cast<uint32_t*>(__vx_host);                          \
      __hip_atomic_store(h + 2, (uint32_t)t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); \
      __hip_atomic_store(h + 3, (uint32_t)(t0 >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); \
      __hip_atomic_store(h + 4, (uint32_t)t1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); \
      __hip_atomic_store(h + 5, (uint32_t)(t1 >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); \
      __hip_atomic_store(h, __vx_nonce, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);  \
    }                                                                                \
  }
#define VX_MAIN_BOUNDS(ArgT, argname, bounds)                                        \
  __VX_DONE_KERNEL                                                                   \
  static __device__ __forceinline__ int __vx_main_body(ArgT* argname, uint32_t vx_launch_tag, \
                                                       vx_launch_words_t vx_launch_words); \
  extern "C" __global__ void bounds VX_ENTRY(uint32_t __vx_tag, vx_launch_words_t __vx_words) { \
    /* the launch's start stamp (one lane of block 0; <entry>_done reads it) */      \
    if (blockIdx.x == 0 && threadIdx.x == 0) __vx_state.t0 = __builtin_amdgcn_s_memrealtime(); \
    /* the block's counter row: only when the driver reads rows (then the   */    \
    /* block's waves meet at entry and exit; without, each wave runs and    */    \
    /* retires on its own)                                                  */    \
    const bool rows_on = !VX_ROWS_GATE || __vx_dcrs[VX_DCR_HIP_MPM_ROWS] != 0;       \
    if (rows_on) {                                                                   \
      if (threadIdx.x < VX_MPM_ROW) __vx_mpm_lds[threadIdx.x] = 0;                   \
      __syncthreads();                                                               \
    }                                                                                \
    const uint64_t a = ((uint64_t)__vx_dcrs[VX_DCR_BASE_STARTUP_ARG1] << 32) |       \
                       (uint64_t)__vx_dcrs[VX_DCR_BASE_STARTUP_ARG0];                \
    (void)__vx_main_body(vx_ptr<ArgT>(a), __vx_tag, __vx_words);                     \
    if (rows_on) {                                                                   \
      __syncthreads();                                                               \
      if (__vx_dcrs[VX_DCR_HIP_MPM_ROWS] && threadIdx.x < VX_MPM_ROW &&              \
          blockIdx.x < VX_MAX_GRID)                                                  \
        __vx_state.mpm[blockIdx.x][threadIdx.x] = __vx_mpm_lds[threadIdx.x];         \
    }                                                                                \
  }                                                                                  \
  static __device__ __forceinline__ int __vx_main_body(ArgT* argname, uint32_t vx_launch_tag, \
                                                       vx_launch_words_t vx_launch_words)

#endif /* VX_SPAWN_H */
