/*
 * vortex_hip.h -- HIP-driver extensions beyond the reference ABI.
 *
 * These are NOT part of runtime/include/vortex.h; they exist so a host app can
 * hand device buffers to PyTorch/RCCL (framebuffer gather) and
 * read per-launch device timing.  Resolve them through vx_driver_symbol()
 * (exported by libvortex.so) so the driver stays a plain dlopen plugin.
 */
#ifndef VX_VORTEX_HIP_H
#define VX_VORTEX_HIP_H

#include "vortex.h"

#ifdef __cplusplus
extern "C" {
#endif

/* libvortex.so: dlsym() in the loaded driver (NULL if absent). */
void* vx_driver_symbol(const char* name);

/* libvortex-hip.so extensions */
typedef int (*vx_hip_mem_ptr_t)(vx_buffer_h hbuffer, void** device_ptr);
typedef int (*vx_hip_stream_t)(vx_device_h hdevice, void** hip_stream);
typedef int (*vx_hip_last_run_t)(vx_device_h hdevice, double* kernel_ms,
                                 uint32_t* grid, uint32_t* block);
typedef int (*vx_hip_device_id_t)(vx_device_h hdevice, int* device_id);
/* waits for every queued run, then, since the device opened: the summed
 * event-timed kernel durations, the number of timed runs and of all runs.
 * A start() behind an in-flight run queues instead of blocking
 * (VX_HIP_QUEUE_DEPTH, default 2); queued runs are timed one in
 * VX_HIP_TIME_EVERY (default 4), a run started on an idle queue always. */
typedef int (*vx_hip_run_totals_t)(vx_device_h hdevice, double* kernel_ms_sum,
                                   uint64_t* timed_runs, uint64_t* runs);
/* the last launch's raw per-workgroup counter rows (vx_spawn.h: 16 u32 per
 * workgroup, in blockIdx order): copies min(grid, max_rows) rows to `rows`,
 * *nrows = grid.  Diagnostics (e.g. in-kernel timestamps). */
typedef int (*vx_hip_mpm_rows_t)(vx_device_h hdevice, uint32_t* rows, uint64_t max_rows,
                                 uint64_t* nrows);
/* per-block counter rows on (1) / off (0, the default): with them off a
 * launch writes no counters -- vx_mpm_query returns its spawned task count
 * for VX_CSR_MINSTRET, device time for VX_CSR_MCYCLE and 0 otherwise.
 * VORTEX_PROFILING (the stub's MPM_CLASS DCR) or env VX_HIP_COUNTERS=1 turn
 * them on as well. */
typedef int (*vx_hip_set_counters_t)(vx_device_h hdevice, int enable);
/* the next n (1..4) vx_start launches form one run -- a frame made of
 * several kernels on the driver's stream: timed as a whole (start event on
 * its first launch, stop event on its last: the frame's span), counted as
 * one run by vx_hip_run_totals / vx_hip_last_run, and vx_mpm_query sums the
 * counters of all its launches; then launches are single runs again.  Only
 * between groups (-1 inside one, or when (VX_HIP_QUEUE_DEPTH +
 * VX_HIP_TIME_EVERY) * n exceeds the driver's 64 in-flight slots); never
 * waits.  n = 0 abandons an open group after a failed launch inside it: the
 * launches already issued retire as one untimed run. */
typedef int (*vx_hip_launch_group_t)(vx_device_h hdevice, uint32_t n);
/* n | VX_HIP_GROUP_UNTIMED: the group runs without events (no timing, no
 * idle gap an event costs) and may hold up to 64 / (VX_HIP_QUEUE_DEPTH +
 * VX_HIP_TIME_EVERY) launches (10 by default) -- a stream-ordered sequence
 * such as the RT app's device setup (app/device_setup.cpp run_seq) */
#define VX_HIP_GROUP_UNTIMED 0x80000000u
/* the device's pinned host buffer (up to 64 KiB, allocated on first use,
 * freed with the device), mapped for the device: *host for the host,
 * *device_addr (a raw 64-bit device pointer, not an arena address) for
 * kernels.  A kernel's stores to it are visible once the host has waited for
 * the run (vx_ready_wait): small results come back without a copy. */
typedef int (*vx_hip_host_mem_t)(vx_device_h hdevice, uint64_t size, void** host, uint64_t* device_addr);
/* timed (1, the default: HIP events on one run in VX_HIP_TIME_EVERY, queue
 * depth VX_HIP_QUEUE_DEPTH) or untimed (0: no events and no queue bound, so
 * back-to-back starts reach the GPU without the idle gap an event costs --
 * for timing a run of launches by a host clock).  Waits for the device. */
typedef int (*vx_hip_set_timing_t)(vx_device_h hdevice, int timed);
/* vx_copy_to_dev without the wait: the bytes (at most 4 KiB; larger copies,
 * and copies into a kernel image, fall back to the synchronous copy) are
 * staged in pinned host memory at once and copied when the driver's stream
 * reaches the copy -- after every vx_start issued before it, before every
 * one issued after it.  `src` may be reused when the call returns.  (simx's
 * copies wait for the device, runtime/simx/vortex.cpp:174-176; a setup chain
 * of dependent launches needs only stream order.) */
typedef int (*vx_hip_copy_to_dev_async_t)(vx_buffer_h hbuf, const void* src, uint64_t off, uint64_t size);
/* the kernel argument of the next vx_start (then 0 again): every image's
 * entry takes a u32 tag, `vx_launch_tag` in its VX_MAIN body (vx_spawn.h) --
 * how the launches of a sequence sharing one argument block tell themselves
 * apart without a device counter or a copy between them */
typedef int (*vx_hip_set_launch_tag_t)(vx_device_h hdevice, uint32_t tag);
/* which clock timed the runs vx_hip_last_run / vx_hip_run_totals report:
 * `last_stamped` 1 when the last timed run was timed by its completion
 * kernel's stamps (a run started on an idle queue: block 0's start to the
 * completion kernel's start, so the kernel plus its launch boundary), 0 by
 * HIP events on the dispatch (queued runs: the kernel alone); the counts of
 * timed runs of each kind since the device opened (their sum is
 * vx_hip_run_totals' timed count, and the total mixes both kinds when both
 * are non-zero) */
typedef int (*vx_hip_timing_source_t)(vx_device_h hdevice, int* last_stamped, uint64_t* stamped_runs,
                                      uint64_t* event_runs);
/* the four launch words of the next vx_start (then 0 again; n <= 4, the rest
 * 0): carried in the dispatch's kernel arguments beside the tag,
 * `vx_launch_words` in the VX_MAIN body -- per-launch values (a frame's light)
 * that reach the kernel with its dispatch packet instead of through a copy
 * queued between two launches */
typedef int (*vx_hip_set_launch_words_t)(vx_device_h hdevice, const uint32_t* words, uint32_t n);

#ifdef __cplusplus
}
#endif

#endif
