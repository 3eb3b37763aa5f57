/*
 * vortex.h -- public host C API of the MI355X-native Vortex/Skybox runtime.
 *
 * Drop-in replacement for the reference's runtime/include/vortex.h:73-139:
 * the same 16 device entry points (served by a driver plugin through
 * callbacks_t, see callbacks.h) plus the 6 stub-side utilities
 * (runtime/stub/utils.cpp:49-155,159-836).  Implemented by
 * skybox_rt_amd/lib/libvortex.so, which dlopens
 * libvortex-${VORTEX_DRIVER:-hip}.so exactly like runtime/stub/vortex.cpp:58-97.
 *
 * Device addresses are driver-defined 64-bit values.  The HIP driver hands out
 * offsets into one device arena starting at USER_BASE_ADDR (0x10000), aligned
 * to 64 B, so `addr / 64` still fits the 32-bit block-address DCRs the apps
 * write (draw3d/main.cpp:216-230).
 *
 * Errors: 0 = success, non-zero (normally -1) = failure.
 */
#ifndef VX_VORTEX_H
#define VX_VORTEX_H

#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* vx_device_h;
typedef void* vx_buffer_h;

/* device caps ids (vortex.h:29-36) */
#define VX_CAPS_VERSION         0x0
#define VX_CAPS_NUM_THREADS     0x1
#define VX_CAPS_NUM_WARPS       0x2
#define VX_CAPS_NUM_CORES       0x3
#define VX_CAPS_CACHE_LINE_SIZE 0x4
#define VX_CAPS_GLOBAL_MEM_SIZE 0x5
#define VX_CAPS_LOCAL_MEM_SIZE  0x6
#define VX_CAPS_ISA_FLAGS       0x7

/* ISA flag bits (hw/rtl/VX_config.vh:943-963) */
#define VX_ISA_EXT_ICACHE  (1ull << (32 + 0))
#define VX_ISA_EXT_DCACHE  (1ull << (32 + 1))
#define VX_ISA_EXT_L2CACHE (1ull << (32 + 2))
#define VX_ISA_EXT_L3CACHE (1ull << (32 + 3))
#define VX_ISA_EXT_LMEM    (1ull << (32 + 4))
#define VX_ISA_EXT_ZICOND  (1ull << (32 + 5))
#define VX_ISA_EXT_TEX     (1ull << (32 + 6))
#define VX_ISA_EXT_RASTER  (1ull << (32 + 7))
#define VX_ISA_EXT_OM      (1ull << (32 + 8))

#define VX_MEM_TYPE_GLOBAL 0
#define VX_MEM_TYPE_LOCAL  1

#define VX_MAX_TIMEOUT (24 * 60 * 60 * 1000) /* 24 h, in ms */

#define VX_MEM_READ       0x1
#define VX_MEM_WRITE      0x2
#define VX_MEM_READ_WRITE 0x3

int vx_dev_open(vx_device_h* hdevice);
int vx_dev_close(vx_device_h hdevice);
int vx_dev_caps(vx_device_h hdevice, uint32_t caps_id, uint64_t* value);

int vx_mem_alloc(vx_device_h hdevice, uint64_t size, int flags, vx_buffer_h* hbuffer);
int vx_mem_reserve(vx_device_h hdevice, uint64_t address, uint64_t size, int flags,
                   vx_buffer_h* hbuffer);
int vx_mem_free(vx_buffer_h hbuffer);
int vx_mem_access(vx_buffer_h hbuffer, uint64_t offset, uint64_t size, int flags);
int vx_mem_address(vx_buffer_h hbuffer, uint64_t* address);
int vx_mem_info(vx_device_h hdevice, uint64_t* mem_free, uint64_t* mem_used);

int vx_copy_to_dev(vx_buffer_h hbuffer, const void* host_ptr, uint64_t dst_offset, uint64_t size);
int vx_copy_from_dev(void* host_ptr, vx_buffer_h hbuffer, uint64_t src_offset, uint64_t size);

/* Asynchronous: launches the kernel image held in `hkernel` with the
 * argument buffer `harguments`; vx_ready_wait() blocks until it finishes. */
int vx_start(vx_device_h hdevice, vx_buffer_h hkernel, vx_buffer_h harguments);
int vx_ready_wait(vx_device_h hdevice, uint64_t timeout);

int vx_dcr_read(vx_device_h hdevice, uint32_t addr, uint32_t* value);
int vx_dcr_write(vx_device_h hdevice, uint32_t addr, uint32_t value);

/* HIP driver: VX_CSR_MCYCLE = device time of the last run in ns (reported on
 * core 0), VX_CSR_MINSTRET = callback invocations (tasks) of the last run. */
int vx_mpm_query(vx_device_h hdevice, uint32_t addr, uint32_t core_id, uint64_t* value);

/* ---- utilities (runtime/stub/utils.cpp) ---- */
int vx_upload_kernel_bytes(vx_device_h hdevice, const void* content, uint64_t size,
                           vx_buffer_h* hbuffer);
int vx_upload_kernel_file(vx_device_h hdevice, const char* filename, vx_buffer_h* hbuffer);
int vx_upload_bytes(vx_device_h hdevice, const void* content, uint64_t size,
                    vx_buffer_h* hbuffer);
int vx_upload_file(vx_device_h hdevice, const char* filename, vx_buffer_h* hbuffer);
int vx_check_occupancy(vx_device_h hdevice, uint32_t group_size, uint32_t* max_localmem);
int vx_dump_perf(vx_device_h hdevice, FILE* stream);

#ifdef __cplusplus
}
#endif

#endif /* VX_VORTEX_H */
