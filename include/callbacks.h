/*
 * callbacks.h -- the driver-plugin ABI (replaces runtime/common/callbacks.h:23-75).
 *
 * A driver is a shared library libvortex-<name>.so exporting one C symbol,
 * vx_dev_init(callbacks_t*), which fills the 16 function pointers below.
 * The stub (libvortex.so) resolves it with dlsym after dlopen
 * (runtime/stub/vortex.cpp:58-97).  libvortex-hip.so is the MI355X driver and
 * takes the place of libvortex-{simx,rtlsim,opae,xrt}.so.
 */
#ifndef VX_CALLBACKS_H
#define VX_CALLBACKS_H

#include "vortex.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int (*dev_open)(vx_device_h* hdevice);
  int (*dev_close)(vx_device_h hdevice);
  int (*dev_caps)(vx_device_h hdevice, uint32_t caps_id, uint64_t* value);
  int (*mem_alloc)(vx_device_h hdevice, uint64_t size, int flags, vx_buffer_h* hbuffer);
  int (*mem_reserve)(vx_device_h hdevice, uint64_t address, uint64_t size, int flags,
                     vx_buffer_h* hbuffer);
  int (*mem_free)(vx_buffer_h hbuffer);
  int (*mem_access)(vx_buffer_h hbuffer, uint64_t offset, uint64_t size, int flags);
  int (*mem_address)(vx_buffer_h hbuffer, uint64_t* address);
  int (*mem_info)(vx_device_h hdevice, uint64_t* mem_free, uint64_t* mem_used);
  int (*copy_to_dev)(vx_buffer_h hbuffer, const void* host_ptr, uint64_t dst_offset,
                     uint64_t size);
  int (*copy_from_dev)(void* host_ptr, vx_buffer_h hbuffer, uint64_t src_offset,
                       uint64_t size);
  int (*start)(vx_device_h hdevice, vx_buffer_h hkernel, vx_buffer_h harguments);
  int (*ready_wait)(vx_device_h hdevice, uint64_t timeout);
  int (*dcr_read)(vx_device_h hdevice, uint32_t addr, uint32_t* value);
  int (*dcr_write)(vx_device_h hdevice, uint32_t addr, uint32_t value);
  int (*mpm_query)(vx_device_h hdevice, uint32_t addr, uint32_t core_id, uint64_t* value);
} callbacks_t;

int vx_dev_init(callbacks_t* callbacks);

#ifdef __cplusplus
}
#endif

#endif /* VX_CALLBACKS_H */
