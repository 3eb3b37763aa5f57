"""ctypes binding of include/vortex.h (libvortex.so).

Mirrors the reference's host API (runtime/include/vortex.h:73-139): every
call returns the C error code and failures raise VortexError, the way the
regression apps wrap calls in RT_CHECK (draw3d/main.cpp:23-31).
"""
from __future__ import annotations

import ctypes as C

from . import _lib

VX_CAPS_VERSION = 0x0
VX_CAPS_NUM_THREADS = 0x1
VX_CAPS_NUM_WARPS = 0x2
VX_CAPS_NUM_CORES = 0x3
VX_CAPS_CACHE_LINE_SIZE = 0x4
VX_CAPS_GLOBAL_MEM_SIZE = 0x5
VX_CAPS_LOCAL_MEM_SIZE = 0x6
VX_CAPS_ISA_FLAGS = 0x7
VX_ISA_EXT_TEX = 1 << (32 + 6)
VX_ISA_EXT_RASTER = 1 << (32 + 7)
VX_ISA_EXT_OM = 1 << (32 + 8)
VX_MEM_READ, VX_MEM_WRITE, VX_MEM_READ_WRITE = 1, 2, 3
VX_MAX_TIMEOUT = 24 * 60 * 60 * 1000
VX_CSR_MCYCLE = 0xB00
VX_CSR_MINSTRET = 0xB02
VX_DCR_BASE_STARTUP_ADDR0 = 0x001
VX_DCR_BASE_STARTUP_ARG0 = 0x003
VX_DCR_BASE_MPM_CLASS = 0x005

# every entry point declared in include/vortex.h (+ the vortex_hip.h hook)
API = {
    "vx_dev_open": [C.POINTER(C.c_void_p)],
    "vx_dev_close": [C.c_void_p],
    "vx_dev_caps": [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint64)],
    "vx_mem_alloc": [C.c_void_p, C.c_uint64, C.c_int, C.POINTER(C.c_void_p)],
    "vx_mem_reserve": [C.c_void_p, C.c_uint64, C.c_uint64, C.c_int, C.POINTER(C.c_void_p)],
    "vx_mem_free": [C.c_void_p],
    "vx_mem_access": [C.c_void_p, C.c_uint64, C.c_uint64, C.c_int],
    "vx_mem_address": [C.c_void_p, C.POINTER(C.c_uint64)],
    "vx_mem_info": [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)],
    "vx_copy_to_dev": [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64],
    "vx_copy_from_dev": [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64],
    "vx_start": [C.c_void_p, C.c_void_p, C.c_void_p],
    "vx_ready_wait": [C.c_void_p, C.c_uint64],
    "vx_dcr_read": [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)],
    "vx_dcr_write": [C.c_void_p, C.c_uint32, C.c_uint32],
    "vx_mpm_query": [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64)],
    "vx_upload_kernel_bytes": [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_void_p)],
    "vx_upload_kernel_file": [C.c_void_p, C.c_char_p, C.POINTER(C.c_void_p)],
    "vx_upload_bytes": [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_void_p)],
    "vx_upload_file": [C.c_void_p, C.c_char_p, C.POINTER(C.c_void_p)],
    "vx_check_occupancy": [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)],
    "vx_dump_perf": [C.c_void_p, C.c_void_p],
}


class VortexError(RuntimeError):
    pass


_lib_handle = None


def lib():
    global _lib_handle
    if _lib_handle is None:
        h = _lib.load("libvortex.so")
        for name, argtypes in API.items():
            fn = getattr(h, name)
            fn.argtypes = argtypes
            fn.restype = C.c_int
        h.vx_driver_symbol.argtypes = [C.c_char_p]
        h.vx_driver_symbol.restype = C.c_void_p
        _lib_handle = h
    return _lib_handle


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise VortexError(f"{what} returned {rc}")


class Buffer:
    def __init__(self, dev: "Device", handle: C.c_void_p, size: int):
        self.dev, self.handle, self.size = dev, handle, size

    @property
    def address(self) -> int:
        a = C.c_uint64()
        check(lib().vx_mem_address(self.handle, C.byref(a)), "vx_mem_address")
        return a.value

    def write(self, data, offset: int = 0) -> None:
        buf = bytes(data)
        check(lib().vx_copy_to_dev(self.handle, buf, offset, len(buf)), "vx_copy_to_dev")

    def read(self, size: int = None, offset: int = 0) -> bytes:
        n = self.size - offset if size is None else size
        out = C.create_string_buffer(n)
        check(lib().vx_copy_from_dev(out, self.handle, offset, n), "vx_copy_from_dev")
        return out.raw

    def free(self) -> None:
        if self.handle:
            lib().vx_mem_free(self.handle)
            self.handle = None


class Device:
    """One vortex device (vx_dev_open .. vx_dev_close)."""

    def __init__(self):
        h = C.c_void_p()
        check(lib().vx_dev_open(C.byref(h)), "vx_dev_open")
        self.handle = h

    def caps(self, cid: int) -> int:
        v = C.c_uint64()
        check(lib().vx_dev_caps(self.handle, cid, C.byref(v)), "vx_dev_caps")
        return v.value

    def mem_alloc(self, size: int, flags: int = VX_MEM_READ_WRITE) -> Buffer:
        b = C.c_void_p()
        check(lib().vx_mem_alloc(self.handle, size, flags, C.byref(b)), "vx_mem_alloc")
        return Buffer(self, b, size)

    def upload_bytes(self, data) -> Buffer:
        buf = bytes(data)
        b = C.c_void_p()
        check(lib().vx_upload_bytes(self.handle, buf, len(buf), C.byref(b)), "vx_upload_bytes")
        return Buffer(self, b, len(buf))

    def upload_kernel_file(self, path: str) -> Buffer:
        b = C.c_void_p()
        check(lib().vx_upload_kernel_file(self.handle, path.encode(), C.byref(b)),
              "vx_upload_kernel_file")
        return Buffer(self, b, 0)

    def dcr_write(self, addr: int, value: int) -> None:
        check(lib().vx_dcr_write(self.handle, addr, value), "vx_dcr_write")

    def dcr_read(self, addr: int) -> int:
        v = C.c_uint32()
        check(lib().vx_dcr_read(self.handle, addr, C.byref(v)), "vx_dcr_read")
        return v.value

    def start(self, kernel: Buffer, args: Buffer) -> None:
        check(lib().vx_start(self.handle, kernel.handle, args.handle), "vx_start")

    def ready_wait(self, timeout_ms: int = VX_MAX_TIMEOUT) -> None:
        check(lib().vx_ready_wait(self.handle, timeout_ms), "vx_ready_wait")

    def mpm_query(self, addr: int, core: int = 0xFFFFFFFF) -> int:
        v = C.c_uint64()
        check(lib().vx_mpm_query(self.handle, addr, core, C.byref(v)), "vx_mpm_query")
        return v.value

    def mem_info(self):
        fr, used = C.c_uint64(), C.c_uint64()
        check(lib().vx_mem_info(self.handle, C.byref(fr), C.byref(used)), "vx_mem_info")
        return fr.value, used.value

    def close(self) -> None:
        if self.handle:
            lib().vx_dev_close(self.handle)
            self.handle = None
