"""Python binding of the texture regression app (include/vx_tex.h,
librtapp.so): the reference's tests/regression/tex host (image conversion,
mip chain, TEX state, launch, read-back) with tex_kernel_f{0,1,2}.vxbin on MI355X.
No CPU fallback: every call goes through the native library."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .rt import RtError, lib as _rtlib

FORMATS = {"A8R8G8B8": 0, "R5G6B5": 1, "A1R5G5B5": 2, "A4R4G4B4": 3, "A8L8": 4, "L8": 5, "A8": 6}
WRAP_CLAMP, WRAP_REPEAT, WRAP_MIRROR = 0, 1, 2


class TexParams(C.Structure):
    _fields_ = [("format", C.c_uint32), ("filter", C.c_uint32), ("wrap", C.c_uint32),
                ("scale", C.c_float), ("num_tasks", C.c_uint32)]


class TexStats(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("dst_width", "dst_height", "lod", "frac", "levels",
                                         "num_tasks")] + [
        ("texture_bytes", C.c_uint64), ("pixels", C.c_uint64), ("kernel_ms", C.c_double),
        ("grid", C.c_uint32), ("block", C.c_uint32)]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


_sig_done = False


def lib():
    global _sig_done
    h = _rtlib()
    if not _sig_done:
        vp, u32, u64 = C.c_void_p, C.c_uint32, C.c_uint64
        sig = {
            "rt_tex_build_image": [vp, u32, u32, u32, vp, C.POINTER(u64), vp, C.POINTER(u32)],
            "rt_tex_create": [C.c_char_p, C.POINTER(vp)],
            "rt_tex_free": [vp],
            "rt_tex_configure": [vp, vp, u32, u32, C.POINTER(TexParams)],
            "rt_tex_render": [vp],
            "rt_tex_stats": [vp, C.POINTER(TexStats)],
            "rt_tex_read": [vp, vp, u64],
        }
        for name, args in sig.items():
            f = getattr(h, name)
            f.argtypes = args
            f.restype = C.c_int
        _sig_done = True
    return h


def _check(rc, what):
    if rc != 0:
        raise RtError(f"{what} failed: {_rtlib().rt_last_error().decode()}")


def build_image(argb: np.ndarray, fmt: int):
    """Host LoadImage conversion + mip chain: (texels uint8[], mipoff uint32[16], levels)."""
    argb = np.ascontiguousarray(argb, np.uint32)
    h, w = argb.shape
    size, levels = C.c_uint64(0), C.c_uint32(0)
    mip = np.zeros(16, np.uint32)
    _check(lib().rt_tex_build_image(argb.ctypes.data, w, h, fmt, None, C.byref(size),
                                    mip.ctypes.data, C.byref(levels)), "rt_tex_build_image")
    out = np.zeros(max(size.value, 1), np.uint8)
    _check(lib().rt_tex_build_image(argb.ctypes.data, w, h, fmt, out.ctypes.data, C.byref(size),
                                    mip.ctypes.data, C.byref(levels)), "rt_tex_build_image")
    return out[:size.value], mip, levels.value


class TexApp:
    """One device + the tex_kernel_f* images; configure() uploads a texture and the
    destination state, render() runs one launch."""

    def __init__(self, kernel_dir: str | None = None):
        _lib.load("librtapp.so")
        h = C.c_void_p()
        _check(lib().rt_tex_create(kernel_dir.encode() if kernel_dir else None, C.byref(h)),
               "rt_tex_create")
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            lib().rt_tex_free(self._h)
            self._h = None

    def configure(self, argb: np.ndarray, fmt: int = 0, filt: int = 0, wrap: int = 0,
                  scale: float = 1.0, num_tasks: int = 0) -> None:
        argb = np.ascontiguousarray(argb, np.uint32)
        self._src = argb
        p = TexParams(fmt, filt, wrap, scale, num_tasks)
        _check(lib().rt_tex_configure(self._h, argb.ctypes.data, argb.shape[1], argb.shape[0],
                                      C.byref(p)), "rt_tex_configure")

    def render(self) -> None:
        _check(lib().rt_tex_render(self._h), "rt_tex_render")

    def stats(self) -> dict:
        s = TexStats()
        _check(lib().rt_tex_stats(self._h, C.byref(s)), "rt_tex_stats")
        return s.as_dict()

    def image(self) -> np.ndarray:
        st = self.stats()
        out = np.zeros((st["dst_height"], st["dst_width"]), np.uint32)
        _check(lib().rt_tex_read(self._h, out.ctypes.data, out.size), "rt_tex_read")
        return out
