"""Loader for the in-tree native libraries (skybox_rt_amd/lib/).

The product path is native: libvortex.so (vortex.h API), libvortex-hip.so
(the MI355X driver plugin) and librtapp.so (the RT host app, vx_rt.h).  There
is no Python or CPU fallback: if a library or kernel image is missing, loading
raises NativeLibraryMissing.

One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so (same
soname, libamdhip64.so.7).  If torch is importable it is imported *before* our
libraries so that their libamdhip64.so.7 dependency binds to the copy torch
already loaded (device pointers and streams can then be shared with
torch.distributed / RCCL).  Set SKYBOX_RT_NO_TORCH=1 to skip that.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(PKG_DIR, "lib")
CSRC_DIR = os.path.join(PKG_DIR, "csrc")

REQUIRED = ("libvortex.so", "libvortex-hip.so", "librtapp.so", "rtapp",
            "rt_kernel.vxbin", "rt_kernel_stats.vxbin", "rt_kernel_deep.vxbin",
            "rt_kernel_deep_stats.vxbin", "spawn_test.vxbin", "edge_kat.vxbin", "pt_kernel.vxbin",
            "pt_kernel_deep.vxbin", "pt_kernel_stats.vxbin", "pt_kernel_deep_stats.vxbin",
            "rt_flat.vxbin", "rt_flat_stats.vxbin", "raster_kernel.vxbin",
            "pt_compact/pt_kernel.vxbin", "pt_compact/pt_kernel_stats.vxbin",
            "tex_kernel_f0.vxbin", "tex_kernel_f1.vxbin", "tex_kernel_f2.vxbin", "texapp", "bvh_build.vxbin",
            "librt_shard.so", "rt_setup.vxbin", "bvh_sah.vxbin", "om.vxbin", "omapp", "rasterapp",
            "pt_primary.vxbin", "pt_primary_stats.vxbin", "pt_queue.vxbin", "pt_queue_stats.vxbin")


class NativeLibraryMissing(RuntimeError):
    pass


def build(jobs: int = 8) -> None:
    """Compile the runtime, app and gfx950 kernel images in-tree."""
    subprocess.check_call(["make", "-s", "-C", CSRC_DIR, f"-j{jobs}"])


def missing() -> list:
    return [f for f in REQUIRED if not os.path.exists(os.path.join(LIB_DIR, f))]


_torch_checked = False


def _bind_torch_runtime() -> None:
    global _torch_checked
    if _torch_checked or os.environ.get("SKYBOX_RT_NO_TORCH"):
        return
    _torch_checked = True
    try:
        import torch  # noqa: F401  (loads torch's libamdhip64.so.7 first)
    except Exception:  # torch absent: the libraries use /opt/rocm's runtime
        pass


_handles = {}


def load(name: str) -> ctypes.CDLL:
    if name in _handles:
        return _handles[name]
    miss = missing()
    if miss:
        raise NativeLibraryMissing(
            f"native build incomplete in {LIB_DIR}: missing {miss}; run "
            f"`python -c 'import __graft_entry__ as g; g.build()'` or `make -C {CSRC_DIR}`")
    _bind_torch_runtime()
    h = ctypes.CDLL(os.path.join(LIB_DIR, name), mode=ctypes.RTLD_GLOBAL)
    _handles[name] = h
    return h
