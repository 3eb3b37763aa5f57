"""skybox_rt_amd -- MI355X-native Vortex/Skybox ray-tracing hot path.

Layers:
  include/vortex.h, callbacks.h  drop-in host API + driver ABI (C)
  lib/libvortex.so               API stub, loads libvortex-${VORTEX_DRIVER:-hip}.so
  lib/libvortex-hip.so           MI355X driver plugin (HBM arena, HIP launch)
  lib/rt_kernel.vxbin            gfx950 kernel image: raygen + BVH + MT + shade + shadow
  lib/librtapp.so, lib/rtapp     RT host app (include/vx_rt.h) and its CLI
  rt.py / vortex.py              ctypes bindings used by tests and bench.py
"""
from ._lib import NativeLibraryMissing, build, missing  # noqa: F401

__all__ = ["NativeLibraryMissing", "build", "missing"]
