// common.h -- shared helpers of the runtime (stub + HIP driver).
// Error convention and the CHECK_ERR message follow runtime/common/common.h:44-51.
#pragma once

#include <cstdint>
#include <cstdio>

#define VX_CHECK_ERR(_expr, _cleanup)                                  \
  do {                                                                 \
    auto err = (_expr);                                                \
    if (err == 0) break;                                               \
    std::printf("[VXDRV] Error: '%s' returned %d!\n", #_expr, (int)err); \
    _cleanup                                                           \
  } while (false)

inline uint64_t vx_align_up(uint64_t v, uint64_t a) { return (v + a - 1) & ~(a - 1); }
