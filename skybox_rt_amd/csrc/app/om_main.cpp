// om_main.cpp -- omapp: the render-output (OM) regression app
// (tests/regression/om/main.cpp) on the public vortex.h API and the MI355X
// driver, kernel image om.vxbin (kernels/om_kernel.hip).
//
// Same flags (om/main.cpp:78-125: -c colour, -d depth test, -b blend, -f
// back face, -k kernel file, -o output, -r reference, -w/-h size, -z), the
// same host sequence (caps -> num_tasks = cores x warps x threads, kernel
// upload, depth buffer cleared to the 0.0 / 0.99 checkerboard, colour buffer
// to 0, OM DCR state of :153-190, start, wait, read back, save flipped) and
// the same verdict lines ("PASSED!" / "FAILED!", exit code = the error count).
// The default kernel file is om.vxbin beside this executable (the reference's
// default is kernel.vxbin in the working directory); the reference image
// resolves through RT_ASSETS_PATHS like ResolveFilePath (app/assets.h).
#include <getopt.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "VX_types.h"
#include "assets.h"
#include "png.h"
#include "vortex.h"

namespace {

std::string kernel_file;
const char* output_file = "output.png";
const char* reference_file = nullptr;
uint32_t color = 0xffffffffu;
const uint32_t kDepthHalf = 0x00800000u;  // TFixed<24>(0.5f).data()
uint32_t depth = kDepthHalf;
bool blend_enable = false, depth_enable = false, backface = false, use_sw = false;
const uint32_t clear_color = 0x00000000u;
uint32_t dst_width = 128, dst_height = 128;

// kernel_arg_t of om/common.h (kernels/om_kernel.hip om_arg_t)
struct OmArg {
  uint32_t num_tasks, dst_width, dst_height, color, depth;
  bool backface, blend_enable, use_sw;
};

vx_device_h device = nullptr;
vx_buffer_h krnl_buffer = nullptr, args_buffer = nullptr, depth_buffer = nullptr,
            color_buffer = nullptr;

void cleanup() {
  vx_mem_free(depth_buffer);
  vx_mem_free(color_buffer);
  vx_mem_free(krnl_buffer);
  vx_mem_free(args_buffer);
  vx_dev_close(device);
}

#define RT_CHECK(_expr)                                         \
  do {                                                          \
    int _ret = (_expr);                                         \
    if (_ret == 0) break;                                       \
    std::printf("Error: '%s' returned %d!\n", #_expr, _ret);    \
    cleanup();                                                  \
    std::exit(-1);                                              \
  } while (false)

void usage() {
  std::printf("Vortex Render Output Test.\n"
              "Usage: [-c color] [-d depth] [-b blend] [-f face] [-k: kernel] [-o image] "
              "[-r reference] [-w width] [-h height] [-z no_hw]\n");
}

std::string exe_dir() {
  char buf[4096];
  const ssize_t n = readlink("/proc/self/exe", buf, sizeof(buf) - 1);
  if (n <= 0) return ".";
  buf[n] = 0;
  std::string p(buf);
  const size_t k = p.rfind('/');
  return k == std::string::npos ? "." : p.substr(0, k);
}

// TFixed<24>(f).data(): truncating float -> Q.24 (pinned by the draw3d goldens)
uint32_t fixed24(float f) { return (uint32_t)(int32_t)(f * 16777216.0f); }

}  // namespace

int main(int argc, char** argv) {
  kernel_file = exe_dir() + "/om.vxbin";
  int c;
  while ((c = getopt(argc, argv, "o:r:k:w:h:c:bdfz?")) != -1) {
    switch (c) {
    case 'o': output_file = optarg; break;
    case 'r': reference_file = optarg; break;
    case 'k': kernel_file = optarg; break;
    case 'w': dst_width = (uint32_t)std::atoi(optarg); break;
    case 'h': dst_height = (uint32_t)std::atoi(optarg); break;
    case 'f': backface = true; break;
    case 'c': color = (uint32_t)std::atoi(optarg); break;
    case 'd': depth_enable = true; break;
    case 'b': blend_enable = true; break;
    case 'z': use_sw = true; break;
    case '?': usage(); return 0;
    default: usage(); return -1;
    }
  }
  if (std::strcmp(output_file, "null") == 0 && reference_file) {
    std::printf("Error: the output file is missing for reference validation!\n");
    return 1;
  }
  RT_CHECK(vx_dev_open(&device));
  uint64_t isa_flags = 0;
  RT_CHECK(vx_dev_caps(device, VX_CAPS_ISA_FLAGS, &isa_flags));
  if ((isa_flags & VX_ISA_EXT_OM) == 0) {
    std::printf("OM extension not supported!\n");
    cleanup();
    return -1;
  }
  std::printf("using color=%x, depth=%x\n", color, depth);
  uint64_t num_cores = 0, num_warps = 0, num_threads = 0;
  RT_CHECK(vx_dev_caps(device, VX_CAPS_NUM_CORES, &num_cores));
  RT_CHECK(vx_dev_caps(device, VX_CAPS_NUM_WARPS, &num_warps));
  RT_CHECK(vx_dev_caps(device, VX_CAPS_NUM_THREADS, &num_threads));
  const uint32_t num_tasks = (uint32_t)(num_cores * num_warps * num_threads);
  std::printf("number of tasks: %u\n", num_tasks);
  RT_CHECK(vx_upload_kernel_file(device, kernel_file.c_str(), &krnl_buffer));

  const uint32_t pitch = dst_width * 4u, size = dst_height * pitch;
  uint64_t zbuf_addr = 0, cbuf_addr = 0;
  RT_CHECK(vx_mem_alloc(device, size, VX_MEM_READ_WRITE, &depth_buffer));
  RT_CHECK(vx_mem_address(depth_buffer, &zbuf_addr));
  RT_CHECK(vx_mem_alloc(device, size, VX_MEM_READ_WRITE, &color_buffer));
  RT_CHECK(vx_mem_address(color_buffer, &cbuf_addr));
  {  // depth: 0.0 where x and y have equal parity, 0.99 elsewhere (om/main.cpp:265-275)
    std::vector<uint32_t> z((size_t)dst_width * dst_height);
    for (uint32_t y = 0; y < dst_height; ++y)
      for (uint32_t x = 0; x < dst_width; ++x)
        z[x + (size_t)y * dst_width] = ((x & 1u) == (y & 1u)) ? fixed24(0.0f) : fixed24(0.99f);
    RT_CHECK(vx_copy_to_dev(depth_buffer, z.data(), 0, size));
    std::vector<uint32_t> col((size_t)dst_width * dst_height, clear_color);
    RT_CHECK(vx_copy_to_dev(color_buffer, col.data(), 0, size));
  }
  OmArg arg = {num_tasks, dst_width, dst_height, color, depth, backface, blend_enable, use_sw};
  RT_CHECK(vx_upload_bytes(device, &arg, sizeof(arg), &args_buffer));

  // OM state (om/main.cpp:153-190; STENCIL_ZPASS written twice as there)
  vx_dcr_write(device, VX_DCR_OM_CBUF_ADDR, (uint32_t)(cbuf_addr / 64));
  vx_dcr_write(device, VX_DCR_OM_CBUF_PITCH, pitch);
  vx_dcr_write(device, VX_DCR_OM_CBUF_WRITEMASK, 0xf);
  vx_dcr_write(device, VX_DCR_OM_ZBUF_ADDR, (uint32_t)(zbuf_addr / 64));
  vx_dcr_write(device, VX_DCR_OM_ZBUF_PITCH, pitch);
  vx_dcr_write(device, VX_DCR_OM_DEPTH_FUNC,
               depth_enable ? VX_OM_DEPTH_FUNC_LESS : VX_OM_DEPTH_FUNC_ALWAYS);
  vx_dcr_write(device, VX_DCR_OM_DEPTH_WRITEMASK, depth_enable ? 1 : 0);
  vx_dcr_write(device, VX_DCR_OM_STENCIL_FUNC, VX_OM_DEPTH_FUNC_ALWAYS);
  vx_dcr_write(device, VX_DCR_OM_STENCIL_ZPASS, VX_OM_STENCIL_OP_KEEP);
  vx_dcr_write(device, VX_DCR_OM_STENCIL_ZPASS, VX_OM_STENCIL_OP_KEEP);
  vx_dcr_write(device, VX_DCR_OM_STENCIL_FAIL, VX_OM_STENCIL_OP_KEEP);
  vx_dcr_write(device, VX_DCR_OM_STENCIL_REF, 0);
  vx_dcr_write(device, VX_DCR_OM_STENCIL_MASK, VX_OM_STENCIL_MASK);
  vx_dcr_write(device, VX_DCR_OM_STENCIL_WRITEMASK, 0);
  vx_dcr_write(device, VX_DCR_OM_BLEND_MODE, (VX_OM_BLEND_MODE_ADD << 16) | VX_OM_BLEND_MODE_ADD);
  if (blend_enable)
    vx_dcr_write(device, VX_DCR_OM_BLEND_FUNC,
                 (VX_OM_BLEND_FUNC_ONE_MINUS_SRC_A << 24) | (VX_OM_BLEND_FUNC_ONE_MINUS_SRC_A << 16) |
                     (VX_OM_BLEND_FUNC_ONE << 8) | VX_OM_BLEND_FUNC_ONE);
  else
    vx_dcr_write(device, VX_DCR_OM_BLEND_FUNC,
                 (VX_OM_BLEND_FUNC_ZERO << 24) | (VX_OM_BLEND_FUNC_ZERO << 16) |
                     (VX_OM_BLEND_FUNC_ONE << 8) | VX_OM_BLEND_FUNC_ONE);

  const auto t0 = std::chrono::high_resolution_clock::now();
  RT_CHECK(vx_start(device, krnl_buffer, args_buffer));
  RT_CHECK(vx_ready_wait(device, VX_MAX_TIMEOUT));
  const auto t1 = std::chrono::high_resolution_clock::now();
  std::printf("Elapsed time: %g ms\n", std::chrono::duration<double, std::milli>(t1 - t0).count());

  int errors = 0;
  if (std::strcmp(output_file, "null") != 0) {
    std::vector<uint32_t> fb((size_t)dst_width * dst_height);
    RT_CHECK(vx_copy_from_dev(fb.data(), color_buffer, 0, size));
    RT_CHECK(rt::SavePngARGB(output_file, fb.data(), dst_width, dst_height));
  }
  cleanup();
  if (reference_file) {
    std::vector<uint32_t> out, ref;
    uint32_t ow = 0, oh = 0, rw = 0, rh = 0;
    if (rt::LoadPngARGB(output_file, &out, &ow, &oh) || rt::LoadPngARGB(rt::ResolveAsset(reference_file), &ref, &rw, &rh) ||
        ow != rw || oh != rh) {
      std::printf("FAILED!\n");
      return -1;
    }
    errors = (int)rt::CompareARGB(out.data(), ref.data(), out.size(), 1);
    std::printf(errors == 0 ? "PASSED!\n" : "FAILED!\n");
  }
  return errors;
}
