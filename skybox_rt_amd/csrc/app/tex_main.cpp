// tex_main.cpp -- texapp: CLI of the texture regression app with the flags
// of the reference's tests/regression/tex/main.cpp:49-117
//   -i image  -o image|null  -r reference  -s scale  -w wrap  -f format
//   -g filter  -z (software sampler: the same sampler here)  -k kernel dir
// Prints "PASSED!" / "FAILED! N errors." against -r like the reference
// (tolerance 1, CompareImages); exit status = error count.
#include <getopt.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "assets.h"
#include "png.h"
#include "vx_rt.h"
#include "vx_tex.h"

namespace {

void usage() {
  std::printf("Vortex Texture Test.\nUsage: [-k: kernel dir] [-i image] [-o image] [-r reference] "
              "[-s scale] [-w wrap] [-f format] [-g filter] [-z no_hw] [-h: help]\n");
}

#define CHECK(expr)                                                                  \
  do {                                                                               \
    if ((expr) != 0) {                                                               \
      std::printf("Error: '%s' failed: %s\n", #expr, rt_last_error());               \
      return -1;                                                                     \
    }                                                                                \
  } while (0)

}  // namespace

int main(int argc, char** argv) {
  std::string input = "palette64.png", output = "output.png", reference, kdir;
  rt_tex_params_t p{};
  p.scale = 1.0f;
  int c;
  while ((c = getopt(argc, argv, "zi:o:k:w:f:g:s:r:h?")) != -1) {
    switch (c) {
      case 'i': input = optarg; break;
      case 'o': output = optarg; break;
      case 'r': reference = optarg; break;
      case 's': p.scale = std::strtof(optarg, nullptr); break;
      case 'w': p.wrap = (uint32_t)std::atoi(optarg); break;
      case 'z': break;  // software sampler: one sampler implementation here
      case 'f':
        p.format = (uint32_t)std::atoi(optarg);
        if (p.format > 6) {
          std::printf("Error: invalid format: %u\n", p.format);
          return 1;
        }
        break;
      case 'g': p.filter = (uint32_t)std::atoi(optarg); break;
      case 'k': {
        kdir = optarg;  // a directory, or the kernel file itself
        const auto n = kdir.size();
        if (n > 6 && kdir.compare(n - 6, 6, ".vxbin") == 0) {
          const auto slash = kdir.rfind('/');
          kdir = slash == std::string::npos ? "." : kdir.substr(0, slash);
        }
      } break;
      case 'h':
      case '?': usage(); return 0;
      default: usage(); return -1;
    }
  }
  if (output == "null" && !reference.empty()) {
    std::printf("Error: the output file is missing for reference validation!\n");
    return 1;
  }
  std::vector<uint32_t> src;
  uint32_t w = 0, h = 0;
  input = rt::ResolveAsset(input);  // tex/main.cpp resolves through ASSETS_PATHS too
  if (!reference.empty()) reference = rt::ResolveAsset(reference);
  if (rt::LoadPngARGB(input, &src, &w, &h) != 0) {
    std::printf("Error: cannot load %s\n", input.c_str());
    return -1;
  }
  rt_tex_h t = nullptr;
  CHECK(rt_tex_create(kdir.empty() ? nullptr : kdir.c_str(), &t));
  CHECK(rt_tex_configure(t, src.data(), w, h, &p));
  rt_tex_stats_t st;
  CHECK(rt_tex_stats(t, &st));
  std::printf("source image: width=%u, heigth=%u, size=%llu bytes\n", w, h,
              (unsigned long long)st.texture_bytes);
  std::printf("destination image: width=%u, heigth=%u, size=%u bytes\n", st.dst_width,
              st.dst_height, st.dst_width * st.dst_height * 4);
  const auto t0 = std::chrono::steady_clock::now();
  CHECK(rt_tex_render(t));
  const double ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  CHECK(rt_tex_stats(t, &st));
  std::printf("Elapsed time: %.3f ms (kernel %.4f ms)\n", ms, st.kernel_ms);
  std::vector<uint32_t> dst((size_t)st.dst_width * st.dst_height);
  CHECK(rt_tex_read(t, dst.data(), dst.size()));
  rt_tex_free(t);
  if (output != "null") {
    // SavePngARGB writes bottom-up framebuffers; the tex app's rows are top-down
    std::vector<uint32_t> flipped(dst.size());
    for (uint32_t y = 0; y < st.dst_height; ++y)
      std::memcpy(&flipped[(size_t)(st.dst_height - 1 - y) * st.dst_width],
                  &dst[(size_t)y * st.dst_width], st.dst_width * 4);
    if (rt::SavePngARGB(output, flipped.data(), st.dst_width, st.dst_height) != 0) {
      std::printf("Error: cannot write %s\n", output.c_str());
      return -1;
    }
  }
  if (!reference.empty()) {
    std::vector<uint32_t> ref;
    uint32_t rw = 0, rh = 0;
    if (rt::LoadPngARGB(reference, &ref, &rw, &rh) != 0 || rw != st.dst_width ||
        rh != st.dst_height) {
      std::printf("FAILED! reference missing or size mismatch\n");
      return 1;
    }
    const int errors = (int)rt::CompareARGB(dst.data(), ref.data(), dst.size(), 1);
    if (errors == 0) std::printf("PASSED!\n");
    else std::printf("FAILED! %d errors.\n", errors);
    return errors;
  }
  return 0;
}
