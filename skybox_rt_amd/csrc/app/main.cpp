// main.cpp -- rtapp (and, built with -DRT_APP_RASTER, rasterapp): the
// command-line regression apps over librtapp.so.
//
// rtapp takes draw3d's command line unchanged (tests/regression/draw3d/
// main.cpp:80-135): -t trace, -s/-e first/last drawcall drawn, -o output,
// -r reference (tolerance-1 compare, "PASSED!"/"FAILED! N errors."), -w/-h
// size, -k tile log size (binning granularity), -u/-x/-y software texture /
// raster / OM switches and -z (accepted; one pipeline serves both here, so
// the output is the same), -? usage.  Files resolve like ResolveFilePath
// (gfxutil.cpp:348-363): as given, else in each directory of the
// comma-separated RT_ASSETS_PATHS (the reference compiles its source
// directory in as ASSETS_PATHS), a scene also as <name>.gz.  The kernel images
// come from the library directory, or from env RT_KERNEL_DIR.
//
// Mode: primary rays by default (raster-exact, draw3d's own output); a scene
// the RT path does not support (blending, stencil, partial colour writes,
// mixed depth functions: DESIGN.md "Scope") and any -k other than the
// RASTER_TILE_LOGSIZE 5 the RT path bins at render through the draw3d raster
// pipeline instead, which is what draw3d itself runs.  Extensions: -S shadow
// rays, -L x,y,w light, -P N path tracing with N bounces, -F flat triangle
// list, -R raster pipeline, -n N repeat launches, -B lbvh|sah device BVH
// build, -H host-loop setup; multi-GPU (one process per GPU over
// librt_shard.so / RCCL): -G rank,ranks -I idfile -- this process renders
// 32x32 tiles t with t % ranks == rank, rank 0 writes the RCCL communicator
// id to `idfile` (the others wait for it), every frame ends with
// rt_render_gather to rank 0, which writes / checks the assembled frame.
//
// rasterapp takes the raster regression app's command line
// (tests/regression/raster/main.cpp:66-107: -t -o -r -w -h -k -z) and writes
// its coverage image (covered pixels white over 0xff000000, raster/
// kernel.cpp:35-45) through the raster pipeline.
#include <getopt.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <thread>

#include "assets.h"
#include "png.h"
#include "rt_shard.h"
#include "vx_rt.h"

namespace {

const char* trace_file = "triangle.cgltrace";
const char* output_file = "output.png";
const char* reference_file = nullptr;
uint32_t width = 128, height = 128, repeat = 1;
uint32_t start_draw = 0, end_draw = 0xffffffffu;
int tile_log = -1;  // -k (-1: RASTER_TILE_LOGSIZE)
bool shadows = false, raster = false, flat = false;
int bounces = -1;  // >= 0: path tracing
float light[3] = {0.0f, 60.0f, 80.0f};
int rank = -1, ranks = 1;            // -G rank,ranks
const char* id_file = "rt_shard.id";  // -I
const char* build = nullptr;          // -B lbvh|sah: build the BVH on the device
bool host_setup = false;              // -H: per-resolution records by the host loops

#ifdef RT_APP_RASTER
const char* kOpts = "t:i:o:r:w:h:k:n:z?";
void usage() {
  std::printf("Vortex rasterizer Test.\n"
              "Usage: [-t trace] [-o output] [-r reference] [-w width] [-h height] [-z no_hw] "
              "[-k tilelogsize] [-n repeat]\n");
}
#else
const char* kOpts = "t:s:e:i:o:r:w:h:k:n:L:P:G:I:B:uxyzSRFH?";
void usage() {
  std::printf("Vortex 3D Rendering Test (MI355X).\n"
              "Usage: [-t trace] [-s startdraw] [-e enddraw] [-o output] [-r reference] [-w width] "
              "[-h height] [-x s/w rast] [-y s/w om] [-u s/w tex] [-k tilelogsize]\n"
              "       [-S shadows] [-L x,y,w] [-n repeat] [-R raster | -P bounces | -F flat] "
              "[-G rank,ranks [-I idfile]] [-B lbvh|sah device BVH build] [-H host setup]\n"
              "       env RT_KERNEL_DIR: kernel images; RT_ASSETS_PATHS: search directories\n");
}
#endif

#define RT_CHECK(_expr)                                                       \
  do {                                                                        \
    int _ret = (_expr);                                                       \
    if (_ret == 0) break;                                                     \
    std::printf("Error: '%s' returned %d! (%s)\n", #_expr, _ret, rt_last_error()); \
    std::exit(-1);                                                            \
  } while (false)

}  // namespace

int main(int argc, char** argv) {
  int c;
  while ((c = getopt(argc, argv, kOpts)) != -1) {
    switch (c) {
    case 't': trace_file = optarg; break;
    case 'o': output_file = optarg; break;
    case 'r': reference_file = optarg; break;
    case 'w': width = (uint32_t)std::atoi(optarg); break;
    case 'h': height = (uint32_t)std::atoi(optarg); break;
    case 'k': tile_log = std::atoi(optarg); break;
    case 'n': repeat = (uint32_t)std::atoi(optarg); break;
    case 'z': break;  // raster / om: software path -- same output here
#ifndef RT_APP_RASTER
    case 's': start_draw = (uint32_t)std::atoi(optarg); break;
    case 'e': end_draw = (uint32_t)std::atoi(optarg); break;
    case 'u': case 'x': case 'y': break;  // software tex / raster / OM: same output here
    case 'S': shadows = true; break;
    case 'R': raster = true; break;
    case 'F': flat = true; break;
    case 'P': bounces = std::atoi(optarg); break;
    case 'L': std::sscanf(optarg, "%f,%f,%f", &light[0], &light[1], &light[2]); break;
    case 'G': std::sscanf(optarg, "%d,%d", &rank, &ranks); break;
    case 'I': id_file = optarg; break;
    case 'B': build = optarg; break;
    case 'H': host_setup = true; break;
#endif
    case '?': usage(); return 0;
    default: usage(); return -1;  // -i: in the reference's option string, never handled
    }
  }
  if (std::strcmp(output_file, "null") == 0 && reference_file) {
    std::printf("Error: the output file is missing for reference validation!\n");
    return 1;
  }
#ifdef RT_APP_RASTER
  raster = true;
#endif
  const bool rt_only = shadows || flat || bounces >= 0 || rank >= 0;  // modes only the RT path has
  if (tile_log >= 0 && tile_log != 5 && !raster) {
    if (rt_only) {
      std::printf("Error: -k %d: the ray-tracing modes bin at RASTER_TILE_LOGSIZE 5\n", tile_log);
      return 1;
    }
    std::printf("Tile log size %d: rendering through the draw3d raster pipeline\n", tile_log);
    raster = true;
  }
  const bool sharded = rank >= 0;
  if (sharded && (ranks < 1 || rank >= ranks || raster)) {
    std::printf("Error: -G rank,ranks needs 0 <= rank < ranks (ray-tracing modes)\n");
    return 1;
  }
  int device = 0;
  rt_shard_comm_h comm = nullptr;
  uint8_t id[RT_SHARD_ID_BYTES] = {};
  if (sharded) {
    // one process per GPU: rank r on device r % (visible devices)
    const int ndev = rt_shard_device_count();
    device = ndev > 0 ? rank % ndev : 0;
    setenv("VX_HIP_DEVICE", std::to_string(device).c_str(), 0);
    device = std::atoi(std::getenv("VX_HIP_DEVICE"));
    if (rank == 0) {  // the communicator id, published atomically
      RT_CHECK(rt_shard_unique_id(id));
      const std::string tmp = std::string(id_file) + ".tmp";
      std::ofstream(tmp, std::ios::binary).write((const char*)id, RT_SHARD_ID_BYTES);
      RT_CHECK(std::rename(tmp.c_str(), id_file));
    } else {
      struct stat sb;
      for (int i = 0; stat(id_file, &sb) != 0 || sb.st_size < RT_SHARD_ID_BYTES; ++i) {
        if (i > 6000) { std::printf("Error: no communicator id in %s\n", id_file); return 1; }
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
      }
      std::ifstream(id_file, std::ios::binary).read((char*)id, RT_SHARD_ID_BYTES);
    }
  }
  const std::string trace = rt::ResolveAsset(trace_file, true);
  rt_scene_h scene = nullptr;
  RT_CHECK(rt_scene_load_range(trace.c_str(), start_draw, end_draw, &scene));
  rt_scene_info_t info;
  RT_CHECK(rt_scene_info(scene, &info));
  std::printf("CGL Trace: drawcalls=%u, primitives=%u, geometry=%u, layers=%u, textures=%u\n",
              info.num_drawcalls, info.num_prims, info.num_geometry, info.num_layer,
              info.num_textures);
  std::printf("BVH: nodes=%u, leaves=%u, depth=%u, build=%.3f ms (parse %.3f ms)\n",
              info.bvh_nodes, info.bvh_leaves, info.bvh_depth, info.bvh_ms, info.parse_ms);
  rt_renderer_h r = nullptr;
  RT_CHECK(rt_renderer_create(scene, std::getenv("RT_KERNEL_DIR"), &r));
  if (build) {
    const uint32_t m = std::strcmp(build, "sah") == 0 ? RT_BVH_BUILD_SAH : RT_BVH_BUILD_LBVH;
    rt_bvh_build_stats_t bs;
    RT_CHECK(rt_renderer_build_bvh_ex(r, m, &bs));
    std::printf("Device BVH (%s): nodes=%u, depth=%u, bvh4 nodes=%u, stack4=%u, %u launches, "
                "%.3f ms (kernels %.3f ms)\n", m == RT_BVH_BUILD_SAH ? "sah" : "lbvh", bs.nodes,
                bs.depth, bs.nodes4, bs.stack4, bs.launches, bs.build_ms, bs.kernel_ms);
  }
  rt_render_params_t p;
  std::memset(&p, 0, sizeof(p));
  p.width = width;
  p.height = height;
  p.bounces = bounces >= 0 ? (uint32_t)bounces : 0u;
  p.seed = 0x5EED;
  std::memcpy(p.light, light, sizeof(light));
  p.clear_color = 0xff000000u;
  p.shard_count = 1;
  p.tile_logsize = tile_log >= 0 ? (uint32_t)tile_log : 0u;
  const uint32_t common = RT_RENDER_COUNTERS |  // the CLI prints ray counts
                          (host_setup ? RT_RENDER_HOST_SETUP : 0u);
  p.flags = common | (shadows ? RT_RENDER_SHADOWS : 0u) | (raster ? RT_RENDER_RASTER : 0u) |
            (flat ? RT_RENDER_FLAT : 0u) | (bounces >= 0 ? RT_RENDER_PATH : 0u);
#ifdef RT_APP_RASTER
  p.flags |= RT_RENDER_COVERAGE;
#endif
  if (sharded) {
    p.shard_index = (uint32_t)rank;
    p.shard_count = (uint32_t)ranks;
    p.flags |= RT_RENDER_COMPACT;
    RT_CHECK(rt_shard_comm_init(&comm, id, (uint32_t)rank, (uint32_t)ranks, device));
    uint32_t seen = 0;
    RT_CHECK(rt_shard_comm_info(comm, nullptr, &seen));
    std::printf("Shard: rank %d of %d on device %d (communicator: %u ranks)\n", rank, ranks, device,
                seen);
  }
  int rc = rt_renderer_configure(r, &p);
  if (rc == -2 && !raster && !rt_only) {
    // a scene the RT path does not support: draw3d's own pipeline renders it
    std::printf("RT path: %s; rendering through the draw3d raster pipeline\n", rt_last_error());
    raster = true;
    p.flags = common | RT_RENDER_RASTER;
    rc = rt_renderer_configure(r, &p);
  }
  RT_CHECK(rc);
  rt_setup_stats_t ss;
  RT_CHECK(rt_renderer_setup_stats(r, &ss));
  std::printf("Setup (%s): %.3f ms, configure %.3f ms\n", ss.device ? "device" : "host", ss.setup_ms,
              ss.configure_ms);
  double total = 0.0;
  rt_stats_t st;
  std::vector<uint32_t> gathered;
  if (sharded && rank == 0) gathered.resize((size_t)width * height);
  for (uint32_t i = 0; i < repeat; ++i) {
    RT_CHECK(rt_render(r));
    RT_CHECK(rt_render_stats(r, &st));
    total += st.kernel_ms;
    if (sharded) RT_CHECK(rt_render_gather(r, comm, rank == 0 ? gathered.data() : nullptr));
  }
  if (raster) {
    std::printf("Elapsed time: %.4f ms/frame (grid %u x %u), pixels=%llu, fragments=%llu, "
                "%.1f Mpixels/s\n",
                total / repeat, st.grid, st.block, (unsigned long long)st.primary_rays,
                (unsigned long long)st.shaded, (double)st.primary_rays / (total / repeat) * 1e-3);
  } else {
    const double rays = (double)(st.primary_rays + st.shadow_rays + st.bounce_rays);
    std::printf("Elapsed time: %.4f ms/frame (grid %u x %u), rays=%.0f (primary %llu, shadow %llu, "
                "bounce %llu, occluded %llu), %.1f Mrays/s\n",
                total / repeat, st.grid, st.block, rays, (unsigned long long)st.primary_rays,
                (unsigned long long)st.shadow_rays, (unsigned long long)st.bounce_rays,
                (unsigned long long)st.occluded, rays / (total / repeat) * 1e-3);
  }
  int errors = 0;
  if (std::strcmp(output_file, "null") != 0 && (!sharded || rank == 0)) {
    std::vector<uint32_t> fb((size_t)width * height);
    if (sharded) fb = gathered;  // the frame assembled from every rank's tiles
    else RT_CHECK(rt_read_framebuffer(r, fb.data(), fb.size()));
    RT_CHECK(rt::SavePngARGB(output_file, fb.data(), width, height));
    if (reference_file) {
      std::vector<uint32_t> out, ref;
      uint32_t ow, oh, rw, rh;
      RT_CHECK(rt::LoadPngARGB(output_file, &out, &ow, &oh));
      RT_CHECK(rt::LoadPngARGB(rt::ResolveAsset(reference_file), &ref, &rw, &rh));
      if (ow != rw || oh != rh) {
        std::printf("FAILED! size mismatch\n");
        errors = -1;
      } else {
        errors = (int)rt::CompareARGB(out.data(), ref.data(), out.size(), 1);
        if (errors == 0) std::printf("PASSED!\n");
        else std::printf("FAILED! %d errors.\n", errors);
      }
    }
  }
  rt_renderer_free(r);
  rt_scene_free(scene);
  if (comm) rt_shard_comm_free(comm);
  return errors;
}
