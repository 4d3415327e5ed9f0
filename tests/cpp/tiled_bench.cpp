// tiled_bench.cpp -- the C++ host path north_star names, timed at frame size.
//
// A reference-style C++ caller (the chain loop of reference/test.cpp:376-401, batched): it builds the cfg4
// workload through the drop-in classes (Mesh::makeEllipsoid, standardize, BezierMesh, BezierLens), hands a
// 4096 x 4096 ray frame to a bzr::TiledChain and traces frame after frame into device outputs, one set of
// outputs per frame slot.  Rays / s are counted the way bench.py counts them: every BezierMesh::intersect
// call (primary + refracted segments, summed from one frame's segment counts), over K timed frames bracketed
// by a device synchronisation on both sides, after a time-based pre-warm and W warm-up frames.
//
// The rays are in bench.py's order: the 64 x 64 tiles of the image nearest its centre first
// (bzr_amd/configs.py shard_pixels, order "centre"), each tile in 8 x 8 sub-tiles (one wavefront each); the
// plan deals tiles round-robin to its devices.  --dump writes the last frame's outputs in image tile order
// (tile ty * 64 + tx) for tests/test_cpp_bench.py, which checks them against the committed oracle digests of
// the whole frame (tests/golden/d_cfg4_4096.npz).
//
// Usage: tiled_bench [--frames K] [--warmup W] [--prewarm-s S] [--slots F] [--devices N [--one-gpu]] [--side S]
//                    [--host-frames H] [--dump path]
// Prints one JSON line.  --host-frames also times H synchronous host-pointer frames (TiledChain::trace into
// host Rays and bzr::traceChain), whose rates include the PCIe copies and the host AoS <-> SoA conversions.
#include <hip/hip_runtime_api.h>

#include <memory>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <stdexcept>
#include <string>
#include <vector>

#include "bezierLens.h"
#include "bezierMesh.h"
#include "mesh.h"

namespace {

constexpr int kTile = 64;

#define HIPCHECK(expr)                                                                          \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

struct Args {
  int frames = 100, warmup = 10, slots = 3, devices = 1, side = 4096, host_frames = 0;
  bool one_gpu = false;  // --one-gpu: every list device is HIP device 0 (the plan's host work at N shares, one GPU)
  double prewarm_s = 0.3;
  std::string dump;
};

Args parse(int argc, char **argv) {
  Args a;
  for (int i = 1; i < argc; ++i) {
    std::string k = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) throw std::invalid_argument("missing value for " + k);
      return argv[++i];
    };
    if (k == "--frames") a.frames = std::stoi(next());
    else if (k == "--warmup") a.warmup = std::stoi(next());
    else if (k == "--slots") a.slots = std::stoi(next());
    else if (k == "--devices") a.devices = std::stoi(next());
    else if (k == "--one-gpu") a.one_gpu = true;
    else if (k == "--side") a.side = std::stoi(next());
    else if (k == "--host-frames") a.host_frames = std::stoi(next());
    else if (k == "--prewarm-s") a.prewarm_s = std::stod(next());
    else if (k == "--dump") a.dump = next();
    else throw std::invalid_argument("unknown argument " + k);
  }
  if (a.frames < 1 || a.slots < 1 || a.devices < 1 || a.side < kTile || a.side % kTile)
    throw std::invalid_argument("need frames >= 1, slots >= 1, devices >= 1, side a multiple of 64");
  return a;
}

// cfg4 (bzr_amd/configs.py): makeEllipsoid(32, 16, (1, 4, 2)) lenses at x = 10 and x = 13, ri 1.3
BezierLens makeLens(float x) {
  Mesh m;
  m.makeEllipsoid(32, 16, Vector(1.0f, 4.0f, 2.0f));
  m += Vector{x, 0.0f, 0.0f};
  m.standardizeVertices();
  m.standardizeNormals();
  return BezierLens(1.3f, BezierMesh(m));
}

// Tiles of the side x side image, nearest the centre first (stable order on equal distance).
std::vector<int> centreFirstTiles(int side) {
  const int nb = side / kTile;
  std::vector<int> tiles(nb * nb);
  std::iota(tiles.begin(), tiles.end(), 0);
  std::vector<double> key(tiles.size());
  for (int t : tiles) {
    const double dy = (t / nb + 0.5) * kTile - side / 2.0, dx = (t % nb + 0.5) * kTile - side / 2.0;
    key[t] = dy * dy + dx * dx;
  }
  std::stable_sort(tiles.begin(), tiles.end(), [&](int a, int b) { return key[a] < key[b]; });
  return tiles;
}

// The frame's rays, tile after tile in `tiles` order, each tile in 8 x 8 sub-tiles: pixel (row, col) starts at
// (0, y0 + (y1 - y0) (col + 0.5) / side, z0 + (z1 - z0) (row + 0.5) / side) and runs along +x (float32, the
// operation order of configs.rays_for).
std::vector<Ray> frameRays(int side, std::vector<int> const &tiles) {
  const int nb = side / kTile;
  const float y0 = -4.2f, y1 = 4.2f, z0 = -2.1f, z1 = 2.1f, s = static_cast<float>(side);
  std::vector<Ray> rays;
  rays.reserve(static_cast<std::size_t>(side) * side);
  for (int t : tiles)
    for (int k = 0; k < kTile * kTile; ++k) {
      const int sub = k / 64, w = k % 64;
      const int row = (t / nb) * kTile + (sub / 8) * 8 + w / 8, col = (t % nb) * kTile + (sub % 8) * 8 + w % 8;
      const float y = y0 + (y1 - y0) * ((static_cast<float>(col) + 0.5f) / s);
      const float z = z0 + (z1 - z0) * ((static_cast<float>(row) + 0.5f) / s);
      rays.emplace_back(Vertex{0.0f, y, z}, Vector{1.0f, 0.0f, 0.0f});
    }
  return rays;
}

double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

}  // namespace

int main(int argc, char **argv) {
  try {
    const Args a = parse(argc, argv);
    // the frame slots need distinct hardware queues: as bench.py, raise HIP's default of 4
    // before the runtime starts unless the caller set at least 16
    const char *hwq = std::getenv("GPU_MAX_HW_QUEUES");
    if (!hwq || std::atoi(hwq) < 16) setenv("GPU_MAX_HW_QUEUES", "16", 1);
    const std::size_t n = static_cast<std::size_t>(a.side) * a.side;

    double t0 = now();
    BezierLens lens1 = makeLens(10.0f), lens2 = makeLens(13.0f);
    const double prep_s = now() - t0;
    const std::vector<int> tiles = centreFirstTiles(a.side);
    const std::vector<Ray> rays = frameRays(a.side, tiles);

    // one context per (slot, device): slot s on device d -- each its own stream
    std::vector<std::unique_ptr<bzr::Context>> owned;
    std::vector<std::vector<bzr::Context *>> slots(a.slots);
    for (int s = 0; s < a.slots; ++s)
      for (int d = 0; d < a.devices; ++d) {
        owned.push_back(std::make_unique<bzr::Context>(a.one_gpu ? 0 : d));
        slots[s].push_back(owned.back().get());
      }
    t0 = now();
    bzr::TiledChain plan(slots, {&lens1, &lens2}, n, kTile * kTile);
    const double plan_s = now() - t0;
    t0 = now();
    plan.setRays(rays.data());
    plan.sync();
    const double set_rays_s = now() - t0;

    // one set of device outputs per slot: rays [6][n], status [n], segments [n]
    std::vector<float *> o_rays(a.slots);
    std::vector<uint32_t *> o_st(a.slots), o_seg(a.slots);
    HIPCHECK(hipSetDevice(0));
    for (int s = 0; s < a.slots; ++s) {
      HIPCHECK(hipMalloc(&o_rays[s], 24 * n));
      HIPCHECK(hipMalloc(&o_st[s], 4 * n));
      HIPCHECK(hipMalloc(&o_seg[s], 4 * n));
    }
    int frame = 0;
    auto trace = [&]() {
      const int s = frame++ % a.slots;
      plan.trace(o_rays[s], o_st[s], o_seg[s]);
    };
    // the counted frame: segments per frame (every BezierMesh::intersect call)
    trace();
    plan.sync();
    std::vector<uint32_t> seg(n), st(n);
    HIPCHECK(hipMemcpy(seg.data(), o_seg[0], 4 * n, hipMemcpyDeviceToHost));
    const uint64_t segments = std::accumulate(seg.begin(), seg.end(), uint64_t{0});

    // pre-warm (clock ramp), then the warm-up frames right before the timed ones
    if (a.prewarm_s > 0) {
      const double tp = now();
      do {
        for (int k = 0; k < 8; ++k) trace();
        plan.sync();
      } while (now() - tp < a.prewarm_s);
    }
    for (int k = 0; k < a.warmup; ++k) trace();
    plan.sync();
    const int first_timed = frame;
    t0 = now();
    double enqueue_s = 0.0;  // host time inside TiledChain::trace (the launches and copies it queues per frame)
    for (int k = 0; k < a.frames; ++k) {
      const double tq = now();
      trace();
      enqueue_s += now() - tq;
    }
    plan.sync();
    const double elapsed = now() - t0;
    const double ms = elapsed / a.frames * 1e3, mrays = static_cast<double>(segments) * a.frames / elapsed / 1e6;

    // the last timed frame's outputs, in image tile order
    if (!a.dump.empty()) {
      const int s = (first_timed + a.frames - 1) % a.slots;
      std::vector<float> r(6 * n);
      HIPCHECK(hipMemcpy(r.data(), o_rays[s], 24 * n, hipMemcpyDeviceToHost));
      HIPCHECK(hipMemcpy(st.data(), o_st[s], 4 * n, hipMemcpyDeviceToHost));
      HIPCHECK(hipMemcpy(seg.data(), o_seg[s], 4 * n, hipMemcpyDeviceToHost));
      const std::size_t tr = kTile * kTile, nt = tiles.size();
      std::vector<float> rr(6 * n);
      std::vector<uint32_t> ss(n), gg(n);
      for (std::size_t j = 0; j < nt; ++j) {  // position j of the frame holds image tile tiles[j]
        const std::size_t dst = static_cast<std::size_t>(tiles[j]) * tr, src = j * tr;
        for (int row = 0; row < 6; ++row)
          std::memcpy(&rr[row * n + dst], &r[row * n + src], tr * sizeof(float));
        std::memcpy(&ss[dst], &st[src], tr * 4);
        std::memcpy(&gg[dst], &seg[src], tr * 4);
      }
      FILE *f = std::fopen(a.dump.c_str(), "wb");
      if (!f) throw std::runtime_error("cannot write " + a.dump);
      const uint64_t hdr[2] = {static_cast<uint64_t>(a.side), n};
      bool ok = std::fwrite(hdr, sizeof(hdr), 1, f) == 1 && std::fwrite(rr.data(), 4, rr.size(), f) == rr.size() &&
                std::fwrite(ss.data(), 4, n, f) == n && std::fwrite(gg.data(), 4, n, f) == n;
      ok = (std::fclose(f) == 0) && ok;
      if (!ok) throw std::runtime_error("short write to " + a.dump);
    }

    // synchronous host-pointer paths (PCIe and host conversions included): TiledChain::trace(Ray *) and
    // bzr::traceChain, one frame per call as a reference caller would issue them
    double host_tiled_ms = 0.0, host_chain_ms = 0.0;
    if (a.host_frames > 0) {
      std::vector<Ray> out(n);
      std::vector<RefractionResult> status(n);
      plan.trace(out.data(), status.data(), seg.data());  // warm
      t0 = now();
      for (int k = 0; k < a.host_frames; ++k) plan.trace(out.data(), status.data(), seg.data());
      host_tiled_ms = (now() - t0) / a.host_frames * 1e3;
      bzr::traceChain({&lens1, &lens2}, rays.data(), n, out.data(), status.data(), seg.data(), slots[0][0]);
      t0 = now();
      for (int k = 0; k < a.host_frames; ++k)
        bzr::traceChain({&lens1, &lens2}, rays.data(), n, out.data(), status.data(), seg.data(), slots[0][0]);
      host_chain_ms = (now() - t0) / a.host_frames * 1e3;
    }
    for (int s = 0; s < a.slots; ++s) {
      (void)hipFree(o_rays[s]);
      (void)hipFree(o_st[s]);
      (void)hipFree(o_seg[s]);
    }
    const char *tp_name[] = {"auto", "rccl", "peer", "direct"};
    const int tp = plan.transport();
    std::printf("{\"metric\": \"Mrays/sec (primary+refracted), C++ host path (bzr::TiledChain)\", \"value\": %.3f, "
                "\"unit\": \"Mrays/s\", \"ms_per_frame\": %.4f, \"host_enqueue_ms_per_frame\": %.4f, \"frames\": %d, "
                "\"warmup\": %d, \"prewarm_s\": %.2f, "
                "\"slots\": %d, \"devices\": %d, \"transport\": \"%s\", \"side\": %d, \"primaries\": %zu, "
                "\"segments_per_frame\": %llu, \"preprocess_s\": %.3f, \"plan_create_s\": %.3f, \"set_rays_s\": %.3f, "
                "\"host_frames\": %d, \"host_tiled_ms_per_frame\": %.3f, \"host_tiled_mrays\": %.3f, "
                "\"host_trace_chain_ms_per_frame\": %.3f, \"host_trace_chain_mrays\": %.3f, "
                "\"gpu_max_hw_queues\": \"%s\", \"workload\": \"cfg4: two makeEllipsoid(32,16,(1,4,2)) lenses at x=10 "
                "and x=13, ri 1.3, centre-first 64x64 tiles\"}\n",
                mrays, ms, enqueue_s / a.frames * 1e3, a.frames, a.warmup, a.prewarm_s, a.slots, a.devices, tp_name[tp & 3], a.side, n,
                static_cast<unsigned long long>(segments), prep_s, plan_s, set_rays_s, a.host_frames, host_tiled_ms,
                host_tiled_ms > 0 ? segments / (host_tiled_ms * 1e3) : 0.0, host_chain_ms,
                host_chain_ms > 0 ? segments / (host_chain_ms * 1e3) : 0.0, std::getenv("GPU_MAX_HW_QUEUES"));
    return 0;
  } catch (std::exception const &e) {
    std::fprintf(stderr, "tiled_bench: %s\n", e.what());
    return 1;
  }
}
