// newton_ceiling.hip -- the issue ceiling of the staged Newton site's arithmetic alone.
//
// k_newton runs the reference's BezierTriangle::intersect tail (patch_intersect<kGated>) on 64-pair chunks of one
// patch, with the record in SGPRs.  Its VALU issue is ~0.6 of the peak; this probe asks how much of the gap is the
// arithmetic's own instruction stream and how much the stage around it (pair records, ray gathers, key atomics,
// slot stores).  Each wave runs K passes, each over one wave-uniform patch record (scalar loads, as k_newton) with
// every lane's ray aimed at a point inside that patch (origin 10 units before the point, direction +x), so the
// Newton iterations take their usual path; nothing but the record loads touches memory inside the loop.
// Waves per SIMD W = 1, 2, 4, 6, 8 (blocks of 256 threads, one wave per SIMD each, 256 CUs x W blocks).
//
// usage: newton_ceiling <patches.f32> <npatches> [K]   (patches: [n][66] float32 records, scripts/newton_ceiling.py)
// Prints one JSON line per W: ms per launch, passes, passes per second.  VALU instructions per launch come from a
// separate `rocprofv3 --pmc SQ_INSTS_VALU` run of the same binary (scripts/newton_ceiling.py does both).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "patch_math.hpp"

using namespace bzr_dev;

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

__device__ __forceinline__ float lane_unit(uint32_t k) {  // a fixed pseudo-random number in [0.05, 0.95)
  k = k * 2654435761u + 0x9E3779B9u;
  k ^= k >> 15;
  k *= 2246822519u;
  k ^= k >> 13;
  return 0.05f + 0.9f * (float)(k >> 8) * (1.0f / 16777216.0f);
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_ceiling(
    const float *__restrict__ full, uint32_t np, uint32_t passes, float *__restrict__ out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
  // the lane's barycentric weights (fixed per lane, inside the triangle)
  float u = lane_unit(lane), v = lane_unit(lane + 977u) * (1.0f - u);
  const float w = 1.0f - u - v;
  float acc = 0.0f;
  for (uint32_t k = 0; k < passes; ++k) {
    const uint32_t b = __builtin_amdgcn_readfirstlane((wave * 131u + k * 977u) % np);
    const auto p = uniform_patch(full, b);
    const f3 c0 = p.cp(0), c1 = p.cp(1), c2 = p.cp(2);
    const f3 q = mk(u * c0.x + v * c1.x + w * c2.x, u * c0.y + v * c1.y + w * c2.y, u * c0.z + v * c1.z + w * c2.z);
    const f3 s = mk(q.x - 10.0f, q.y, q.z), d = mk(1.0f, 0.0f, 0.0f);
    const Hit h = patch_intersect<true, false>(p, s, d, false);
    acc += h.what == kIntersect ? 1.0f : (h.what <= kFollow2 ? 128.0f : 16384.0f);  // outcome counts (< 2^21: exact)
  }
  out[blockIdx.x * 256u + threadIdx.x] = acc;
}

int main(int argc, char **argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s patches.f32 npatches [passes]\n", argv[0]);
    return 2;
  }
  const uint32_t np = (uint32_t)std::atoi(argv[2]);
  const uint32_t passes = argc > 3 ? (uint32_t)std::atoi(argv[3]) : 64u;
  if (passes == 0 || passes > 127) {
    std::fprintf(stderr, "passes must be in [1, 127]\n");
    return 2;
  }
  std::vector<float> host((size_t)np * rec::kWords);
  FILE *f = std::fopen(argv[1], "rb");
  if (!f || std::fread(host.data(), sizeof(float), host.size(), f) != host.size()) {
    std::fprintf(stderr, "cannot read %u records from %s\n", np, argv[1]);
    return 2;
  }
  std::fclose(f);
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  float *full = nullptr, *out = nullptr;
  CHECK(hipMalloc(&full, host.size() * sizeof(float)));
  CHECK(hipMemcpy(full, host.data(), host.size() * sizeof(float), hipMemcpyHostToDevice));
  CHECK(hipMalloc(&out, (size_t)cus * 8u * 256u * sizeof(float)));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int ws[] = {1, 2, 4, 6, 8};
  for (int W : ws) {
    const uint32_t blocks = (uint32_t)cus * (uint32_t)W;
    hipLaunchKernelGGL(k_ceiling, dim3(blocks), dim3(256), 0, 0, full, np, passes, out);  // warm-up
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CHECK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(k_ceiling, dim3(blocks), dim3(256), 0, 0, full, np, passes, out);
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms = 0.0f;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    CHECK(hipGetLastError());
    const double npass = (double)blocks * 4.0 * passes;
    std::printf("{\"waves_per_simd\": %d, \"blocks\": %u, \"passes_per_wave\": %u, \"ms\": %.4f, \"passes\": %.0f, "
                "\"passes_per_s\": %.4e}\n",
                W, blocks, passes, best, npass, npass / (best * 1e-3));
    std::fflush(stdout);
  }
  std::vector<float> chk((size_t)cus * 8u * 256u);
  CHECK(hipMemcpy(chk.data(), out, chk.size() * sizeof(float), hipMemcpyDeviceToHost));
  // each lane's passes at W = 8 as intersections + 128 follows + 16384 nones (passes <= 127 per lane)
  double hit = 0.0, fol = 0.0, none = 0.0;
  for (float x : chk) {
    const uint32_t a = (uint32_t)x;
    hit += a & 127u;
    fol += (a >> 7) & 127u;
    none += a >> 14;
  }
  const double all = hit + fol + none;
  std::printf("{\"outcomes_at_w8\": {\"intersect\": %.4f, \"follow\": %.4f, \"none\": %.4f}}\n", hit / all, fol / all,
              none / all);
  CHECK(hipFree(full));
  CHECK(hipFree(out));
  return 0;
}
