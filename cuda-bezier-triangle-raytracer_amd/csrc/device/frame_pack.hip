// frame_pack.hip -- one chain frame's results into a gather buffer (bzr_pack_frame, include/bzr.h): the
// three layouts of bzr_amd/frame.py, on the context's stream, without a host sync.  Byte work, HBM-bound.
//   image    word i = status | segments << 8                        (frame.pack, IMAGE_ROWS)
//   rays     the 6 ray rows, then the word row                       (frame.pack, PACKED_ROWS)
//   compact  byte i = (status & 3) | segments << 2, the survivor count, then the survivors' rays in
//            index order, 6 rows of cap + 1 floats                    (frame.pack_compact)
// A survivor is a primary whose final ray differs from its primary: segments >= 2 or status != 0
// (frame.survivors).  The compact layout is an order-preserving stream compaction in three launches:
// per-block survivor counts (and the bytes), one block's exclusive scan of those counts (and the count
// word), then each block's scatter from its offset -- the same ray order as frame.pack_compact's cumsum.
#include <hip/hip_runtime.h>

#include <string>

#include "bzr.h"
#include "ctx.hpp"

extern "C" void bzr_internal_set_error(const char *msg);

namespace {

constexpr uint32_t kPackThreads = 256;
constexpr uint32_t kPackRays = 4 * kPackThreads;  // rays per block: 4 coalesced rounds of 256
constexpr uint32_t kScanThreads = 1024;

__device__ __forceinline__ bool survivor(uint32_t st, uint32_t sg) { return sg >= 2u || st != 0u; }

__global__ __launch_bounds__(kPackThreads) void k_pack_words(const float *__restrict__ rays,
                                                             const uint32_t *__restrict__ status,
                                                             const uint32_t *__restrict__ segments, uint32_t n,
                                                             uint32_t npad, uint32_t with_rays,
                                                             float *__restrict__ packed) {
  const uint32_t i = blockIdx.x * kPackThreads + threadIdx.x;
  if (i >= n) return;
  const uint32_t word = status[i] | (segments[i] << 8);
  if (with_rays) {
#pragma unroll
    for (uint32_t r = 0; r < 6u; ++r) packed[(size_t)r * npad + i] = rays[(size_t)r * n + i];
    packed[(size_t)6 * npad + i] = __uint_as_float(word);
  } else {
    packed[i] = __uint_as_float(word);
  }
}

// Pass 1: the bytes of this block's rays and its survivor count.
__global__ __launch_bounds__(kPackThreads) void k_compact_count(const uint32_t *__restrict__ status,
                                                                const uint32_t *__restrict__ segments, uint32_t n,
                                                                unsigned char *__restrict__ bytes,
                                                                uint32_t *__restrict__ block_count) {
  __shared__ uint32_t wave_sum[kPackThreads / 64];
  const uint32_t base = blockIdx.x * kPackRays, lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  uint32_t mine = 0;
#pragma unroll
  for (uint32_t k = 0; k < 4u; ++k) {
    const uint32_t i = base + k * kPackThreads + threadIdx.x;
    bool keep = false;
    if (i < n) {
      const uint32_t st = status[i], sg = segments[i];
      bytes[i] = (unsigned char)((st & 3u) | (sg << 2));
      keep = survivor(st, sg);
    }
    mine += (uint32_t)__popcll(__ballot(keep));
  }
  if (lane == 0u) wave_sum[w] = mine;
  __syncthreads();
  if (threadIdx.x == 0u) {
    uint32_t t = 0;
#pragma unroll
    for (uint32_t k = 0; k < kPackThreads / 64; ++k) t += wave_sum[k];
    block_count[blockIdx.x] = t;
  }
}

// Pass 2 (one block): exclusive offsets of the block counts; the total goes to the count word.
__global__ __launch_bounds__(kScanThreads) void k_compact_scan(const uint32_t *__restrict__ block_count, uint32_t nblk,
                                                               uint32_t *__restrict__ block_off,
                                                               uint32_t *__restrict__ count_word) {
  __shared__ uint32_t part[kScanThreads];
  const uint32_t per = (nblk + kScanThreads - 1) / kScanThreads;
  const uint32_t lo = threadIdx.x * per, hi = min(nblk, lo + per);
  uint32_t sum = 0;
  for (uint32_t b = lo; b < hi; ++b) sum += block_count[b];
  part[threadIdx.x] = sum;
  __syncthreads();
  for (uint32_t d = 1; d < kScanThreads; d <<= 1) {  // inclusive Hillis-Steele over the thread sums
    const uint32_t v = threadIdx.x >= d ? part[threadIdx.x - d] : 0u;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t run = threadIdx.x ? part[threadIdx.x - 1] : 0u;
  for (uint32_t b = lo; b < hi; ++b) {
    block_off[b] = run;
    run += block_count[b];
  }
  if (threadIdx.x == kScanThreads - 1) *count_word = part[kScanThreads - 1];
}

// Pass 3: the survivors' rays at their index-order positions (those below cap).
__global__ __launch_bounds__(kPackThreads) void k_compact_scatter(const float *__restrict__ rays,
                                                                  const uint32_t *__restrict__ status,
                                                                  const uint32_t *__restrict__ segments, uint32_t n,
                                                                  const uint32_t *__restrict__ block_off, uint32_t cap,
                                                                  float *__restrict__ out) {
  __shared__ uint32_t cnt[4][kPackThreads / 64];
  const uint32_t base = blockIdx.x * kPackRays, lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  bool keep[4];
  unsigned long long bal[4];
#pragma unroll
  for (uint32_t k = 0; k < 4u; ++k) {
    const uint32_t i = base + k * kPackThreads + threadIdx.x;
    keep[k] = i < n && survivor(status[i], segments[i]);
    bal[k] = __ballot(keep[k]);
    if (lane == 0u) cnt[k][w] = (uint32_t)__popcll(bal[k]);
  }
  __syncthreads();
  const uint32_t off = block_off[blockIdx.x];
  const unsigned long long below = lane ? (~0ull >> (64u - lane)) : 0ull;
  uint32_t before = 0;  // survivors of this block ahead of round k, wave w (index order: k-major, then w)
#pragma unroll
  for (uint32_t k = 0; k < 4u; ++k) {
    for (uint32_t v = 0; v < kPackThreads / 64; ++v)
      if (v < w) before += cnt[k][v];
    if (keep[k]) {
      const uint32_t pos = off + before + (uint32_t)__popcll(bal[k] & below);
      const uint32_t i = base + k * kPackThreads + threadIdx.x;
      if (pos < cap) {
#pragma unroll
        for (uint32_t r = 0; r < 6u; ++r) out[(size_t)r * (cap + 1u) + pos] = rays[(size_t)r * n + i];
      }
    }
    for (uint32_t v = w; v < kPackThreads / 64; ++v) before += cnt[k][v];
  }
}

// BZR_RAYS_AOS: the reference's Ray records ([n][6]: start xyz, direction xyz, 24 bytes) <-> the kernels'
// rows ([6][n]).  A block moves 256 rays' 6 KB through LDS so that both sides are read and written
// contiguously; stride 6 in LDS is a 2-way bank conflict.  HBM-bound: 48 bytes per ray.  The record side moves
// 8-byte pairs (3 per thread; a ray is 3 of them) when the records are 8-byte aligned, else single words.
constexpr uint32_t kRayWords = 6;
template <bool kPairs>
__global__ __launch_bounds__(kPackThreads) void k_rays_aos_to_soa(const float *__restrict__ aos, uint32_t n,
                                                                  float *__restrict__ soa) {
  __shared__ __attribute__((aligned(16))) float t[kRayWords * kPackThreads];
  const size_t r0 = (size_t)blockIdx.x * kPackThreads;
  const uint32_t m = static_cast<uint32_t>(min<size_t>(kPackThreads, n - r0));
  if constexpr (kPairs) {
    const float2 *src = reinterpret_cast<const float2 *>(aos + kRayWords * r0);
#pragma unroll
    for (uint32_t k = 0; k < kRayWords / 2; ++k) {
      const uint32_t w = k * kPackThreads + threadIdx.x;
      if (w < (kRayWords / 2) * m) reinterpret_cast<float2 *>(t)[w] = src[w];
    }
  } else {
#pragma unroll
    for (uint32_t k = 0; k < kRayWords; ++k) {
      const uint32_t w = k * kPackThreads + threadIdx.x;
      if (w < kRayWords * m) t[w] = aos[kRayWords * r0 + w];
    }
  }
  __syncthreads();
  if (threadIdx.x < m) {
#pragma unroll
    for (uint32_t k = 0; k < kRayWords; ++k) soa[(size_t)k * n + r0 + threadIdx.x] = t[kRayWords * threadIdx.x + k];
  }
}
template <bool kPairs>
__global__ __launch_bounds__(kPackThreads) void k_rays_soa_to_aos(const float *__restrict__ soa, uint32_t n,
                                                                  float *__restrict__ aos) {
  __shared__ __attribute__((aligned(16))) float t[kRayWords * kPackThreads];
  const size_t r0 = (size_t)blockIdx.x * kPackThreads;
  const uint32_t m = static_cast<uint32_t>(min<size_t>(kPackThreads, n - r0));
  if (threadIdx.x < m) {
#pragma unroll
    for (uint32_t k = 0; k < kRayWords; ++k) t[kRayWords * threadIdx.x + k] = soa[(size_t)k * n + r0 + threadIdx.x];
  }
  __syncthreads();
  if constexpr (kPairs) {
    float2 *dst = reinterpret_cast<float2 *>(aos + kRayWords * r0);
#pragma unroll
    for (uint32_t k = 0; k < kRayWords / 2; ++k) {
      const uint32_t w = k * kPackThreads + threadIdx.x;
      if (w < (kRayWords / 2) * m) dst[w] = reinterpret_cast<const float2 *>(t)[w];
    }
  } else {
#pragma unroll
    for (uint32_t k = 0; k < kRayWords; ++k) {
      const uint32_t w = k * kPackThreads + threadIdx.x;
      if (w < kRayWords * m) aos[kRayWords * r0 + w] = t[w];
    }
  }
}

// bzr_intersect_records: hit rows ([13][n]: t, point, cos, bary, normal, what, patch) -> n bzr_hit_record (the
// reference's BezierIntersection, 13 words) + the patch words.  256 hits' 13 KB through LDS per block, the
// records written as one contiguous run of 13 x 256 words.
constexpr uint32_t kHitWords = 13;
__global__ __launch_bounds__(kPackThreads) void k_hits_to_records(const float *__restrict__ rows, uint32_t n,
                                                                  uint32_t *__restrict__ rec,
                                                                  uint32_t *__restrict__ patch) {
  __shared__ uint32_t t[kHitWords * kPackThreads];
  const size_t r0 = (size_t)blockIdx.x * kPackThreads;
  const uint32_t m = static_cast<uint32_t>(min<size_t>(kPackThreads, n - r0)), i = threadIdx.x;
  if (i < m) {
    const size_t g = r0 + i;
    float f[kHitWords];
#pragma unroll
    for (uint32_t k = 0; k < kHitWords; ++k) f[k] = rows[(size_t)k * n + g];
    const uint32_t what = __float_as_uint(f[11]);
    uint32_t *o = t + kHitWords * i;  // stride 13: conflict-free
    o[0] = what == BZR_WHAT_INTERSECT ? 1u : 0u;  // mValid
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) o[1 + k] = __float_as_uint(f[1 + k]);  // point, cos
    o[5] = __float_as_uint(f[0]);                                          // distance
#pragma unroll
    for (uint32_t k = 0; k < 6; ++k) o[6 + k] = __float_as_uint(f[5 + k]);  // bary, normal
    o[12] = what;
    if (patch) patch[g] = __float_as_uint(f[12]);
  }
  __syncthreads();
  for (uint32_t w = i; w < kHitWords * m; w += kPackThreads) rec[kHitWords * r0 + w] = t[w];
}

bzr_status fail(bzr_status s, const std::string &msg) {
  bzr_internal_set_error(msg.c_str());
  return s;
}

}  // namespace

hipError_t bzr_hits_to_records(hipStream_t stream, const float *rows, uint32_t n, void *records, uint32_t *patch) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_hits_to_records, dim3((n + kPackThreads - 1) / kPackThreads), dim3(kPackThreads), 0, stream,
                     rows, n, static_cast<uint32_t *>(records), patch);
  return hipGetLastError();
}

hipError_t bzr_rays_relayout(hipStream_t stream, const float *src, float *dst, uint32_t n, bool to_soa) {
  if (n == 0) return hipSuccess;
  const dim3 grid((n + kPackThreads - 1) / kPackThreads);
  const bool pairs = (reinterpret_cast<uintptr_t>(to_soa ? src : dst) & 7u) == 0u;  // the records' alignment
  if (to_soa && pairs)
    hipLaunchKernelGGL(k_rays_aos_to_soa<true>, grid, dim3(kPackThreads), 0, stream, src, n, dst);
  else if (to_soa)
    hipLaunchKernelGGL(k_rays_aos_to_soa<false>, grid, dim3(kPackThreads), 0, stream, src, n, dst);
  else if (pairs)
    hipLaunchKernelGGL(k_rays_soa_to_aos<true>, grid, dim3(kPackThreads), 0, stream, src, n, dst);
  else
    hipLaunchKernelGGL(k_rays_soa_to_aos<false>, grid, dim3(kPackThreads), 0, stream, src, n, dst);
  return hipGetLastError();
}

extern "C" bzr_status bzr_pack_frame(bzr_ctx *ctx, int32_t layout, const float *rays_soa, const uint32_t *status,
                                     const uint32_t *segments, uint32_t n, uint32_t npad, uint32_t cap, void *packed) {
  // the arguments first (no device needed), then the context
  if (layout != BZR_PACK_IMAGE && layout != BZR_PACK_RAYS && layout != BZR_PACK_COMPACT)
    return fail(BZR_ERR_INVALID_ARGUMENT, "unknown pack layout " + std::to_string(layout));
  if (n > npad) return fail(BZR_ERR_INVALID_ARGUMENT, "n > npad");
  if (layout == BZR_PACK_COMPACT) {
    if (npad % 4u) return fail(BZR_ERR_INVALID_ARGUMENT, "compact layout: npad must be a multiple of 4");
    if (cap == 0u || cap > npad) return fail(BZR_ERR_INVALID_ARGUMENT, "compact layout needs 0 < cap <= npad");
  }
  if (!packed || (n && (!status || !segments))) return fail(BZR_ERR_INVALID_ARGUMENT, "null status / segments / packed");
  if (n && layout != BZR_PACK_IMAGE && !rays_soa) return fail(BZR_ERR_INVALID_ARGUMENT, "null rays");  // (n = 0: empty tensors)
  if (!ctx) return fail(BZR_ERR_INVALID_ARGUMENT, "null context");
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  if (prev != ctx->device) (void)hipSetDevice(ctx->device);
  struct Restore {
    int dev;
    ~Restore() {
      if (dev >= 0) (void)hipSetDevice(dev);
    }
  } restore{prev != ctx->device ? prev : -1};
  float *out = static_cast<float *>(packed);
  hipError_t e = hipSuccess;
  if (layout != BZR_PACK_COMPACT) {
    if (n) {
      hipLaunchKernelGGL(k_pack_words, dim3((n + kPackThreads - 1) / kPackThreads), dim3(kPackThreads), 0, ctx->stream,
                         rays_soa, status, segments, n, npad, layout == BZR_PACK_RAYS ? 1u : 0u, out);
      e = hipGetLastError();
    }
  } else {
    const uint32_t nw = npad / 4u, nblk = (n + kPackRays - 1) / kPackRays;
    uint32_t *count_word = reinterpret_cast<uint32_t *>(out + nw);
    if (nblk == 0u) {
      e = hipMemsetAsync(count_word, 0, 4, ctx->stream);
    } else {
      const size_t need = (size_t)2 * nblk * sizeof(uint32_t);
      if (ctx->pack_bytes < need) {
        if (ctx->pack) (void)hipFree(ctx->pack);
        ctx->pack = nullptr;
        ctx->pack_bytes = 0;
        if ((e = hipMalloc(&ctx->pack, need)) != hipSuccess)
          return fail(BZR_ERR_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
        ctx->pack_bytes = need;
      }
      uint32_t *block_count = static_cast<uint32_t *>(ctx->pack), *block_off = block_count + nblk;
      hipLaunchKernelGGL(k_compact_count, dim3(nblk), dim3(kPackThreads), 0, ctx->stream, status, segments, n,
                         reinterpret_cast<unsigned char *>(out), block_count);
      hipLaunchKernelGGL(k_compact_scan, dim3(1), dim3(kScanThreads), 0, ctx->stream, block_count, nblk, block_off,
                         count_word);
      hipLaunchKernelGGL(k_compact_scatter, dim3(nblk), dim3(kPackThreads), 0, ctx->stream, rays_soa, status, segments,
                         n, block_off, cap, out + nw + 1);
      e = hipGetLastError();
    }
  }
  if (e != hipSuccess) return fail(BZR_ERR_HIP, std::string("bzr_pack_frame: ") + hipGetErrorString(e));
  return BZR_OK;
}
