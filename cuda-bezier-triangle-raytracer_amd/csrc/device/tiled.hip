// tiled.hip -- the refraction chain (reference/test.cpp:376-401) over several devices from ONE process, with
// the results gathered to device 0 on the device side (SURVEY.md 8b bzr_trace_tiled, 8e).
//
// A plan (bzr_tiled) deals the tiles of a tile-major frame round-robin to ndev devices: device d owns tiles
// d, d + ndev, d + 2 ndev, ... packed back to back (its "share").  Per frame, on slot s = frame % nslot:
//   1. device d traces its share on ctxs[s * ndev + d]'s stream (bzr_trace_chain, device pointers);
//   2. packs it in bzr_pack_frame's rays layout, [7][npad] floats (6 ray rows + status | segments << 8), or
//      (bzr_tiled_set_layout / bzr_tiled_calibrate) its compact layout: a status/segment byte per ray, the
//      survivor count and the final rays of the survivors only, up to a capacity per share;
//   3. the packed shares travel to device 0: RCCL (ncclCommInitAll over the devices, one grouped call of
//      ncclSend from every rank to rank 0 and ncclRecv of every rank on rank 0 -- rank 0 included, so a
//      one-device plan runs the same collective code) on a plan-owned stream per device, or hipMemcpyPeerAsync
//      when two list entries are the same device (RCCL needs distinct devices);
//   4. k_tiled_unpack on device 0 scatters the gathered shares into the caller's outputs in input order
//      (compact: three kernels -- survivor counts per 1024 columns, their scan per share with the capacity
//      check, the scatter; a ray that never refracted gets its primary ray back from device 0's copy).
// Events order the steps without host waits: the gather waits for each device's pack, the next frame on the
// same slot packs only after that slot's previous gather has left the buffer, device 0's stream of the
// gather serialises the receive buffers.  Bytes: 28 per primary cross to device 0, (ndev - 1) / ndev of them
// over xGMI.  Byte work only: the kernels here are HBM-bound copies.
// A one-device plan (BZR_GATHER_DIRECT, AUTO's choice for ndev == 1) skips steps 2-4: its share is the frame
// in frame order, so each frame is one bzr_trace_chain from the resident rays into the caller's outputs.
// bzr_tiled_set_rays lands the frame on device 0 once and sends every other device only its share.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <string>
#include <vector>

#include "bzr.h"
#include "ctx.hpp"

extern "C" void bzr_internal_set_error(const char *msg);

namespace {

constexpr uint32_t kThreads = 256;
constexpr uint32_t kRows = 7;  // bzr_pack_frame's BZR_PACK_RAYS rows

bzr_status fail(bzr_status s, const std::string &msg) {
  bzr_internal_set_error(msg.c_str());
  return s;
}

#define TILED_HIP(expr)                                                                       \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess) return fail(BZR_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)
#define TILED_NCCL(expr)                                                                      \
  do {                                                                                        \
    ncclResult_t r_ = (expr);                                                                 \
    if (r_ != ncclSuccess) return fail(BZR_ERR_HIP, std::string(#expr ": ") + ncclGetErrorString(r_)); \
  } while (0)

// Column `col` of device d's share <-> ray index of the frame.
__device__ __forceinline__ uint32_t frame_index(uint32_t d, uint32_t col, uint32_t ndev, uint32_t tile_rays) {
  const uint32_t j = col / tile_rays;  // d's j-th tile = frame tile j * ndev + d
  return (j * ndev + d) * tile_rays + (col - j * tile_rays);
}

// Device d's share of a frame-ordered SoA [6][n] (src may live on another device when peer access is on; the
// plan copies it over first otherwise).
__global__ __launch_bounds__(kThreads) void k_share_extract(const float *__restrict__ src, uint32_t n, uint32_t d,
                                                            uint32_t ndev, uint32_t tile_rays, uint32_t nd,
                                                            float *__restrict__ dst) {
  const uint32_t col = blockIdx.x * kThreads + threadIdx.x;
  if (col >= nd) return;
  const uint32_t i = frame_index(d, col, ndev, tile_rays);
#pragma unroll
  for (uint32_t r = 0; r < 6u; ++r) dst[(size_t)r * nd + col] = src[(size_t)r * n + i];
}

// Device 0: the gathered shares recv[d][7][npad] -> frame-ordered outputs.
__global__ __launch_bounds__(kThreads) void k_tiled_unpack(const float *__restrict__ recv, size_t stride, uint32_t ndev,
                                                           uint32_t npad, uint32_t tile_rays, uint32_t n,
                                                           float *__restrict__ out_rays, uint32_t *__restrict__ out_status,
                                                           uint32_t *__restrict__ out_segments) {
  const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = i / tile_rays, d = k % ndev, col = (k / ndev) * tile_rays + (i - k * tile_rays);
  const float *p = recv + (size_t)d * stride + col;
#pragma unroll
  for (uint32_t r = 0; r < 6u; ++r) out_rays[(size_t)r * n + i] = p[(size_t)r * npad];
  const uint32_t word = __float_as_uint(p[(size_t)6 * npad]);
  out_status[i] = word & 0xFFu;
  if (out_segments) out_segments[i] = word >> 8;
}

// Calibration (device 0): survivors of a traced frame per share (frame order in, the deal's share index out).
__global__ __launch_bounds__(kThreads) void k_count_survivors(const uint32_t *__restrict__ status,
                                                              const uint32_t *__restrict__ segments, uint32_t n,
                                                              uint32_t ndev, uint32_t tile_rays,
                                                              uint32_t *__restrict__ count) {
  const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  if (segments[i] >= 2u || status[i] != 0u) atomicAdd(&count[(i / tile_rays) % ndev], 1u);
}

constexpr uint32_t kUnpackThreads = 256;
constexpr uint32_t kUnpackCols = 4 * kUnpackThreads;  // columns per block (bzr_pack_frame's compact blocks)
constexpr uint32_t kUnpackScan = 1024;

__device__ __forceinline__ bool survivor_byte(uint32_t b) { return (b >> 2) >= 2u || (b & 3u) != 0u; }

// Compact pass 1 (device 0): survivors among the columns of block b of share d (blockIdx = d * nblk + b).
__global__ __launch_bounds__(kUnpackThreads) void k_unpack_count(const float *__restrict__ recv, size_t stride,
                                                                 const uint32_t *__restrict__ share, uint32_t nblk,
                                                                 uint32_t *__restrict__ block_count) {
  __shared__ uint32_t wave_sum[kUnpackThreads / 64];
  const uint32_t d = blockIdx.x / nblk, b = blockIdx.x - d * nblk, nd = share[d];
  const unsigned char *bytes = reinterpret_cast<const unsigned char *>(recv + (size_t)d * stride);
  uint32_t mine = 0;
#pragma unroll
  for (uint32_t k = 0; k < 4u; ++k) {
    const uint32_t col = b * kUnpackCols + k * kUnpackThreads + threadIdx.x;
    mine += (uint32_t)__popcll(__ballot(col < nd && survivor_byte(bytes[col])));
  }
  if ((threadIdx.x & 63u) == 0u) wave_sum[threadIdx.x >> 6] = mine;
  __syncthreads();
  if (threadIdx.x == 0u) {
    uint32_t t = 0;
#pragma unroll
    for (uint32_t w = 0; w < kUnpackThreads / 64; ++w) t += wave_sum[w];
    block_count[blockIdx.x] = t;
  }
}

// Compact pass 2 (device 0, one block per share): exclusive offsets of the block counts; a share whose
// survivors do not match its count word, or exceed the capacity, raises the overflow flag (its frame was
// not fully gathered).
__global__ __launch_bounds__(kUnpackScan) void k_unpack_scan(const float *__restrict__ recv, size_t stride, uint32_t cpad,
                                                             uint32_t cap, const uint32_t *__restrict__ share, uint32_t nblk,
                                                             const uint32_t *__restrict__ block_count,
                                                             uint32_t *__restrict__ block_off, uint32_t *__restrict__ flag) {
  __shared__ uint32_t part[kUnpackScan];
  const uint32_t d = blockIdx.x;
  const uint32_t *bc = block_count + (size_t)d * nblk;
  uint32_t *bo = block_off + (size_t)d * nblk;
  const uint32_t per = (nblk + kUnpackScan - 1) / kUnpackScan;
  const uint32_t lo = threadIdx.x * per, hi = min(nblk, lo + per);
  uint32_t sum = 0;
  for (uint32_t b = lo; b < hi; ++b) sum += bc[b];
  part[threadIdx.x] = sum;
  __syncthreads();
  for (uint32_t k = 1; k < kUnpackScan; k <<= 1) {
    const uint32_t v = threadIdx.x >= k ? part[threadIdx.x - k] : 0u;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t run = threadIdx.x ? part[threadIdx.x - 1] : 0u;
  for (uint32_t b = lo; b < hi; ++b) {
    bo[b] = run;
    run += bc[b];
  }
  if (threadIdx.x == kUnpackScan - 1 && share[d] > 0u) {  // (an empty share packed nothing)
    const uint32_t total = part[kUnpackScan - 1];
    const uint32_t count = __float_as_uint(recv[(size_t)d * stride + cpad / 4u]);
    if (total != count || count > cap) atomicOr(flag, 1u);
  }
}

// Compact pass 3 (device 0): every column of share d to its frame position -- a survivor's final ray from
// the packed rows (its rank among the share's survivors), anyone else's primary ray from prim.
__global__ __launch_bounds__(kUnpackThreads) void k_unpack_compact(const float *__restrict__ recv, size_t stride,
                                                                   uint32_t cpad, uint32_t cap,
                                                                   const uint32_t *__restrict__ share, uint32_t nblk,
                                                                   const uint32_t *__restrict__ block_off,
                                                                   const float *__restrict__ prim, uint32_t ndev,
                                                                   uint32_t tile_rays, uint32_t n,
                                                                   float *__restrict__ out_rays,
                                                                   uint32_t *__restrict__ out_status,
                                                                   uint32_t *__restrict__ out_segments) {
  __shared__ uint32_t cnt[4][kUnpackThreads / 64];
  const uint32_t d = blockIdx.x / nblk, b = blockIdx.x - d * nblk, nd = share[d];
  const float *base = recv + (size_t)d * stride;
  const unsigned char *bytes = reinterpret_cast<const unsigned char *>(base);
  const float *rows = base + cpad / 4u + 1u;
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  bool keep[4];
  uint32_t byte[4];
  unsigned long long bal[4];
#pragma unroll
  for (uint32_t k = 0; k < 4u; ++k) {
    const uint32_t col = b * kUnpackCols + k * kUnpackThreads + threadIdx.x;
    byte[k] = col < nd ? bytes[col] : 0u;
    keep[k] = col < nd && survivor_byte(byte[k]);
    bal[k] = __ballot(keep[k]);
    if (lane == 0u) cnt[k][w] = (uint32_t)__popcll(bal[k]);
  }
  __syncthreads();
  const uint32_t off = block_off[(size_t)d * nblk + b];
  const unsigned long long below = lane ? (~0ull >> (64u - lane)) : 0ull;
  uint32_t before = 0;
#pragma unroll
  for (uint32_t k = 0; k < 4u; ++k) {
    for (uint32_t v = 0; v < kUnpackThreads / 64; ++v)
      if (v < w) before += cnt[k][v];
    const uint32_t col = b * kUnpackCols + k * kUnpackThreads + threadIdx.x;
    if (col < nd) {
      const uint32_t i = frame_index(d, col, ndev, tile_rays);
      const uint32_t pos = off + before + (uint32_t)__popcll(bal[k] & below);
      const bool from_rows = keep[k] && pos < cap;
#pragma unroll
      for (uint32_t r = 0; r < 6u; ++r)
        out_rays[(size_t)r * n + i] = from_rows ? rows[(size_t)r * (cap + 1u) + pos] : prim[(size_t)r * n + i];
      out_status[i] = byte[k] & 3u;
      if (out_segments) out_segments[i] = byte[k] >> 2;
    }
    for (uint32_t v = w; v < kUnpackThreads / 64; ++v) before += cnt[k][v];
  }
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

}  // namespace

struct bzr_tiled {
  uint32_t ndev = 0, nslot = 0, n = 0, tile_rays = 0, npad = 0;
  int32_t transport = BZR_GATHER_PEER;
  std::vector<bzr_ctx *> ctxs;       // [slot][device]
  std::vector<int> dev;              // HIP device of list entry d
  std::vector<uint32_t> share;       // rays of device d's share
  std::vector<float *> in;           // [d] share input rays [6][share]
  struct Slot {
    std::vector<float *> rays;       // [d] chain outputs (not allocated by a DIRECT plan)
    std::vector<uint32_t *> status, segments;
    std::vector<float *> packed;     // [d] [7][npad]
    float *recv = nullptr;           // device 0: [ndev][7][npad]
    std::vector<hipEvent_t> packed_ev;  // [d] on ctx stream: share packed (DIRECT: [0] the frame traced)
    // [d] the packed buffer is free again; created on the device of the stream that records it (RCCL: the
    // gather stream of d, on dev[d]; peer: gstream[0], on dev[0]) -- HIP records an event only on a stream of
    // the event's own device
    std::vector<hipEvent_t> sent_ev;
    float *rows = nullptr;           // BZR_RAYS_AOS: device 0, the frame's output rays [6][n] before they become
                                     // records (per slot: a DIRECT frame writes them on its own slot stream)
    bool used = false;
  };
  std::vector<Slot> slot;
  std::vector<hipStream_t> gstream;  // [d] gather stream (RCCL: one per device; peer: only [0])
  std::vector<ncclComm_t> comm;      // RCCL communicators, rank d on dev[d]
  hipEvent_t done = nullptr;         // device 0: last unpack
  float *host_out = nullptr;         // host-pointer frames: device-0 staging for [6][n] + 2 x [n]
  uint64_t frames = 0;
  // gather layout (bzr_tiled_set_layout): BZR_PACK_RAYS, or BZR_PACK_COMPACT with `cap` survivors per share
  int32_t layout = BZR_PACK_RAYS;
  uint32_t cap = 0, cpad = 0;        // compact: capacity; npad rounded up to a multiple of 4 (byte words)
  size_t words = 0;                  // floats of one packed share (the allocation: the larger layout)
  // device 0: the frame's primary rays [6][n] (bzr_tiled_set_rays) -- prim_buf with several devices; with
  // one device the share is the frame in frame order, so prim0 is in[0] itself
  float *prim0 = nullptr, *prim_buf = nullptr;
  float *stage = nullptr;            // device 0: the other devices' shares before their peer copies
  hipEvent_t rays_ev = nullptr;      // device 0, on ctxs[0]'s stream: the last set_rays' copies are queued before it
  uint64_t rays_gen = 0;             // set_rays calls so far; rays_seen[k]: the last one context k's stream waited for
  std::vector<uint64_t> rays_seen;
  bool prim_valid = false;
  uint32_t *dshare = nullptr;        // device 0: share sizes [ndev]
  uint32_t *unpack = nullptr;        // device 0: compact block counts / offsets [2][ndev][nblk], overflow flag
  uint32_t nblk = 0;                 // compact: 1024-column blocks per share
  size_t packed_words() const {
    return layout == BZR_PACK_COMPACT ? (size_t)cpad / 4u + 1u + 6u * ((size_t)cap + 1u) : (size_t)kRows * npad;
  }

  ~bzr_tiled() {
    for (uint32_t d = 0; d < gstream.size(); ++d)
      if (gstream[d]) {
        DeviceGuard g(dev[d]);
        (void)hipStreamSynchronize(gstream[d]);
      }
    for (bzr_ctx *c : ctxs) (void)bzr_sync(c);
    for (ncclComm_t c : comm)
      if (c) (void)ncclCommDestroy(c);
    auto free_on = [](int device, void *p) {
      if (!p) return;
      DeviceGuard g(device);
      (void)hipFree(p);
    };
    for (uint32_t d = 0; d < in.size(); ++d) free_on(dev[d], in[d]);
    for (Slot &s : slot) {
      for (uint32_t d = 0; d < s.rays.size(); ++d) {
        free_on(dev[d], s.rays[d]);
        free_on(dev[d], s.status[d]);
        free_on(dev[d], s.segments[d]);
        free_on(dev[d], s.packed[d]);
      }
      free_on(dev.empty() ? 0 : dev[0], s.recv);
      free_on(dev.empty() ? 0 : dev[0], s.rows);
      for (hipEvent_t e : s.packed_ev) if (e) (void)hipEventDestroy(e);
      for (hipEvent_t e : s.sent_ev) if (e) (void)hipEventDestroy(e);
    }
    if (!dev.empty()) {
      free_on(dev[0], host_out);
      free_on(dev[0], prim_buf);
      free_on(dev[0], stage);
      free_on(dev[0], dshare);
      free_on(dev[0], unpack);
    }
    for (uint32_t d = 0; d < gstream.size(); ++d)
      if (gstream[d]) (void)hipStreamDestroy(gstream[d]);
    if (done) (void)hipEventDestroy(done);
    if (rays_ev) (void)hipEventDestroy(rays_ev);
  }
};

namespace {

template <typename T>
bzr_status alloc_on(int device, T *&p, size_t count) {
  DeviceGuard g(device);
  void *v = nullptr;
  hipError_t e = hipMalloc(&v, std::max<size_t>(count, 1) * sizeof(T));
  if (e != hipSuccess) return fail(BZR_ERR_OUT_OF_MEMORY, std::string("bzr_tiled: hipMalloc: ") + hipGetErrorString(e));
  p = static_cast<T *>(v);
  return BZR_OK;
}

bzr_status build(bzr_tiled &t, bzr_ctx *const *ctxs, int32_t transport) {
  const uint32_t ndev = t.ndev;
  t.ctxs.assign(ctxs, ctxs + (size_t)ndev * t.nslot);
  t.rays_seen.assign(t.ctxs.size(), 0);
  for (uint32_t d = 0; d < ndev; ++d) t.dev.push_back(ctxs[d]->device);
  for (uint32_t s = 1; s < t.nslot; ++s)
    for (uint32_t d = 0; d < ndev; ++d)
      if (ctxs[s * ndev + d]->device != t.dev[d])
        return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_create: slot " + std::to_string(s) + " lists its devices in another order");
  bool distinct = true;
  for (uint32_t d = 0; d < ndev; ++d)
    if (std::count(t.dev.begin(), t.dev.end(), t.dev[d]) > 1) distinct = false;
  if (transport == BZR_GATHER_AUTO)
    transport = ndev == 1 ? BZR_GATHER_DIRECT : distinct ? BZR_GATHER_RCCL : BZR_GATHER_PEER;
  if (transport == BZR_GATHER_RCCL && !distinct)
    return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_create: RCCL needs distinct devices (use BZR_GATHER_PEER)");
  if (transport == BZR_GATHER_DIRECT && ndev != 1)
    return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_create: BZR_GATHER_DIRECT is the one-device plan");
  t.transport = transport;
  const bool direct = transport == BZR_GATHER_DIRECT;

  // the deal: tile k -> device k % ndev
  const uint32_t tiles = (t.n + t.tile_rays - 1) / t.tile_rays;
  t.share.assign(ndev, 0);
  for (uint32_t k = 0; k < tiles; ++k) t.share[k % ndev] += std::min(t.tile_rays, t.n - k * t.tile_rays);
  t.npad = ((tiles + ndev - 1) / ndev) * t.tile_rays;
  t.cpad = (t.npad + 3u) / 4u * 4u;
  t.words = std::max((size_t)kRows * t.npad, (size_t)t.cpad / 4u + 1u + 6u * ((size_t)t.npad + 1u));
  t.nblk = (t.npad + kUnpackCols - 1) / kUnpackCols;

  t.in.assign(ndev, nullptr);
  for (uint32_t d = 0; d < ndev; ++d)
    if (bzr_status s = alloc_on(t.dev[d], t.in[d], (size_t)6 * t.share[d])) return s;
  if (ndev == 1) t.prim0 = t.in[0];  // one device: its share is the frame, in frame order
  t.slot.resize(t.nslot);
  for (auto &sl : t.slot) {
    sl.rays.assign(ndev, nullptr);
    sl.status.assign(ndev, nullptr);
    sl.segments.assign(ndev, nullptr);
    sl.packed.assign(ndev, nullptr);
    sl.packed_ev.assign(ndev, nullptr);
    sl.sent_ev.assign(ndev, nullptr);
    for (uint32_t d = 0; d < ndev; ++d) {
      if (!direct) {  // a DIRECT frame is traced into the caller's outputs: no share outputs, no packing
        if (bzr_status s = alloc_on(t.dev[d], sl.rays[d], (size_t)6 * t.share[d])) return s;
        if (bzr_status s = alloc_on(t.dev[d], sl.status[d], t.share[d])) return s;
        if (bzr_status s = alloc_on(t.dev[d], sl.segments[d], t.share[d])) return s;
        if (bzr_status s = alloc_on(t.dev[d], sl.packed[d], t.words)) return s;
      }
      {
        DeviceGuard g(t.dev[d]);
        TILED_HIP(hipEventCreateWithFlags(&sl.packed_ev[d], hipEventDisableTiming));
      }
      DeviceGuard g(t.transport == BZR_GATHER_RCCL ? t.dev[d] : t.dev[0]);  // the device of the recording stream
      TILED_HIP(hipEventCreateWithFlags(&sl.sent_ev[d], hipEventDisableTiming));
    }
    if (!direct)
      if (bzr_status s = alloc_on(t.dev[0], sl.recv, (size_t)ndev * t.words)) return s;
  }
  const uint32_t nstreams = t.transport == BZR_GATHER_RCCL ? ndev : 1u;
  t.gstream.assign(nstreams, nullptr);
  for (uint32_t d = 0; d < nstreams; ++d) {
    DeviceGuard g(t.dev[d]);
    TILED_HIP(hipStreamCreateWithFlags(&t.gstream[d], hipStreamNonBlocking));
  }
  {
    DeviceGuard g(t.dev[0]);
    TILED_HIP(hipEventCreateWithFlags(&t.done, hipEventDisableTiming));
    TILED_HIP(hipEventCreateWithFlags(&t.rays_ev, hipEventDisableTiming));
    if (bzr_status s = alloc_on(t.dev[0], t.dshare, ndev)) return s;
    if (bzr_status s = alloc_on(t.dev[0], t.unpack, (size_t)2 * ndev * t.nblk + 1)) return s;
    TILED_HIP(hipMemcpy(t.dshare, t.share.data(), ndev * sizeof(uint32_t), hipMemcpyHostToDevice));
    TILED_HIP(hipMemset(t.unpack + (size_t)2 * ndev * t.nblk, 0, sizeof(uint32_t)));
  }
  if (t.transport == BZR_GATHER_RCCL) {
    t.comm.assign(ndev, nullptr);
    TILED_NCCL(ncclCommInitAll(t.comm.data(), static_cast<int>(ndev), t.dev.data()));
  }
  return BZR_OK;
}

}  // namespace

extern "C" bzr_status bzr_tiled_create(bzr_ctx *const *ctxs, uint32_t ndev, uint32_t nslot, uint32_t n,
                                       uint32_t tile_rays, int32_t transport, bzr_tiled **out) {
  if (!out) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_create: null out");
  *out = nullptr;
  if (!ctxs || ndev == 0 || nslot == 0) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_create: no contexts");
  if (tile_rays == 0) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_create: tile_rays must be > 0");
  if (n == 0) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_create: empty frame");
  if (transport != BZR_GATHER_AUTO && transport != BZR_GATHER_RCCL && transport != BZR_GATHER_PEER &&
      transport != BZR_GATHER_DIRECT)
    return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_create: unknown transport " + std::to_string(transport));
  const size_t nctx = (size_t)ndev * nslot;
  for (size_t k = 0; k < nctx; ++k)
    if (!ctxs[k] || std::find(ctxs, ctxs + k, ctxs[k]) != ctxs + k)
      return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_create: null or repeated context (one stream per slot and device)");
  auto *t = new (std::nothrow) bzr_tiled;
  if (!t) return fail(BZR_ERR_OUT_OF_MEMORY, "bzr_tiled_create: out of host memory");
  t->ndev = ndev;
  t->nslot = nslot;
  t->n = n;
  t->tile_rays = tile_rays;
  bzr_status s;
  try {
    s = build(*t, ctxs, transport);
  } catch (std::exception const &e) {
    s = fail(BZR_ERR_OUT_OF_MEMORY, std::string("bzr_tiled_create: ") + e.what());
  }
  if (s != BZR_OK) {
    delete t;
    return s;
  }
  *out = t;
  return BZR_OK;
}

extern "C" bzr_status bzr_tiled_destroy(bzr_tiled *t) {
  delete t;
  return BZR_OK;
}

extern "C" bzr_status bzr_tiled_info(const bzr_tiled *t, int32_t *transport, uint32_t *share_rays, uint32_t *npad) {
  if (!t) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_info: null plan");
  if (transport) *transport = t->transport;
  if (share_rays) std::copy(t->share.begin(), t->share.end(), share_rays);
  if (npad) *npad = t->npad;
  return BZR_OK;
}

extern "C" bzr_status bzr_tiled_share_rays(bzr_tiled *t, uint32_t d, float **rays_soa) {
  if (!t || !rays_soa) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_share_rays: null argument");
  if (d >= t->ndev) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_share_rays: device index out of range");
  *rays_soa = t->in[d];
  t->prim_valid = false;  // the caller writes the shares: device 0's copy of the frame is no longer known good
  return BZR_OK;
}

extern "C" bzr_status bzr_tiled_set_rays(bzr_tiled *t, const float *rays, uint32_t flags) {
  if (!t) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_set_rays: null plan");
  if (!rays) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_set_rays: null rays");
  if (flags & ~uint32_t(BZR_DEVICE_PTRS | BZR_RAYS_AOS))
    return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_set_rays: unknown flags");
  // frames in flight read the share inputs and device 0's frame copy: they finish first
  if (bzr_status s = bzr_tiled_sync(t)) return s;
  t->prim_valid = false;
  const size_t bytes = (size_t)6 * t->n * sizeof(float);
  // Device 0 keeps the whole frame (the compact layout returns a ray that never refracted from it): one copy
  // there, then device 0 extracts every share and sends each other device only its own -- (ndev - 1) / ndev
  // of the frame over xGMI in all.  Everything is queued on ctxs[0]'s stream; rays_ev orders the slots'
  // next frames after it, with no host wait (a host source is waited for, so the caller may reuse it).
  if (t->ndev > 1 && !t->prim_buf)
    if (bzr_status s = alloc_on(t->dev[0], t->prim_buf, (size_t)6 * t->n)) return s;
  if (t->ndev > 1) t->prim0 = t->prim_buf;
  size_t stage_words = 0;
  for (uint32_t d = 1; d < t->ndev; ++d)
    if (t->dev[d] != t->dev[0]) stage_words += (size_t)6 * t->share[d];
  if (stage_words && !t->stage)
    if (bzr_status s = alloc_on(t->dev[0], t->stage, stage_words)) return s;
  bzr_ctx *c0 = t->ctxs[0];
  DeviceGuard g(t->dev[0]);
  const bool host = !(flags & BZR_DEVICE_PTRS), aos = (flags & BZR_RAYS_AOS) != 0;
  if (aos) {  // [n][6] records: (copied to device 0's host_out staging, idle after the sync above and) transposed
    const float *src = rays;
    if (host) {
      if (!t->host_out)
        if (bzr_status s = alloc_on(t->dev[0], t->host_out, (size_t)8 * t->n)) return s;
      TILED_HIP(hipMemcpyAsync(t->host_out, rays, bytes, hipMemcpyHostToDevice, c0->stream));
      src = t->host_out;
    }
    TILED_HIP(bzr_rays_relayout(c0->stream, src, t->prim0, t->n, true));
  } else {
    TILED_HIP(hipMemcpyAsync(t->prim0, rays, bytes, host ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice, c0->stream));
  }
  if (host) TILED_HIP(hipStreamSynchronize(c0->stream));  // the caller's host buffer has been read
  if (t->ndev > 1) {
    size_t off = 0;
    for (uint32_t d = 0; d < t->ndev; ++d) {
      if (t->share[d] == 0) continue;
      const bool local = t->dev[d] == t->dev[0];
      float *dst = local ? t->in[d] : t->stage + off;
      hipLaunchKernelGGL(k_share_extract, dim3((t->share[d] + kThreads - 1) / kThreads), dim3(kThreads), 0, c0->stream,
                         t->prim0, t->n, d, t->ndev, t->tile_rays, t->share[d], dst);
      TILED_HIP(hipGetLastError());
      if (!local) {
        TILED_HIP(hipMemcpyPeerAsync(t->in[d], t->dev[d], dst, t->dev[0], (size_t)6 * t->share[d] * sizeof(float),
                                     c0->stream));
        off += (size_t)6 * t->share[d];
      }
    }
  }
  TILED_HIP(hipEventRecord(t->rays_ev, c0->stream));
  ++t->rays_gen;
  t->prim_valid = true;
  return BZR_OK;
}

namespace {

bzr_status gather_and_unpack(bzr_tiled &t, bzr_tiled::Slot &sl, float *out_rays, uint32_t *out_status,
                             uint32_t *out_segments) {
  const size_t count = t.packed_words(), stride = t.words;
  if (t.transport == BZR_GATHER_RCCL) {
    for (uint32_t d = 0; d < t.ndev; ++d) {
      DeviceGuard g(t.dev[d]);
      TILED_HIP(hipStreamWaitEvent(t.gstream[d], sl.packed_ev[d], 0));
    }
    TILED_NCCL(ncclGroupStart());
    for (uint32_t d = 0; d < t.ndev; ++d) {
      ncclResult_t r = ncclSend(sl.packed[d], count, ncclFloat32, 0, t.comm[d], t.gstream[d]);
      if (r == ncclSuccess) r = ncclRecv(sl.recv + (size_t)d * stride, count, ncclFloat32, static_cast<int>(d), t.comm[0],
                                         t.gstream[0]);
      if (r != ncclSuccess) {
        (void)ncclGroupEnd();
        return fail(BZR_ERR_HIP, std::string("bzr_tiled_trace: ncclSend/ncclRecv: ") + ncclGetErrorString(r));
      }
    }
    TILED_NCCL(ncclGroupEnd());
    for (uint32_t d = 0; d < t.ndev; ++d) {
      DeviceGuard g(t.dev[d]);
      TILED_HIP(hipEventRecord(sl.sent_ev[d], t.gstream[d]));
    }
  } else {
    DeviceGuard g(t.dev[0]);
    for (uint32_t d = 0; d < t.ndev; ++d) {
      TILED_HIP(hipStreamWaitEvent(t.gstream[0], sl.packed_ev[d], 0));
      TILED_HIP(hipMemcpyPeerAsync(sl.recv + (size_t)d * stride, t.dev[0], sl.packed[d], t.dev[d], count * sizeof(float),
                                   t.gstream[0]));
    }
    for (uint32_t d = 0; d < t.ndev; ++d) TILED_HIP(hipEventRecord(sl.sent_ev[d], t.gstream[0]));
  }
  DeviceGuard g(t.dev[0]);
  if (t.layout == BZR_PACK_COMPACT) {
    uint32_t *bc = t.unpack, *bo = t.unpack + (size_t)t.ndev * t.nblk, *flag = t.unpack + (size_t)2 * t.ndev * t.nblk;
    const dim3 grid(t.ndev * t.nblk);
    hipLaunchKernelGGL(k_unpack_count, grid, dim3(kUnpackThreads), 0, t.gstream[0], sl.recv, stride, t.dshare, t.nblk, bc);
    hipLaunchKernelGGL(k_unpack_scan, dim3(t.ndev), dim3(kUnpackScan), 0, t.gstream[0], sl.recv, stride, t.cpad, t.cap,
                       t.dshare, t.nblk, bc, bo, flag);
    hipLaunchKernelGGL(k_unpack_compact, grid, dim3(kUnpackThreads), 0, t.gstream[0], sl.recv, stride, t.cpad, t.cap,
                       t.dshare, t.nblk, bo, t.prim0, t.ndev, t.tile_rays, t.n, out_rays, out_status, out_segments);
  } else {
    hipLaunchKernelGGL(k_tiled_unpack, dim3((t.n + kThreads - 1) / kThreads), dim3(kThreads), 0, t.gstream[0], sl.recv,
                       stride, t.ndev, t.npad, t.tile_rays, t.n, out_rays, out_status, out_segments);
  }
  TILED_HIP(hipGetLastError());
  TILED_HIP(hipEventRecord(t.done, t.gstream[0]));
  return BZR_OK;
}

}  // namespace

extern "C" bzr_status bzr_tiled_trace(bzr_tiled *t, const bzr_mesh *const *lenses, const float *ri, uint32_t nlens,
                                      float *out_rays, uint32_t *out_status, uint32_t *out_segments, uint32_t flags) {
  if (!t) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_trace: null plan");
  if (!lenses || !ri || nlens == 0) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_trace: null lens list");
  if (!out_rays || !out_status) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_trace: null output");
  const bool host = !(flags & BZR_DEVICE_PTRS), aos = (flags & BZR_RAYS_AOS) != 0;
  const uint32_t cflags = (flags & ~uint32_t(BZR_RAYS_AOS)) | BZR_DEVICE_PTRS;  // the share inputs are rows
  if (t->layout == BZR_PACK_COMPACT && !t->prim_valid)
    return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_trace: the compact layout needs the frame's rays through "
                                          "bzr_tiled_set_rays (device 0 returns the rays that never refracted)");
  const uint32_t s = static_cast<uint32_t>(t->frames % t->nslot);
  bzr_tiled::Slot &sl = t->slot[s];
  for (uint32_t d = 0; d < t->ndev; ++d) {  // the slot's streams see the last set_rays' copies
    const size_t k = (size_t)s * t->ndev + d;
    if (t->rays_seen[k] != t->rays_gen) {
      DeviceGuard g(t->dev[d]);
      TILED_HIP(hipStreamWaitEvent(t->ctxs[k]->stream, t->rays_ev, 0));
      t->rays_seen[k] = t->rays_gen;
    }
  }
  // where the frame's outputs land on device 0: the caller's device buffers, or staging -- host outputs in
  // host_out ([6][n] rays, status, segments; copied back and waited for), BZR_RAYS_AOS rays in the slot's rows
  // (then transposed into the caller's records, or into host_out's rays for a host caller)
  float *o_rays = out_rays;
  uint32_t *o_st = out_status, *o_seg = out_segments;
  if (host) {
    if (!t->host_out)
      if (bzr_status st = alloc_on(t->dev[0], t->host_out, (size_t)8 * t->n)) return st;
    o_rays = t->host_out;
    o_st = reinterpret_cast<uint32_t *>(t->host_out + (size_t)6 * t->n);
    o_seg = o_st + t->n;
  }
  if (aos) {
    if (!sl.rows)
      if (bzr_status st = alloc_on(t->dev[0], sl.rows, (size_t)6 * t->n)) return st;
    o_rays = sl.rows;
  }
  // on device 0's stream that produced them: AoS records, then the copies back to the host
  auto deliver = [&](hipStream_t os) -> bzr_status {
    DeviceGuard g(t->dev[0]);
    if (aos) TILED_HIP(bzr_rays_relayout(os, sl.rows, host ? t->host_out : out_rays, t->n, false));
    if (!host) return BZR_OK;
    TILED_HIP(hipMemcpyAsync(out_rays, t->host_out, (size_t)24 * t->n, hipMemcpyDeviceToHost, os));
    TILED_HIP(hipMemcpyAsync(out_status, o_st, (size_t)4 * t->n, hipMemcpyDeviceToHost, os));
    if (out_segments) TILED_HIP(hipMemcpyAsync(out_segments, o_seg, (size_t)4 * t->n, hipMemcpyDeviceToHost, os));
    TILED_HIP(hipStreamSynchronize(os));
    return BZR_OK;
  };
  if (t->transport == BZR_GATHER_DIRECT) {
    // one device: its share is the frame in frame order -- trace straight into the outputs (or the staging
    // above, delivered on the same stream), then hand the frame to the gather stream so bzr_tiled_stream keeps
    // its meaning
    bzr_ctx *c = t->ctxs[s];
    bzr_status st = bzr_trace_chain(c, lenses, ri, nlens, t->in[0], t->n, o_rays, o_st, o_seg, cflags);
    if (st != BZR_OK) return fail(st, std::string("bzr_tiled_trace: ") + bzr_last_error());
    ++t->frames;
    if (bzr_status e = deliver(c->stream)) return e;
    if (host) return BZR_OK;
    DeviceGuard g(t->dev[0]);
    TILED_HIP(hipEventRecord(sl.packed_ev[0], c->stream));
    TILED_HIP(hipStreamWaitEvent(t->gstream[0], sl.packed_ev[0], 0));
    return BZR_OK;
  }
  for (uint32_t d = 0; d < t->ndev; ++d) {
    bzr_ctx *c = t->ctxs[(size_t)s * t->ndev + d];
    if (t->share[d]) {
      bzr_status st = bzr_trace_chain(c, lenses + (size_t)d * nlens, ri, nlens, t->in[d], t->share[d], sl.rays[d],
                                      sl.status[d], sl.segments[d], cflags);
      if (st != BZR_OK) return fail(st, "bzr_tiled_trace: device " + std::to_string(d) + ": " + bzr_last_error());
    }
    DeviceGuard g(t->dev[d]);
    if (sl.used) TILED_HIP(hipStreamWaitEvent(c->stream, sl.sent_ev[d], 0));  // the previous gather left the buffer
    if (t->share[d]) {
      const bool compact = t->layout == BZR_PACK_COMPACT;
      bzr_status st = bzr_pack_frame(c, t->layout, sl.rays[d], sl.status[d], sl.segments[d], t->share[d],
                                     compact ? t->cpad : t->npad, compact ? t->cap : 0u, sl.packed[d]);
      if (st != BZR_OK) return fail(st, "bzr_tiled_trace: pack, device " + std::to_string(d) + ": " + bzr_last_error());
    }
    TILED_HIP(hipEventRecord(sl.packed_ev[d], c->stream));
  }
  sl.used = true;
  ++t->frames;
  if (bzr_status st = gather_and_unpack(*t, sl, o_rays, o_st, o_seg)) return st;
  if (bzr_status st = deliver(t->gstream[0])) return st;
  if (host && t->layout == BZR_PACK_COMPACT) {  // a synchronous caller learns of an incomplete frame now
    DeviceGuard g(t->dev[0]);
    uint32_t *flag = t->unpack + (size_t)2 * t->ndev * t->nblk, h = 0;
    TILED_HIP(hipMemcpy(&h, flag, sizeof(h), hipMemcpyDeviceToHost));
    if (h) {
      TILED_HIP(hipMemset(flag, 0, sizeof(h)));
      return fail(BZR_ERR_CAPACITY, "bzr_tiled_trace: the frame had more survivors than the compact capacity " +
                                        std::to_string(t->cap) + ": its outputs are incomplete (bzr_tiled_calibrate "
                                        "or a larger cap)");
    }
  }
  return BZR_OK;
}

extern "C" bzr_status bzr_tiled_stream(bzr_tiled *t, void **hip_stream) {
  if (!t || !hip_stream) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_stream: null argument");
  *hip_stream = t->gstream[0];
  return BZR_OK;
}

extern "C" bzr_status bzr_tiled_sync(bzr_tiled *t) {
  if (!t) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_sync: null plan");
  for (uint32_t d = 0; d < t->gstream.size(); ++d) {
    DeviceGuard g(t->dev[d]);
    TILED_HIP(hipStreamSynchronize(t->gstream[d]));
  }
  for (bzr_ctx *c : t->ctxs)
    if (bzr_status s = bzr_sync(c)) return s;
  if (t->unpack) {  // a compact frame whose survivors exceeded the capacity since the last sync
    DeviceGuard g(t->dev[0]);
    uint32_t *flag = t->unpack + (size_t)2 * t->ndev * t->nblk, h = 0;
    TILED_HIP(hipMemcpy(&h, flag, sizeof(h), hipMemcpyDeviceToHost));
    if (h) {
      TILED_HIP(hipMemset(flag, 0, sizeof(h)));
      return fail(BZR_ERR_CAPACITY, "bzr_tiled_sync: a frame had more survivors than the compact capacity " +
                                        std::to_string(t->cap) + ": its outputs are incomplete (bzr_tiled_calibrate or a "
                                        "larger cap)");
    }
  }
  return BZR_OK;
}

extern "C" bzr_status bzr_tiled_set_layout(bzr_tiled *t, int32_t layout, uint32_t cap) {
  if (!t) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_set_layout: null plan");
  if (layout != BZR_PACK_RAYS && layout != BZR_PACK_COMPACT)
    return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_set_layout: BZR_PACK_RAYS or BZR_PACK_COMPACT");
  if (layout == BZR_PACK_COMPACT && (cap == 0 || cap > t->npad))
    return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_set_layout: compact needs 0 < cap <= npad (" + std::to_string(t->npad) + ")");
  if (bzr_status s = bzr_tiled_sync(t)) return s;  // frames in flight finish under the old layout
  t->layout = layout;
  t->cap = layout == BZR_PACK_COMPACT ? cap : 0u;
  return BZR_OK;
}

extern "C" bzr_status bzr_tiled_calibrate(bzr_tiled *t, const bzr_mesh *const *lenses, const float *ri, uint32_t nlens,
                                          uint32_t flags, uint32_t *cap_out) {
  if (!t) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_calibrate: null plan");
  if (!t->prim_valid)
    return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_calibrate: set the frame's rays first (bzr_tiled_set_rays)");
  if (bzr_status s = bzr_tiled_set_layout(t, BZR_PACK_RAYS, 0)) return s;
  float *o = nullptr;
  uint32_t *cnt = nullptr;
  if (bzr_status s = alloc_on(t->dev[0], o, (size_t)8 * t->n)) return s;
  bzr_status s = alloc_on(t->dev[0], cnt, t->ndev);
  uint32_t *st = reinterpret_cast<uint32_t *>(o + (size_t)6 * t->n), *sg = st + t->n;
  if (s == BZR_OK) s = bzr_tiled_trace(t, lenses, ri, nlens, o, st, sg, flags | BZR_DEVICE_PTRS);
  std::vector<uint32_t> h(t->ndev, 0u);
  if (s == BZR_OK) {
    DeviceGuard g(t->dev[0]);
    hipStream_t gs = t->gstream[0];
    hipError_t e = hipMemsetAsync(cnt, 0, t->ndev * sizeof(uint32_t), gs);
    if (e == hipSuccess) {
      hipLaunchKernelGGL(k_count_survivors, dim3((t->n + kThreads - 1) / kThreads), dim3(kThreads), 0, gs, st, sg, t->n,
                         t->ndev, t->tile_rays, cnt);
      e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(h.data(), cnt, t->ndev * sizeof(uint32_t), hipMemcpyDeviceToHost, gs);
    if (e == hipSuccess) e = hipStreamSynchronize(gs);
    if (e != hipSuccess) s = fail(BZR_ERR_HIP, std::string("bzr_tiled_calibrate: ") + hipGetErrorString(e));
  }
  if (s == BZR_OK) s = bzr_tiled_sync(t);
  {
    DeviceGuard g(t->dev[0]);
    (void)hipFree(o);
    if (cnt) (void)hipFree(cnt);
  }
  if (s != BZR_OK) return s;
  // the largest share's survivors + 1/64 + 64 rays of headroom (bench.py's rule, frame.compact_capacity)
  const uint32_t most = *std::max_element(h.begin(), h.end());
  const uint32_t cap = static_cast<uint32_t>(std::min<uint64_t>(t->npad, (uint64_t)most + most / 64u + 64u));
  if (cap_out) *cap_out = cap;
  return bzr_tiled_set_layout(t, BZR_PACK_COMPACT, cap);
}

// The one-call form (include/bzr.h): a one-slot plan over ctxs for this frame only.  Host pointers: results
// copied back to host memory.  BZR_DEVICE_PTRS: rays and outputs on ctxs[0]'s device; returns once the
// results are complete (the plan is freed).
extern "C" bzr_status bzr_trace_tiled(bzr_ctx *const *ctxs, uint32_t nctx, const bzr_mesh *const *lenses,
                                      const float *ri, uint32_t nlens, const float *rays, uint32_t n,
                                      uint32_t tile_rays, float *out_rays, uint32_t *out_status,
                                      uint32_t *out_segments, uint32_t flags) {
  if (nctx == 0 || !ctxs) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_trace_tiled: no contexts");
  for (uint32_t d = 0; d < nctx; ++d)
    if (!ctxs[d] || std::find(ctxs, ctxs + d, ctxs[d]) != ctxs + d)
      return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_trace_tiled: null or repeated context (one host thread per context)");
  if (!lenses || !ri || nlens == 0) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_trace_tiled: null lens list");
  if (tile_rays == 0) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_trace_tiled: tile_rays must be > 0");
  if (n == 0) return BZR_OK;
  if (!rays || !out_rays || !out_status) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_trace_tiled: null buffer");
  bzr_tiled *t = nullptr;
  if (bzr_status s = bzr_tiled_create(ctxs, nctx, 1, n, tile_rays, BZR_GATHER_AUTO, &t)) return s;
  bzr_status s = bzr_tiled_set_rays(t, rays, flags & (BZR_DEVICE_PTRS | BZR_RAYS_AOS));
  if (s == BZR_OK) s = bzr_tiled_trace(t, lenses, ri, nlens, out_rays, out_status, out_segments, flags);
  if (s == BZR_OK) s = bzr_tiled_sync(t);
  bzr_tiled_destroy(t);
  return s;
}
