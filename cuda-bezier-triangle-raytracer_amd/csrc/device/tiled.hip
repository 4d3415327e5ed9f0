// tiled.hip -- the refraction chain (reference/test.cpp:376-401) over several devices from ONE process, with
// the results gathered to device 0 on the device side (SURVEY.md 8b bzr_trace_tiled, 8e).
//
// A plan (bzr_tiled) deals the tiles of a tile-major frame round-robin to ndev devices: device d owns tiles
// d, d + ndev, d + 2 ndev, ... packed back to back (its "share").  Per frame, on slot s = frame % nslot:
//   1. device d traces its share on ctxs[s * ndev + d]'s stream (bzr_trace_chain, device pointers);
//   2. packs it in bzr_pack_frame's rays layout, [7][npad] floats (6 ray rows + status | segments << 8);
//   3. the packed shares travel to device 0: RCCL (ncclCommInitAll over the devices, one grouped call of
//      ncclSend from every rank to rank 0 and ncclRecv of every rank on rank 0 -- rank 0 included, so a
//      one-device plan runs the same collective code) on a plan-owned stream per device, or hipMemcpyPeerAsync
//      when two list entries are the same device (RCCL needs distinct devices);
//   4. k_tiled_unpack on device 0 scatters the gathered shares into the caller's outputs in input order.
// Events order the steps without host waits: the gather waits for each device's pack, the next frame on the
// same slot packs only after that slot's previous gather has left the buffer, device 0's stream of the
// gather serialises the receive buffers.  Bytes: 28 per primary cross to device 0, (ndev - 1) / ndev of them
// over xGMI.  Byte work only: the kernels here are HBM-bound copies.
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
__global__ __launch_bounds__(kThreads) void k_tiled_unpack(const float *__restrict__ recv, uint32_t ndev, uint32_t npad,
                                                           uint32_t tile_rays, uint32_t n, float *__restrict__ out_rays,
                                                           uint32_t *__restrict__ out_status,
                                                           uint32_t *__restrict__ out_segments) {
  const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = i / tile_rays, d = k % ndev, col = (k / ndev) * tile_rays + (i - k * tile_rays);
  const float *p = recv + (size_t)d * kRows * npad + col;
#pragma unroll
  for (uint32_t r = 0; r < 6u; ++r) out_rays[(size_t)r * n + i] = p[(size_t)r * npad];
  const uint32_t word = __float_as_uint(p[(size_t)6 * npad]);
  out_status[i] = word & 0xFFu;
  if (out_segments) out_segments[i] = word >> 8;
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
    std::vector<float *> rays;       // [d] chain outputs
    std::vector<uint32_t *> status, segments;
    std::vector<float *> packed;     // [d] [7][npad]
    float *recv = nullptr;           // device 0: [ndev][7][npad]
    std::vector<hipEvent_t> packed_ev;  // [d] on ctx stream: share packed
    std::vector<hipEvent_t> sent_ev;    // [d] on the gather stream of d: packed buffer free again
    bool used = false;
  };
  std::vector<Slot> slot;
  std::vector<hipStream_t> gstream;  // [d] gather stream (RCCL: one per device; peer: only [0])
  std::vector<ncclComm_t> comm;      // RCCL communicators, rank d on dev[d]
  hipEvent_t done = nullptr;         // device 0: last unpack
  float *host_out = nullptr;         // host-pointer frames: device-0 staging for [6][n] + 2 x [n]
  uint64_t frames = 0;

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
      for (hipEvent_t e : s.packed_ev) if (e) (void)hipEventDestroy(e);
      for (hipEvent_t e : s.sent_ev) if (e) (void)hipEventDestroy(e);
    }
    if (!dev.empty()) free_on(dev[0], host_out);
    for (uint32_t d = 0; d < gstream.size(); ++d)
      if (gstream[d]) (void)hipStreamDestroy(gstream[d]);
    if (done) (void)hipEventDestroy(done);
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
  for (uint32_t d = 0; d < ndev; ++d) t.dev.push_back(ctxs[d]->device);
  for (uint32_t s = 1; s < t.nslot; ++s)
    for (uint32_t d = 0; d < ndev; ++d)
      if (ctxs[s * ndev + d]->device != t.dev[d])
        return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_create: slot " + std::to_string(s) + " lists its devices in another order");
  bool distinct = true;
  for (uint32_t d = 0; d < ndev; ++d)
    if (std::count(t.dev.begin(), t.dev.end(), t.dev[d]) > 1) distinct = false;
  if (transport == BZR_GATHER_AUTO) transport = distinct ? BZR_GATHER_RCCL : BZR_GATHER_PEER;
  if (transport == BZR_GATHER_RCCL && !distinct)
    return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_create: RCCL needs distinct devices (use BZR_GATHER_PEER)");
  t.transport = transport;

  // the deal: tile k -> device k % ndev
  const uint32_t tiles = (t.n + t.tile_rays - 1) / t.tile_rays;
  t.share.assign(ndev, 0);
  for (uint32_t k = 0; k < tiles; ++k) t.share[k % ndev] += std::min(t.tile_rays, t.n - k * t.tile_rays);
  t.npad = ((tiles + ndev - 1) / ndev) * t.tile_rays;

  t.in.assign(ndev, nullptr);
  for (uint32_t d = 0; d < ndev; ++d)
    if (bzr_status s = alloc_on(t.dev[d], t.in[d], (size_t)6 * t.share[d])) return s;
  t.slot.resize(t.nslot);
  for (auto &sl : t.slot) {
    sl.rays.assign(ndev, nullptr);
    sl.status.assign(ndev, nullptr);
    sl.segments.assign(ndev, nullptr);
    sl.packed.assign(ndev, nullptr);
    sl.packed_ev.assign(ndev, nullptr);
    sl.sent_ev.assign(ndev, nullptr);
    for (uint32_t d = 0; d < ndev; ++d) {
      if (bzr_status s = alloc_on(t.dev[d], sl.rays[d], (size_t)6 * t.share[d])) return s;
      if (bzr_status s = alloc_on(t.dev[d], sl.status[d], t.share[d])) return s;
      if (bzr_status s = alloc_on(t.dev[d], sl.segments[d], t.share[d])) return s;
      if (bzr_status s = alloc_on(t.dev[d], sl.packed[d], (size_t)kRows * t.npad)) return s;
      DeviceGuard g(t.dev[d]);
      TILED_HIP(hipEventCreateWithFlags(&sl.packed_ev[d], hipEventDisableTiming));
      TILED_HIP(hipEventCreateWithFlags(&sl.sent_ev[d], hipEventDisableTiming));
    }
    if (bzr_status s = alloc_on(t.dev[0], sl.recv, (size_t)ndev * kRows * t.npad)) return s;
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
  if (transport != BZR_GATHER_AUTO && transport != BZR_GATHER_RCCL && transport != BZR_GATHER_PEER)
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
  return BZR_OK;
}

extern "C" bzr_status bzr_tiled_set_rays(bzr_tiled *t, const float *rays, uint32_t flags) {
  if (!t) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_set_rays: null plan");
  if (!rays) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_set_rays: null rays");
  if (flags & ~uint32_t(BZR_DEVICE_PTRS)) return fail(BZR_ERR_INVALID_ARGUMENT, "bzr_tiled_set_rays: unknown flags");
  const size_t bytes = (size_t)6 * t->n * sizeof(float);
  // the whole frame on each device (host: H2D; device 0: peer copies), then each device extracts its share
  const float *src0 = rays;
  float *stage0 = nullptr;
  bzr_ctx *c0 = t->ctxs[0];
  if (!(flags & BZR_DEVICE_PTRS)) {
    if (bzr_status s = alloc_on(t->dev[0], stage0, (size_t)6 * t->n)) return s;
    DeviceGuard g(t->dev[0]);
    hipError_t e = hipMemcpyAsync(stage0, rays, bytes, hipMemcpyHostToDevice, c0->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c0->stream);
    if (e != hipSuccess) {
      (void)hipFree(stage0);
      return fail(BZR_ERR_HIP, std::string("bzr_tiled_set_rays: ") + hipGetErrorString(e));
    }
    src0 = stage0;
  }
  bzr_status result = BZR_OK;
  for (uint32_t d = 0; d < t->ndev && result == BZR_OK; ++d) {
    if (t->share[d] == 0) continue;
    bzr_ctx *c = t->ctxs[d];
    const float *src = src0;
    float *tmp = nullptr;
    if (t->dev[d] != t->dev[0]) {
      if ((result = alloc_on(t->dev[d], tmp, (size_t)6 * t->n)) != BZR_OK) break;
      DeviceGuard g(t->dev[d]);
      hipError_t e = hipMemcpyPeerAsync(tmp, t->dev[d], src0, t->dev[0], bytes, c->stream);
      if (e != hipSuccess) result = fail(BZR_ERR_HIP, std::string("bzr_tiled_set_rays: peer copy: ") + hipGetErrorString(e));
      src = tmp;
    }
    if (result == BZR_OK) {
      DeviceGuard g(t->dev[d]);
      hipLaunchKernelGGL(k_share_extract, dim3((t->share[d] + kThreads - 1) / kThreads), dim3(kThreads), 0, c->stream,
                         src, t->n, d, t->ndev, t->tile_rays, t->share[d], t->in[d]);
      hipError_t e = hipGetLastError();
      if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
      if (e != hipSuccess) result = fail(BZR_ERR_HIP, std::string("bzr_tiled_set_rays: ") + hipGetErrorString(e));
    }
    if (tmp) {
      DeviceGuard g(t->dev[d]);
      (void)hipFree(tmp);
    }
  }
  if (stage0) {
    DeviceGuard g(t->dev[0]);
    (void)hipFree(stage0);
  }
  // every slot's stream sees the rays (the extract ran on slot 0's streams, now synchronised)
  return result;
}

namespace {

bzr_status gather_and_unpack(bzr_tiled &t, bzr_tiled::Slot &sl, float *out_rays, uint32_t *out_status,
                             uint32_t *out_segments) {
  const size_t count = (size_t)kRows * t.npad;
  if (t.transport == BZR_GATHER_RCCL) {
    for (uint32_t d = 0; d < t.ndev; ++d) {
      DeviceGuard g(t.dev[d]);
      TILED_HIP(hipStreamWaitEvent(t.gstream[d], sl.packed_ev[d], 0));
    }
    TILED_NCCL(ncclGroupStart());
    for (uint32_t d = 0; d < t.ndev; ++d) {
      ncclResult_t r = ncclSend(sl.packed[d], count, ncclFloat32, 0, t.comm[d], t.gstream[d]);
      if (r == ncclSuccess) r = ncclRecv(sl.recv + (size_t)d * count, count, ncclFloat32, static_cast<int>(d), t.comm[0],
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
      TILED_HIP(hipMemcpyPeerAsync(sl.recv + (size_t)d * count, t.dev[0], sl.packed[d], t.dev[d], count * sizeof(float),
                                   t.gstream[0]));
    }
    for (uint32_t d = 0; d < t.ndev; ++d) TILED_HIP(hipEventRecord(sl.sent_ev[d], t.gstream[0]));
  }
  DeviceGuard g(t.dev[0]);
  hipLaunchKernelGGL(k_tiled_unpack, dim3((t.n + kThreads - 1) / kThreads), dim3(kThreads), 0, t.gstream[0], sl.recv,
                     t.ndev, t.npad, t.tile_rays, t.n, out_rays, out_status, out_segments);
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
  const bool host = !(flags & BZR_DEVICE_PTRS);
  const uint32_t s = static_cast<uint32_t>(t->frames % t->nslot);
  bzr_tiled::Slot &sl = t->slot[s];
  for (uint32_t d = 0; d < t->ndev; ++d) {
    bzr_ctx *c = t->ctxs[(size_t)s * t->ndev + d];
    if (t->share[d]) {
      bzr_status st = bzr_trace_chain(c, lenses + (size_t)d * nlens, ri, nlens, t->in[d], t->share[d], sl.rays[d],
                                      sl.status[d], sl.segments[d], flags | BZR_DEVICE_PTRS);
      if (st != BZR_OK) return fail(st, "bzr_tiled_trace: device " + std::to_string(d) + ": " + bzr_last_error());
    }
    DeviceGuard g(t->dev[d]);
    if (sl.used) TILED_HIP(hipStreamWaitEvent(c->stream, sl.sent_ev[d], 0));  // the previous gather left the buffer
    if (t->share[d]) {
      bzr_status st = bzr_pack_frame(c, BZR_PACK_RAYS, sl.rays[d], sl.status[d], sl.segments[d], t->share[d], t->npad, 0,
                                     sl.packed[d]);
      if (st != BZR_OK) return fail(st, "bzr_tiled_trace: pack, device " + std::to_string(d) + ": " + bzr_last_error());
    }
    TILED_HIP(hipEventRecord(sl.packed_ev[d], c->stream));
  }
  sl.used = true;
  ++t->frames;
  float *o_rays = out_rays;
  uint32_t *o_st = out_status, *o_seg = out_segments;
  if (host) {  // unpack into device-0 staging, then copy out and wait
    if (!t->host_out)
      if (bzr_status st = alloc_on(t->dev[0], t->host_out, (size_t)8 * t->n)) return st;
    o_rays = t->host_out;
    o_st = reinterpret_cast<uint32_t *>(t->host_out + (size_t)6 * t->n);
    o_seg = o_st + t->n;
  }
  if (bzr_status st = gather_and_unpack(*t, sl, o_rays, o_st, o_seg)) return st;
  if (host) {
    DeviceGuard g(t->dev[0]);
    hipStream_t gs = t->gstream[0];
    TILED_HIP(hipMemcpyAsync(out_rays, o_rays, (size_t)24 * t->n, hipMemcpyDeviceToHost, gs));
    TILED_HIP(hipMemcpyAsync(out_status, o_st, (size_t)4 * t->n, hipMemcpyDeviceToHost, gs));
    if (out_segments) TILED_HIP(hipMemcpyAsync(out_segments, o_seg, (size_t)4 * t->n, hipMemcpyDeviceToHost, gs));
    TILED_HIP(hipStreamSynchronize(gs));
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
  return BZR_OK;
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
  bzr_status s = bzr_tiled_set_rays(t, rays, flags & BZR_DEVICE_PTRS);
  if (s == BZR_OK) s = bzr_tiled_trace(t, lenses, ri, nlens, out_rays, out_status, out_segments, flags);
  if (s == BZR_OK) s = bzr_tiled_sync(t);
  bzr_tiled_destroy(t);
  return s;
}
