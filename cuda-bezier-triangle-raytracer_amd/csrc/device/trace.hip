// trace.hip -- CDNA4 kernels of the hot path + the device half of the C ABI.
//
//   k_intersect     BezierMesh::intersect over a ray batch   (reference/bezierMesh.cpp:206-227)
//   k_patch         BezierTriangle::intersect per (patch, ray) (reference/bezierTriangle.cpp:123-195)
//   k_refract       BezierLens::refract                        (reference/bezierLens.cpp:4-34)
//   k_chain         the refraction chain driver                (reference/test.cpp:376-401)
//
// One ray per lane.  The brute-force patch scan walks the mesh in index order
// with a wave-uniform patch index, so each patch's 64-byte planar record is
// fetched once per wave with scalar loads (s_load, SGPR operands) and shared by
// the 64 rays of the wave; only lanes whose ray passes the planar gate run the
// Newton stage, which loads the full 264-byte record per lane.  See DESIGN.md.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "bzr.h"
#include "patch_math.hpp"

using namespace bzr_dev;

// ------------------------------------------------------------------ errors
namespace {
thread_local std::string t_error;
bzr_status set_error(bzr_status s, const std::string &msg) {
  t_error = msg;
  return s;
}
#define BZR_HIP(call)                                                                                 \
  do {                                                                                                \
    hipError_t e_ = (call);                                                                           \
    if (e_ != hipSuccess) return set_error(BZR_ERR_HIP, std::string(#call ": ") + hipGetErrorString(e_)); \
  } while (0)
}  // namespace

extern "C" const char *bzr_last_error(void) { return t_error.c_str(); }
extern "C" int32_t bzr_abi_version(void) { return BZR_ABI_VERSION; }
// the host half of the library reports its errors through here
extern "C" void bzr_internal_set_error(const char *msg) { t_error = msg ? msg : ""; }

// ------------------------------------------------------------ device mesh
// planar record (64 B) for the scan: n.xyz c | hin hout M00 M01 | M02 M10 M11 M12 | M20 M21 M22 0
struct bzr_mesh {
  int device;
  uint32_t n;
  float4 *planar;  // 4 float4 per patch
  float *full;     // 66 words per patch (bzr_patch)
};

struct bzr_ctx {
  int device;
  hipStream_t own;
  hipStream_t stream;
  // staging buffers for host-pointer calls
  void *scratch = nullptr;
  size_t scratch_bytes = 0;
};

namespace {

constexpr int kBlock = 256;
constexpr uint32_t kMaxLenses = 8;

struct MeshView {
  const float4 *__restrict__ planar;
  const float *__restrict__ full;
  uint32_t n;
  float ri;
};
struct LensSet {
  MeshView lens[kMaxLenses];
  uint32_t count;
};

__device__ __forceinline__ void store_hit(float *__restrict__ hits, uint32_t n, uint32_t i, const Hit &h,
                                          uint32_t patch) {
  hits[i] = h.t;
  hits[(size_t)1 * n + i] = h.point.x;
  hits[(size_t)2 * n + i] = h.point.y;
  hits[(size_t)3 * n + i] = h.point.z;
  hits[(size_t)4 * n + i] = h.cs;
  hits[(size_t)5 * n + i] = h.bary.x;
  hits[(size_t)6 * n + i] = h.bary.y;
  hits[(size_t)7 * n + i] = h.bary.z;
  hits[(size_t)8 * n + i] = h.normal.x;
  hits[(size_t)9 * n + i] = h.normal.y;
  hits[(size_t)10 * n + i] = h.normal.z;
  reinterpret_cast<uint32_t *>(hits)[(size_t)11 * n + i] = h.what;
  reinterpret_cast<uint32_t *>(hits)[(size_t)12 * n + i] = patch;
}

// Planar gate of BezierTriangle::intersect with cThis (reference/bezierTriangle.cpp:124-131),
// evaluated from the 64-byte scan record; same arithmetic as patch_intersect's first lines.
__device__ __forceinline__ bool planar_gate(float4 q0, float4 q1, float4 q2, float4 q3, f3 s, f3 d) {
  f3 n = mk(q0.x, q0.y, q0.z);
  f3 ip;
  float ic, it;
  bool valid = plane_ray(n, q0.w, s, d, ip, ic, it);
  if (!(valid && fabsf(it) > -q1.x && fabsf(it) > q1.y)) return false;
  // row-major copy of M: rows (q1.z q1.w q2.x) (q2.y q2.z q2.w) (q3.x q3.y q3.z)
  float b0 = q1.z * ip.x + (q1.w * ip.y + q2.x * ip.z);
  float b1 = q2.y * ip.x + (q2.z * ip.y + q2.w * ip.z);
  float b2 = q3.x * ip.x + (q3.y * ip.y + q3.z * ip.z);
  return b0 >= 0.0f && b0 <= 1.0f && b1 >= 0.0f && b1 <= 1.0f && b2 >= 0.0f && b2 <= 1.0f;
}

// BezierMesh::intersect: brute force in index order, one follow-side retry, strict-< minimum.
__device__ __forceinline__ Hit mesh_intersect(const MeshView &m, f3 s, f3 d, uint32_t &patch) {
  Hit best;
  best.t = FLT_MAX;
  best.what = kNone;
  best.point = best.bary = best.normal = mk(0.0f, 0.0f, 0.0f);
  best.cs = 0.0f;
  patch = 0xFFFFFFFFu;
  for (uint32_t b = 0; b < m.n; ++b) {
    const float4 *q = m.planar + 4u * b;  // wave-uniform address -> scalar loads
    if (!planar_gate(q[0], q[1], q[2], q[3], s, d)) continue;
    // Newton stage for this lane; a follow-side result retries the named neighbour once with cNone
    uint32_t idx = b;
    bool limitNone = false;
    Hit h;
    for (int pass = 0; pass < 2; ++pass) {
      Patch p = load_patch(m.full + (size_t)rec::kWords * idx);
      h = patch_intersect(p, s, d, limitNone);
      if (pass == 0 && h.what <= kFollow2) {
        idx = __float_as_uint(m.full[(size_t)rec::kWords * idx + rec::kNeigh + h.what]);
        limitNone = true;
        continue;
      }
      break;
    }
    if (h.what == kIntersect && h.t < best.t) {
      best = h;
      patch = idx;
    }
  }
  return best;
}

// BezierLens::refract.  Returns the status; o_s/o_d = refracted ray when status != NONE.
__device__ __forceinline__ uint32_t lens_refract(const MeshView &m, f3 s, f3 d, uint32_t expected, f3 &o_s, f3 &o_d,
                                                 uint32_t &patch) {
  Hit h = mesh_intersect(m, s, d, patch);
  o_s = s;
  o_d = d;
  uint32_t st = BZR_RR_NONE;
  if (h.what == kIntersect) {
    st = h.cs < 0.0f ? BZR_RR_INSIDE : BZR_RR_OUTSIDE;
    o_s = h.point;
    float eta = st == BZR_RR_INSIDE ? div_rn(1.0f, m.ri) : m.ri;
    float s2 = eta * eta * (1.0f - h.cs * h.cs);
    if (s2 < 0.99f) {
      if (s2 > 1e-12f) {
        float sgn = st == BZR_RR_INSIDE ? 1.0f : -1.0f;
        f3 nn = scale(h.normal, sgn);
        float c1 = fabsf(h.cs);
        float c2 = sqrt_rn(1.0f - s2);
        o_d = normalized(add(scale(d, eta), scale(nn, eta * c1 - c2)));
      }
    } else {
      st = BZR_RR_NONE;
    }
  }
  return st == expected ? st : BZR_RR_NONE;
}

__device__ __forceinline__ void load_ray(const float *__restrict__ r, uint32_t n, uint32_t i, f3 &s, f3 &d) {
  s = mk(r[i], r[(size_t)n + i], r[(size_t)2 * n + i]);
  d = mk(r[(size_t)3 * n + i], r[(size_t)4 * n + i], r[(size_t)5 * n + i]);
}
__device__ __forceinline__ void store_ray(float *__restrict__ r, uint32_t n, uint32_t i, f3 s, f3 d) {
  r[i] = s.x;
  r[(size_t)n + i] = s.y;
  r[(size_t)2 * n + i] = s.z;
  r[(size_t)3 * n + i] = d.x;
  r[(size_t)4 * n + i] = d.y;
  r[(size_t)5 * n + i] = d.z;
}

__global__ __launch_bounds__(kBlock) void k_intersect(MeshView m, const float *__restrict__ rays, uint32_t n,
                                                      float *__restrict__ hits) {
  uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  f3 s, d;
  load_ray(rays, n, i, s, d);
  uint32_t patch;
  Hit h = mesh_intersect(m, s, d, patch);
  store_hit(hits, n, i, h, patch);
}

__global__ __launch_bounds__(kBlock) void k_patch(MeshView m, const uint32_t *__restrict__ idx,
                                                  const uint32_t *__restrict__ limit, const float *__restrict__ rays,
                                                  uint32_t n, float *__restrict__ hits) {
  uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  f3 s, d;
  load_ray(rays, n, i, s, d);
  uint32_t pi = idx[i];
  Hit h;
  if (pi < m.n) {
    Patch p = load_patch(m.full + (size_t)rec::kWords * pi);
    h = patch_intersect(p, s, d, limit[i] != 0u);
  } else {
    h.t = 0.0f;
    h.point = h.bary = h.normal = mk(0.0f, 0.0f, 0.0f);
    h.cs = 0.0f;
    h.what = kNone;
  }
  store_hit(hits, n, i, h, pi);
}

__global__ __launch_bounds__(kBlock) void k_refract(MeshView m, const float *__restrict__ rays,
                                                    const uint32_t *__restrict__ expected, uint32_t expected_all,
                                                    uint32_t n, float *__restrict__ out_rays,
                                                    uint32_t *__restrict__ out_status) {
  uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  f3 s, d, os, od;
  load_ray(rays, n, i, s, d);
  uint32_t patch;
  uint32_t st = lens_refract(m, s, d, expected ? expected[i] : expected_all, os, od, patch);
  if (st == BZR_RR_NONE) {
    os = s;
    od = d;
  }
  store_ray(out_rays, n, i, os, od);
  out_status[i] = st;
}

__global__ __launch_bounds__(kBlock) void k_chain(LensSet lenses, const float *__restrict__ rays, uint32_t n,
                                                  float *__restrict__ out_rays, uint32_t *__restrict__ out_status,
                                                  uint32_t *__restrict__ out_segments) {
  uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  f3 s, d;
  load_ray(rays, n, i, s, d);
  uint32_t st = BZR_RR_NONE, seg = 0;
  bool alive = true;
  for (uint32_t l = 0; l < lenses.count && alive; ++l) {
    for (uint32_t j = 0; j < 2u && alive; ++j) {
      f3 os, od;
      uint32_t patch;
      ++seg;
      st = lens_refract(lenses.lens[l], s, d, j == 0 ? BZR_RR_INSIDE : BZR_RR_OUTSIDE, os, od, patch);
      if (st == BZR_RR_NONE) {
        alive = false;
      } else {
        s = os;
        d = od;
      }
    }
  }
  store_ray(out_rays, n, i, s, d);
  out_status[i] = st;
  if (out_segments) out_segments[i] = seg;
}

// ------------------------------------------------------------ host helpers
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

MeshView view_of(const bzr_mesh *m, float ri = 1.0f) { return MeshView{m->planar, m->full, m->n, ri}; }
unsigned grid_for(uint32_t n) { return (n + kBlock - 1) / kBlock; }

// Host-pointer calls stage through one device allocation owned by the context.
bzr_status ensure_scratch(bzr_ctx *ctx, size_t bytes) {
  if (ctx->scratch_bytes >= bytes) return BZR_OK;
  if (ctx->scratch) BZR_HIP(hipFree(ctx->scratch));
  ctx->scratch = nullptr;
  ctx->scratch_bytes = 0;
  BZR_HIP(hipMalloc(&ctx->scratch, bytes));
  ctx->scratch_bytes = bytes;
  return BZR_OK;
}

struct Staging {  // carves device buffers out of the scratch area
  char *base;
  size_t off = 0;
  template <typename T>
  T *take(size_t count) {
    T *p = reinterpret_cast<T *>(base + off);
    off += (count * sizeof(T) + 255) & ~size_t(255);
    return p;
  }
};
size_t round256(size_t b) { return (b + 255) & ~size_t(255); }

bzr_status check_ctx_mesh(bzr_ctx *ctx, const bzr_mesh *mesh) {
  if (!ctx) return set_error(BZR_ERR_INVALID_ARGUMENT, "null context");
  if (!mesh) return set_error(BZR_ERR_INVALID_ARGUMENT, "null mesh");
  if (mesh->device != ctx->device) return set_error(BZR_ERR_INVALID_ARGUMENT, "mesh lives on another device");
  return BZR_OK;
}

}  // namespace

// ------------------------------------------------------------------- C ABI
extern "C" bzr_status bzr_device_count(int32_t *count) {
  if (!count) return set_error(BZR_ERR_INVALID_ARGUMENT, "null count");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) c = 0;
  *count = c;
  return BZR_OK;
}

extern "C" bzr_status bzr_ctx_create(int32_t device, bzr_ctx **out) {
  if (!out) return set_error(BZR_ERR_INVALID_ARGUMENT, "null out");
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
    return set_error(BZR_ERR_NO_DEVICE, "no HIP device visible: libbzr has no CPU path");
  if (device < 0 || device >= count) return set_error(BZR_ERR_INVALID_ARGUMENT, "device index out of range");
  DeviceGuard g(device);
  bzr_ctx *c = new (std::nothrow) bzr_ctx();
  if (!c) return set_error(BZR_ERR_OUT_OF_MEMORY, "context allocation");
  c->device = device;
  hipError_t e = hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    return set_error(BZR_ERR_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(e));
  }
  c->stream = c->own;
  *out = c;
  return BZR_OK;
}

extern "C" bzr_status bzr_ctx_destroy(bzr_ctx *ctx) {
  if (!ctx) return BZR_OK;
  DeviceGuard g(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  (void)hipStreamSynchronize(ctx->own);
  if (ctx->scratch) (void)hipFree(ctx->scratch);
  (void)hipStreamDestroy(ctx->own);
  delete ctx;
  return BZR_OK;
}

extern "C" bzr_status bzr_ctx_set_stream(bzr_ctx *ctx, void *stream) {
  if (!ctx) return set_error(BZR_ERR_INVALID_ARGUMENT, "null context");
  ctx->stream = reinterpret_cast<hipStream_t>(stream);
  return BZR_OK;
}

extern "C" bzr_status bzr_ctx_use_own_stream(bzr_ctx *ctx) {
  if (!ctx) return set_error(BZR_ERR_INVALID_ARGUMENT, "null context");
  ctx->stream = ctx->own;
  return BZR_OK;
}

extern "C" bzr_status bzr_ctx_get_stream(bzr_ctx *ctx, void **stream) {
  if (!ctx || !stream) return set_error(BZR_ERR_INVALID_ARGUMENT, "null argument");
  *stream = reinterpret_cast<void *>(ctx->stream);
  return BZR_OK;
}

extern "C" bzr_status bzr_sync(bzr_ctx *ctx) {
  if (!ctx) return set_error(BZR_ERR_INVALID_ARGUMENT, "null context");
  DeviceGuard g(ctx->device);
  BZR_HIP(hipStreamSynchronize(ctx->stream));
  return BZR_OK;
}

extern "C" bzr_status bzr_mesh_create(bzr_ctx *ctx, const void *patches, uint32_t n, uint32_t stride, bzr_mesh **out) {
  if (!ctx || !out || (!patches && n)) return set_error(BZR_ERR_INVALID_ARGUMENT, "null argument");
  if (stride < sizeof(bzr_patch)) return set_error(BZR_ERR_INVALID_ARGUMENT, "stride smaller than bzr_patch");
  *out = nullptr;
  DeviceGuard g(ctx->device);
  std::vector<float> full((size_t)n * rec::kWords);
  std::vector<float4> planar((size_t)n * 4);
  const char *src = static_cast<const char *>(patches);
  for (uint32_t i = 0; i < n; ++i) {
    float *r = &full[(size_t)i * rec::kWords];
    std::memcpy(r, src + (size_t)i * stride, sizeof(bzr_patch));
    const float *m = r + rec::kMinv;  // col-major: M(i,j) = m[j*3+i]
    planar[4 * i + 0] = make_float4(r[0], r[1], r[2], r[3]);
    planar[4 * i + 1] = make_float4(r[rec::kHin], r[rec::kHout], m[0], m[3]);
    planar[4 * i + 2] = make_float4(m[6], m[1], m[4], m[7]);
    planar[4 * i + 3] = make_float4(m[2], m[5], m[8], 0.0f);
  }
  bzr_mesh *mesh = new (std::nothrow) bzr_mesh();
  if (!mesh) return set_error(BZR_ERR_OUT_OF_MEMORY, "mesh allocation");
  mesh->device = ctx->device;
  mesh->n = n;
  size_t pb = planar.size() * sizeof(float4), fb = full.size() * sizeof(float);
  hipError_t e = hipMalloc(&mesh->planar, pb ? pb : 16);
  if (e == hipSuccess) e = hipMalloc(&mesh->full, fb ? fb : 16);
  if (e == hipSuccess && pb) e = hipMemcpyAsync(mesh->planar, planar.data(), pb, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess && fb) e = hipMemcpyAsync(mesh->full, full.data(), fb, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) {
    (void)hipFree(mesh->planar);
    (void)hipFree(mesh->full);
    delete mesh;
    return set_error(BZR_ERR_HIP, std::string("mesh upload: ") + hipGetErrorString(e));
  }
  *out = mesh;
  return BZR_OK;
}

extern "C" bzr_status bzr_mesh_destroy(bzr_mesh *mesh) {
  if (!mesh) return BZR_OK;
  DeviceGuard g(mesh->device);
  (void)hipDeviceSynchronize();
  (void)hipFree(mesh->planar);
  (void)hipFree(mesh->full);
  delete mesh;
  return BZR_OK;
}

extern "C" bzr_status bzr_mesh_size(const bzr_mesh *mesh, uint32_t *n) {
  if (!mesh || !n) return set_error(BZR_ERR_INVALID_ARGUMENT, "null argument");
  *n = mesh->n;
  return BZR_OK;
}

extern "C" bzr_status bzr_intersect(bzr_ctx *ctx, const bzr_mesh *mesh, const float *rays, uint32_t n, float *hits,
                                    uint32_t flags) {
  if (bzr_status s = check_ctx_mesh(ctx, mesh)) return s;
  if (n == 0) return BZR_OK;
  if (!rays || !hits) return set_error(BZR_ERR_INVALID_ARGUMENT, "null buffer");
  DeviceGuard g(ctx->device);
  const float *d_rays = rays;
  float *d_hits = hits;
  bool host = !(flags & BZR_DEVICE_PTRS);
  if (host) {
    size_t rb = (size_t)n * 6 * sizeof(float), hb = (size_t)n * 13 * sizeof(float);
    if (bzr_status s = ensure_scratch(ctx, round256(rb) + round256(hb))) return s;
    Staging st{static_cast<char *>(ctx->scratch)};
    float *r = st.take<float>((size_t)n * 6);
    d_hits = st.take<float>((size_t)n * 13);
    BZR_HIP(hipMemcpyAsync(r, rays, rb, hipMemcpyHostToDevice, ctx->stream));
    d_rays = r;
  }
  hipLaunchKernelGGL(k_intersect, dim3(grid_for(n)), dim3(kBlock), 0, ctx->stream, view_of(mesh), d_rays, n, d_hits);
  BZR_HIP(hipGetLastError());
  if (host) {
    BZR_HIP(hipMemcpyAsync(hits, d_hits, (size_t)n * 13 * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    BZR_HIP(hipStreamSynchronize(ctx->stream));
  }
  return BZR_OK;
}

extern "C" bzr_status bzr_patch_intersect(bzr_ctx *ctx, const bzr_mesh *mesh, const uint32_t *idx, const uint32_t *limit,
                                          const float *rays, uint32_t n, float *hits, uint32_t flags) {
  if (bzr_status s = check_ctx_mesh(ctx, mesh)) return s;
  if (n == 0) return BZR_OK;
  if (!idx || !limit || !rays || !hits) return set_error(BZR_ERR_INVALID_ARGUMENT, "null buffer");
  DeviceGuard g(ctx->device);
  const uint32_t *d_idx = idx, *d_lim = limit;
  const float *d_rays = rays;
  float *d_hits = hits;
  bool host = !(flags & BZR_DEVICE_PTRS);
  if (host) {
    size_t ib = (size_t)n * 4, rb = (size_t)n * 24, hb = (size_t)n * 52;
    if (bzr_status s = ensure_scratch(ctx, 2 * round256(ib) + round256(rb) + round256(hb))) return s;
    Staging st{static_cast<char *>(ctx->scratch)};
    uint32_t *a = st.take<uint32_t>(n), *b = st.take<uint32_t>(n);
    float *r = st.take<float>((size_t)n * 6);
    d_hits = st.take<float>((size_t)n * 13);
    BZR_HIP(hipMemcpyAsync(a, idx, ib, hipMemcpyHostToDevice, ctx->stream));
    BZR_HIP(hipMemcpyAsync(b, limit, ib, hipMemcpyHostToDevice, ctx->stream));
    BZR_HIP(hipMemcpyAsync(r, rays, rb, hipMemcpyHostToDevice, ctx->stream));
    d_idx = a;
    d_lim = b;
    d_rays = r;
  }
  hipLaunchKernelGGL(k_patch, dim3(grid_for(n)), dim3(kBlock), 0, ctx->stream, view_of(mesh), d_idx, d_lim, d_rays, n,
                     d_hits);
  BZR_HIP(hipGetLastError());
  if (host) {
    BZR_HIP(hipMemcpyAsync(hits, d_hits, (size_t)n * 52, hipMemcpyDeviceToHost, ctx->stream));
    BZR_HIP(hipStreamSynchronize(ctx->stream));
  }
  return BZR_OK;
}

extern "C" bzr_status bzr_refract(bzr_ctx *ctx, const bzr_mesh *mesh, float ri, const float *rays, const uint32_t *expected,
                                  uint32_t expected_all, uint32_t n, float *out_rays, uint32_t *out_status,
                                  uint32_t flags) {
  if (bzr_status s = check_ctx_mesh(ctx, mesh)) return s;
  if (n == 0) return BZR_OK;
  if (!rays || !out_rays || !out_status) return set_error(BZR_ERR_INVALID_ARGUMENT, "null buffer");
  DeviceGuard g(ctx->device);
  const float *d_rays = rays;
  const uint32_t *d_exp = expected;
  float *d_out = out_rays;
  uint32_t *d_st = out_status;
  bool host = !(flags & BZR_DEVICE_PTRS);
  if (host) {
    size_t rb = (size_t)n * 24, ib = (size_t)n * 4;
    if (bzr_status s = ensure_scratch(ctx, 2 * round256(rb) + 2 * round256(ib))) return s;
    Staging st{static_cast<char *>(ctx->scratch)};
    float *r = st.take<float>((size_t)n * 6);
    uint32_t *e = st.take<uint32_t>(n);
    d_out = st.take<float>((size_t)n * 6);
    d_st = st.take<uint32_t>(n);
    BZR_HIP(hipMemcpyAsync(r, rays, rb, hipMemcpyHostToDevice, ctx->stream));
    if (expected) BZR_HIP(hipMemcpyAsync(e, expected, ib, hipMemcpyHostToDevice, ctx->stream));
    d_rays = r;
    d_exp = expected ? e : nullptr;
  }
  hipLaunchKernelGGL(k_refract, dim3(grid_for(n)), dim3(kBlock), 0, ctx->stream, view_of(mesh, ri), d_rays, d_exp,
                     expected_all, n, d_out, d_st);
  BZR_HIP(hipGetLastError());
  if (host) {
    BZR_HIP(hipMemcpyAsync(out_rays, d_out, (size_t)n * 24, hipMemcpyDeviceToHost, ctx->stream));
    BZR_HIP(hipMemcpyAsync(out_status, d_st, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream));
    BZR_HIP(hipStreamSynchronize(ctx->stream));
  }
  return BZR_OK;
}

extern "C" bzr_status bzr_trace_chain(bzr_ctx *ctx, const bzr_mesh *const *lenses, const float *ri, uint32_t nlens,
                                      const float *rays, uint32_t n, float *out_rays, uint32_t *out_status,
                                      uint32_t *out_segments, uint32_t flags) {
  if (!ctx) return set_error(BZR_ERR_INVALID_ARGUMENT, "null context");
  if (nlens == 0 || nlens > kMaxLenses) return set_error(BZR_ERR_INVALID_ARGUMENT, "nlens must be 1..8");
  if (!lenses || !ri) return set_error(BZR_ERR_INVALID_ARGUMENT, "null lens list");
  LensSet set{};
  set.count = nlens;
  for (uint32_t l = 0; l < nlens; ++l) {
    if (bzr_status s = check_ctx_mesh(ctx, lenses[l])) return s;
    set.lens[l] = view_of(lenses[l], ri[l]);
  }
  if (n == 0) return BZR_OK;
  if (!rays || !out_rays || !out_status) return set_error(BZR_ERR_INVALID_ARGUMENT, "null buffer");
  DeviceGuard g(ctx->device);
  const float *d_rays = rays;
  float *d_out = out_rays;
  uint32_t *d_st = out_status, *d_seg = out_segments;
  bool host = !(flags & BZR_DEVICE_PTRS);
  if (host) {
    size_t rb = (size_t)n * 24, ib = (size_t)n * 4;
    if (bzr_status s = ensure_scratch(ctx, 2 * round256(rb) + 2 * round256(ib))) return s;
    Staging st{static_cast<char *>(ctx->scratch)};
    float *r = st.take<float>((size_t)n * 6);
    d_out = st.take<float>((size_t)n * 6);
    d_st = st.take<uint32_t>(n);
    d_seg = out_segments ? st.take<uint32_t>(n) : nullptr;
    BZR_HIP(hipMemcpyAsync(r, rays, rb, hipMemcpyHostToDevice, ctx->stream));
    d_rays = r;
  }
  hipLaunchKernelGGL(k_chain, dim3(grid_for(n)), dim3(kBlock), 0, ctx->stream, set, d_rays, n, d_out, d_st, d_seg);
  BZR_HIP(hipGetLastError());
  if (host) {
    BZR_HIP(hipMemcpyAsync(out_rays, d_out, (size_t)n * 24, hipMemcpyDeviceToHost, ctx->stream));
    BZR_HIP(hipMemcpyAsync(out_status, d_st, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream));
    if (out_segments)
      BZR_HIP(hipMemcpyAsync(out_segments, d_seg, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream));
    BZR_HIP(hipStreamSynchronize(ctx->stream));
  }
  return BZR_OK;
}
