// bridge.cpp -- the drop-in classes' hot-path methods, forwarded to the GPU
// through the C ABI.  No CPU implementation of intersect/refract exists in the
// product: without a HIP device these calls throw (bzr::check).
//   BezierTriangle::intersect  reference/bezierTriangle.cpp:123-195
//   BezierMesh::intersect      reference/bezierMesh.cpp:206-227
//   BezierLens::refract        reference/bezierLens.cpp:4-34
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "bzr/bzr.hpp"

namespace bzr {

void check(bzr_status s) {
  if (s != BZR_OK) throw std::runtime_error(std::string("libbzr: ") + bzr_last_error());
}

namespace {
std::atomic<uint64_t> g_next_context_id{1};
std::mutex g_device_cache;  // guards every BezierMesh::mDevices (meshes are shared read-only across threads)
// The C ABI counts rays in uint32_t: larger host batches are issued in slices of at most this many rays.
constexpr std::size_t kMaxBatch = std::size_t(1) << 30;
}  // namespace

Context::Context(int device) : mId(g_next_context_id.fetch_add(1)) { check(bzr_ctx_create(device, &mCtx)); }
Context::~Context() { bzr_ctx_destroy(mCtx); }
void Context::sync() const { check(bzr_sync(mCtx)); }

Context &defaultContext() {
  // device from BZR_DEVICE (default 0), created on first use
  static std::once_flag once;
  static std::unique_ptr<Context> ctx;
  std::call_once(once, [] {
    char const *env = std::getenv("BZR_DEVICE");
    ctx = std::make_unique<Context>(env ? std::atoi(env) : 0);
  });
  return *ctx;
}

struct DeviceMesh {
  uint64_t owner = 0;  // Context::id()
  bzr_mesh *mesh = nullptr;
  ~DeviceMesh() { bzr_mesh_destroy(mesh); }
};

namespace {
std::vector<float> raysToSoa(Ray const *rays, std::size_t n) {
  std::vector<float> soa(6 * n);
  for (std::size_t i = 0; i < n; ++i) {
    for (int k = 0; k < 3; ++k) {
      soa[k * n + i] = rays[i].mStart(k);
      soa[(3 + k) * n + i] = rays[i].mDirection(k);
    }
  }
  return soa;
}
Ray soaToRay(std::vector<float> const &soa, std::size_t n, std::size_t i) {
  Ray r;
  for (int k = 0; k < 3; ++k) {
    r.mStart(k) = soa[k * n + i];
    r.mDirection(k) = soa[(3 + k) * n + i];
  }
  return r;
}
BezierIntersection hitFromSoa(std::vector<float> const &h, std::size_t n, std::size_t i) {
  BezierIntersection b;
  b.mIntersection.mDistance = h[i];
  b.mIntersection.mPoint = Vertex(h[n + i], h[2 * n + i], h[3 * n + i]);
  b.mIntersection.mCosIncidence = h[4 * n + i];
  b.mBarycentric = Vertex(h[5 * n + i], h[6 * n + i], h[7 * n + i]);
  b.mNormal = Vector(h[8 * n + i], h[9 * n + i], h[10 * n + i]);
  uint32_t what;
  std::memcpy(&what, &h[11 * n + i], 4);
  b.mWhat = static_cast<BezierIntersection::What>(what);
  b.mIntersection.mValid = what == BZR_WHAT_INTERSECT;
  return b;
}
}  // namespace

void traceChain(std::vector<BezierLens const *> const &lenses, Ray const *rays, std::size_t n, Ray *outRays,
                RefractionResult *outStatus, uint32_t *outSegments, Context *ctx) {
  Context &c = ctx ? *ctx : defaultContext();
  std::vector<bzr_mesh const *> meshes;
  std::vector<float> ri;
  for (auto const *l : lenses) {
    meshes.push_back(l->getMesh().device(c));
    ri.push_back(l->getRefractiveIndex());
  }
  for (std::size_t off = 0; off < n; off += kMaxBatch) {
    const std::size_t m = std::min(kMaxBatch, n - off);
    std::vector<float> in = raysToSoa(rays + off, m), out(6 * m);
    std::vector<uint32_t> st(m);
    check(bzr_trace_chain(c.get(), meshes.data(), ri.data(), static_cast<uint32_t>(meshes.size()), in.data(),
                          static_cast<uint32_t>(m), out.data(), st.data(), outSegments ? outSegments + off : nullptr,
                          BZR_HOST_PTRS));
    for (std::size_t i = 0; i < m; ++i) {
      outRays[off + i] = soaToRay(out, m, i);
      outStatus[off + i] = static_cast<RefractionResult>(st[i]);
    }
  }
}

void traceChainTiled(std::vector<Context *> const &ctxs, std::vector<BezierLens const *> const &lenses,
                     Ray const *rays, std::size_t n, Ray *outRays, RefractionResult *outStatus,
                     uint32_t *outSegments, uint32_t tileRays) {
  std::vector<bzr_ctx *> handles;
  std::vector<bzr_mesh const *> meshes;  // [context][lens]
  std::vector<float> ri;
  for (auto const *l : lenses) ri.push_back(l->getRefractiveIndex());
  for (Context *c : ctxs) {
    handles.push_back(c->get());
    for (auto const *l : lenses) meshes.push_back(l->getMesh().device(*c));
  }
  if (n > UINT32_MAX) throw std::length_error("traceChainTiled: more than 2^32-1 rays in one call");
  std::vector<float> in = raysToSoa(rays, n), out(6 * n);
  std::vector<uint32_t> st(n);
  check(bzr_trace_tiled(handles.data(), static_cast<uint32_t>(handles.size()), meshes.data(), ri.data(),
                        static_cast<uint32_t>(lenses.size()), in.data(), static_cast<uint32_t>(n), tileRays, out.data(),
                        st.data(), outSegments, BZR_HOST_PTRS));
  for (std::size_t i = 0; i < n; ++i) {
    outRays[i] = soaToRay(out, n, i);
    outStatus[i] = static_cast<RefractionResult>(st[i]);
  }
}

}  // namespace bzr

bzr_mesh *BezierMesh::device(bzr::Context &ctx) const {
  std::lock_guard<std::mutex> lock(bzr::g_device_cache);
  for (auto const &dm : mDevices)
    if (dm->owner == ctx.id()) return dm->mesh;
  auto dm = std::make_shared<bzr::DeviceMesh>();
  dm->owner = ctx.id();
  bzr::check(bzr_mesh_create(ctx.get(), mMesh.empty() ? nullptr : mMesh.data(), static_cast<uint32_t>(mMesh.size()),
                             sizeof(BezierTriangle), &dm->mesh));
  mDevices.push_back(dm);
  return dm->mesh;
}

void BezierMesh::intersect(Ray const *rays, std::size_t n, BezierIntersection *out, uint32_t *patchIndex,
                           bzr::Context *ctx) const {
  bzr::Context &c = ctx ? *ctx : bzr::defaultContext();
  bzr_mesh *dm = device(c);
  for (std::size_t off = 0; off < n; off += bzr::kMaxBatch) {
    const std::size_t m = std::min(bzr::kMaxBatch, n - off);
    std::vector<float> in = bzr::raysToSoa(rays + off, m), hits(13 * m);
    bzr::check(bzr_intersect(c.get(), dm, in.data(), static_cast<uint32_t>(m), hits.data(), BZR_HOST_PTRS));
    for (std::size_t i = 0; i < m; ++i) {
      out[off + i] = bzr::hitFromSoa(hits, m, i);
      if (patchIndex) std::memcpy(&patchIndex[off + i], &hits[12 * m + i], 4);
    }
  }
}

BezierIntersection BezierMesh::intersect(Ray const &ray) const {
  BezierIntersection r;
  intersect(&ray, 1, &r);
  return r;
}

BezierIntersection BezierTriangle::intersect(Ray const &ray, LimitPlaneIntersection limit) const {
  bzr::Context &c = bzr::defaultContext();
  bzr_mesh *m = nullptr;
  bzr::check(bzr_mesh_create(c.get(), this, 1, sizeof(BezierTriangle), &m));
  std::vector<float> in = bzr::raysToSoa(&ray, 1), hits(13);
  uint32_t idx = 0, lim = static_cast<uint32_t>(limit);
  bzr_status s = bzr_patch_intersect(c.get(), m, &idx, &lim, in.data(), 1, hits.data(), BZR_HOST_PTRS);
  bzr_mesh_destroy(m);
  bzr::check(s);
  return bzr::hitFromSoa(hits, 1, 0);
}

void BezierLens::refract(Ray const *rays, RefractionResult const *expected, std::size_t n, Ray *outRays,
                         RefractionResult *outStatus, bzr::Context *ctx) const {
  bzr::Context &c = ctx ? *ctx : bzr::defaultContext();
  bzr_mesh *dm = mMesh.device(c);
  for (std::size_t off = 0; off < n; off += bzr::kMaxBatch) {
    const std::size_t m = std::min(bzr::kMaxBatch, n - off);
    std::vector<float> in = bzr::raysToSoa(rays + off, m), out(6 * m);
    std::vector<uint32_t> exp(m), st(m);
    for (std::size_t i = 0; i < m; ++i) exp[i] = static_cast<uint32_t>(expected[off + i]);
    bzr::check(bzr_refract(c.get(), dm, mRefractiveIndex, in.data(), exp.data(), 0u, static_cast<uint32_t>(m),
                           out.data(), st.data(), BZR_HOST_PTRS));
    for (std::size_t i = 0; i < m; ++i) {
      outRays[off + i] = bzr::soaToRay(out, m, i);
      outStatus[off + i] = static_cast<RefractionResult>(st[i]);
    }
  }
}

std::pair<Ray, RefractionResult> BezierLens::refract(Ray const &ray, RefractionResult expected) const {
  Ray out;
  RefractionResult st;
  refract(&ray, &expected, 1, &out, &st);
  return {out, st};
}
