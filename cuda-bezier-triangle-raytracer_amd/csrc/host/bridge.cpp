// bridge.cpp -- the drop-in classes' hot-path methods.  The batch overloads, bzr::traceChain and the
// multi-device calls forward to the GPU through the C ABI (without a HIP device they throw, bzr::check);
// the reference's single-ray methods run the same arithmetic on the host (single_ray.cpp, SURVEY.md
// 8b.1), bit-identical to the batch path, without a launch or PCIe round trip per ray.
//   BezierTriangle::intersect  reference/bezierTriangle.cpp:123-195
//   BezierMesh::intersect      reference/bezierMesh.cpp:206-227
//   BezierLens::refract        reference/bezierLens.cpp:4-34
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <type_traits>

#include "bzr/bzr.hpp"
#include "single_ray.hpp"

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
// The batch calls hand the caller's Ray arrays to the C ABI as they are (BZR_RAYS_AOS: [n][6] records, transposed
// on the device) and RefractionResult arrays as uint32 words.
static_assert(sizeof(Ray) == 6 * sizeof(float) && alignof(Ray) == alignof(float) && std::is_standard_layout<Ray>::value,
              "Ray must be the 24-byte [start xyz, direction xyz] record BZR_RAYS_AOS reads");
static_assert(sizeof(RefractionResult) == sizeof(uint32_t), "RefractionResult must be a uint32 word");
float const *records(Ray const *r) { return reinterpret_cast<float const *>(r); }
float *records(Ray *r) { return reinterpret_cast<float *>(r); }
uint32_t *words(RefractionResult *s) { return reinterpret_cast<uint32_t *>(s); }
uint32_t const *words(RefractionResult const *s) { return reinterpret_cast<uint32_t const *>(s); }
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
  std::lock_guard<std::mutex> hold(c.lock());
  for (std::size_t off = 0; off < n; off += kMaxBatch) {
    const std::size_t m = std::min(kMaxBatch, n - off);
    check(bzr_trace_chain(c.get(), meshes.data(), ri.data(), static_cast<uint32_t>(meshes.size()), records(rays + off),
                          static_cast<uint32_t>(m), records(outRays + off), words(outStatus + off),
                          outSegments ? outSegments + off : nullptr, BZR_HOST_PTRS | BZR_RAYS_AOS));
  }
}

namespace {
// The contexts' locks, taken in id order: two calls over shared contexts cannot deadlock (a repeated context is
// locked once).
std::vector<std::unique_lock<std::mutex>> lock_in_order(std::vector<Context *> order) {
  std::sort(order.begin(), order.end(), [](Context *a, Context *b) { return a->id() < b->id(); });
  order.erase(std::unique(order.begin(), order.end()), order.end());
  std::vector<std::unique_lock<std::mutex>> hold;
  for (Context *c : order) hold.emplace_back(c->lock());
  return hold;
}
}  // namespace

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
  auto hold = lock_in_order(ctxs);
  if (n > UINT32_MAX) throw std::length_error("traceChainTiled: more than 2^32-1 rays in one call");
  check(bzr_trace_tiled(handles.data(), static_cast<uint32_t>(handles.size()), meshes.data(), ri.data(),
                        static_cast<uint32_t>(lenses.size()), records(rays), static_cast<uint32_t>(n), tileRays,
                        records(outRays), words(outStatus), outSegments, BZR_HOST_PTRS | BZR_RAYS_AOS));
}

TiledChain::TiledChain(std::vector<std::vector<Context *>> const &slots, std::vector<BezierLens const *> const &lenses,
                       std::size_t n, uint32_t tileRays, int transport) {
  if (slots.empty() || slots[0].empty()) throw std::invalid_argument("TiledChain: no contexts");
  if (n == 0 || n > UINT32_MAX) throw std::length_error("TiledChain: frame of 1..2^32-1 rays");
  mDevices = slots[0].size();
  mN = n;
  std::vector<bzr_ctx *> handles;
  for (auto const &slot : slots) {
    if (slot.size() != mDevices) throw std::invalid_argument("TiledChain: every slot lists the same devices");
    for (Context *c : slot) {
      handles.push_back(c->get());
      mContexts.push_back(c);
    }
  }
  for (auto const *l : lenses) mRi.push_back(l->getRefractiveIndex());
  for (Context *c : slots[0])  // device d's lens copies (meshes are device-scoped: every slot's context on d uses them)
    for (auto const *l : lenses) mMeshes.push_back(l->getMesh().device(*c));
  check(bzr_tiled_create(handles.data(), static_cast<uint32_t>(mDevices), static_cast<uint32_t>(slots.size()),
                         static_cast<uint32_t>(n), tileRays, transport, &mPlan));
}

TiledChain::~TiledChain() { bzr_tiled_destroy(mPlan); }

int TiledChain::transport() const {
  int32_t t = 0;
  check(bzr_tiled_info(mPlan, &t, nullptr, nullptr));
  return t;
}

void TiledChain::setRays(Ray const *rays) {
  auto hold = lock_in_order(mContexts);
  check(bzr_tiled_set_rays(mPlan, records(rays), BZR_HOST_PTRS | BZR_RAYS_AOS));
}

void TiledChain::setRaysDevice(float const *raysSoaOnDevice0) {
  auto hold = lock_in_order(mContexts);
  check(bzr_tiled_set_rays(mPlan, raysSoaOnDevice0, BZR_DEVICE_PTRS));
}

void TiledChain::trace(float *outRays, uint32_t *outStatus, uint32_t *outSegments, uint32_t flags) {
  auto hold = lock_in_order(mContexts);
  check(bzr_tiled_trace(mPlan, mMeshes.data(), mRi.data(), static_cast<uint32_t>(mRi.size()), outRays, outStatus,
                        outSegments, flags | BZR_DEVICE_PTRS));
}

void TiledChain::trace(Ray *outRays, RefractionResult *outStatus, uint32_t *outSegments, uint32_t flags) {
  auto hold = lock_in_order(mContexts);
  check(bzr_tiled_trace(mPlan, mMeshes.data(), mRi.data(), static_cast<uint32_t>(mRi.size()), records(outRays),
                        words(outStatus), outSegments, (flags & ~uint32_t(BZR_DEVICE_PTRS)) | BZR_RAYS_AOS));
}

uint32_t TiledChain::calibrate(uint32_t flags) {
  uint32_t cap = 0;
  auto hold = lock_in_order(mContexts);
  check(bzr_tiled_calibrate(mPlan, mMeshes.data(), mRi.data(), static_cast<uint32_t>(mRi.size()), flags, &cap));
  return cap;
}

void TiledChain::sync() {
  auto hold = lock_in_order(mContexts);
  check(bzr_tiled_sync(mPlan));
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
  std::lock_guard<std::mutex> hold(c.lock());
  for (std::size_t off = 0; off < n; off += bzr::kMaxBatch) {
    const std::size_t m = std::min(bzr::kMaxBatch, n - off);
    bzr::check(bzr_intersect_records(c.get(), dm, bzr::records(rays + off), static_cast<uint32_t>(m),
                                     reinterpret_cast<bzr_hit_record *>(out + off), patchIndex ? patchIndex + off : nullptr,
                                     BZR_HOST_PTRS | BZR_RAYS_AOS));
  }
}

BezierIntersection BezierMesh::intersect(Ray const &ray) const {
  return bzr::host::meshIntersect(mMesh.data(), mMesh.size(), ray, nullptr);
}

BezierIntersection BezierMesh::intersect(Ray const &ray, uint32_t *patchIndex) const {
  return bzr::host::meshIntersect(mMesh.data(), mMesh.size(), ray, patchIndex);
}

BezierIntersection BezierTriangle::intersect(Ray const &ray, LimitPlaneIntersection limit) const {
  return bzr::host::patchIntersect(*this, ray, limit == LimitPlaneIntersection::cNone);
}

void BezierLens::refract(Ray const *rays, RefractionResult const *expected, std::size_t n, Ray *outRays,
                         RefractionResult *outStatus, bzr::Context *ctx) const {
  bzr::Context &c = ctx ? *ctx : bzr::defaultContext();
  bzr_mesh *dm = mMesh.device(c);
  std::lock_guard<std::mutex> hold(c.lock());
  for (std::size_t off = 0; off < n; off += bzr::kMaxBatch) {
    const std::size_t m = std::min(bzr::kMaxBatch, n - off);
    bzr::check(bzr_refract(c.get(), dm, mRefractiveIndex, bzr::records(rays + off), bzr::words(expected + off), 0u,
                           static_cast<uint32_t>(m), bzr::records(outRays + off), bzr::words(outStatus + off),
                           BZR_HOST_PTRS | BZR_RAYS_AOS));
  }
}

std::pair<Ray, RefractionResult> BezierLens::refract(Ray const &ray, RefractionResult expected) const {
  return bzr::host::lensRefract(&mMesh[0], mMesh.size(), mRefractiveIndex, ray, expected);
}
