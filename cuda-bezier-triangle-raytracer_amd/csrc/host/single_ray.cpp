// single_ray.cpp -- the drop-in's single-ray methods on the host ("the single-ray
// intersect/refract stay CPU (bit-faithful)").
//
// The reference's own callers trace one ray per call (reference/test.cpp:268,281,380).  Through the GPU
// each such call is a launch, two PCIe copies and a sync; here it is the product's own arithmetic text
// (csrc/device/patch_math_body.inc, the `exact::` namespace the kernels run) compiled for the host with
// -ffp-contract=off: IEEE binary32, Eigen 3.3's operation order, correctly rounded division and square
// root -- the same bits as the GPU batch path (tests/cpp/dropin_test.cpp checks every field).  This is not
// a fallback for the batch path: the batch overloads, bzr::traceChain and the C ABI run on the GPU only
// and fail without a device.
//   patchIntersect  BezierTriangle::intersect   reference/bezierTriangle.cpp:123-195
//   meshIntersect   BezierMesh::intersect       reference/bezierMesh.cpp:206-227 (brute force, index order)
//   lensRefract     BezierLens::refract         reference/bezierLens.cpp:4-34
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <math.h>

#include "single_ray.hpp"

// patch_math_body.inc is device code text; on the host its qualifiers are plain inline functions.
#define __device__
#define __forceinline__ inline
#define BZR_NEWTON_ITERS 4
#define BZR_NEWTON_UNROLL 0

namespace bzr_host {

struct f3 {
  float x, y, z;
};
inline f3 mk(float x, float y, float z) { return f3{x, y, z}; }
constexpr uint32_t kFollow2 = 2u, kNone = 3u, kIntersect = 4u;

struct Hit {
  float t;
  f3 point;
  float cs;
  f3 bary;
  f3 normal;
  uint32_t what;
};

// The 66-word record (include/bzr.h bzr_patch) read in place, as the device's PatchView does.
struct PatchView {
  const float *r;
  f3 v3(int o) const { return mk(r[o], r[o + 1], r[o + 2]); }
  f3 n() const { return v3(0); }
  float c() const { return r[3]; }
  f3 dn(int k) const { return v3(4 + 4 * k); }
  float dc(int k) const { return r[4 + 4 * k + 3]; }
  f3 cp(int k) const { return v3(19 + 3 * k); }
  float m(int k) const { return r[49 + k]; }
  float hin() const { return r[58]; }
  float hout() const { return r[59]; }
  f3 da() const { return v3(60); }
  f3 db() const { return v3(63); }
};
constexpr int kNeigh = 16, kWords = 66;

namespace exact {
inline float div_rn(float a, float b) { return a / b; }
inline float sqrt_rn(float a) { return std::sqrt(a); }
inline bool sqrt_above_hundredth(float z) { return sqrt_rn(z) > 0.01f; }  // norm(perp) > 0.01f
inline f3 unit_or_self(f3 a, float z) {  // Eigen normalized(): a / sqrt(z) when z > 0
  if (!(z > 0.0f)) return a;
  const float s = sqrt_rn(z);
  return mk(div_rn(a.x, s), div_rn(a.y, s), div_rn(a.z, s));
}
inline void div_heights(float hin, float hout, float ic, float &din, float &dout) {
  din = div_rn(hin, ic);
  dout = div_rn(hout, ic);
}
#include "../device/patch_math_body.inc"
}  // namespace exact
using namespace exact;

// patch_math.hpp patch_intersect (ungated): the planar gate (reference/bezierTriangle.cpp:124-131), then the
// bracket, Newton steps and classification.
Hit patch_intersect(const PatchView &p, f3 s, f3 d, bool limitNone) {
  Hit h;
  h.t = 0.0f;
  h.point = mk(0.0f, 0.0f, 0.0f);
  h.cs = 0.0f;
  h.bary = h.point;
  h.normal = h.point;
  h.what = kNone;
  f3 ip;
  float ic, it;
  const bool valid = plane_ray(p.n(), p.c(), s, d, ip, ic, it);
  if (!(valid && fabsf(it) > -p.hin() && fabsf(it) > p.hout())) return h;
  const f3 b0 = matvec(p, ip);
  if (!(limitNone || (b0.x >= 0.0f && b0.x <= 1.0f && b0.y >= 0.0f && b0.y <= 1.0f && b0.z >= 0.0f && b0.z <= 1.0f)))
    return h;
  return newton_tail(p, s, d, ic, it);
}

Hit no_hit() {
  Hit h;
  h.t = FLT_MAX;
  h.what = kNone;
  h.point = h.bary = h.normal = mk(0.0f, 0.0f, 0.0f);
  h.cs = 0.0f;
  return h;
}

// BezierMesh::intersect: every patch in index order with cThis; a follow-side result retries the named
// neighbour once with cNone (reference/bezierMesh.cpp:212-216); the first smallest t wins (strict <).
Hit mesh_intersect(const float *records, std::size_t n, f3 s, f3 d, uint32_t &patch) {
  Hit best = no_hit();
  patch = 0xFFFFFFFFu;
  for (std::size_t b = 0; b < n; ++b) {
    const float *rec = records + kWords * b;
    Hit h = patch_intersect(PatchView{rec}, s, d, false);
    uint32_t src = static_cast<uint32_t>(b);
    if (h.what <= kFollow2) {
      uint32_t nb;
      std::memcpy(&nb, rec + kNeigh + h.what, 4);
      h = patch_intersect(PatchView{records + kWords * static_cast<std::size_t>(nb)}, s, d, true);
      src = nb;
    }
    if (h.what == kIntersect && h.t < best.t) {
      best = h;
      patch = src;
    }
  }
  return best;
}

// BezierLens::refract after the intersection (trace.hip refract_hit, reference/bezierLens.cpp:8-32).
uint32_t refract_hit(const Hit &h, float ri, f3 s, f3 d, uint32_t expected, f3 &o_s, f3 &o_d) {
  o_s = s;
  o_d = d;
  uint32_t st = BZR_RR_NONE;
  if (h.what == kIntersect) {
    st = h.cs < 0.0f ? uint32_t(BZR_RR_INSIDE) : uint32_t(BZR_RR_OUTSIDE);
    o_s = h.point;
    const float eta = st == BZR_RR_INSIDE ? div_rn(1.0f, ri) : ri;
    const float s2 = eta * eta * (1.0f - h.cs * h.cs);
    if (s2 < 0.99f) {
      if (s2 > 1e-12f) {
        const float sgn = st == BZR_RR_INSIDE ? 1.0f : -1.0f;
        const f3 nn = scale(h.normal, sgn);
        const float c1 = fabsf(h.cs);
        const float c2 = sqrt_rn(1.0f - s2);
        o_d = normalized(add(scale(d, eta), scale(nn, eta * c1 - c2)));
      }
    } else {
      st = BZR_RR_NONE;
    }
  }
  return st == expected ? st : uint32_t(BZR_RR_NONE);
}

f3 v3(Vector const &v) { return mk(v(0), v(1), v(2)); }
Vector vec(f3 v) { return Vector(v.x, v.y, v.z); }

BezierIntersection to_reference(const Hit &h) {
  BezierIntersection b;
  b.mIntersection.mDistance = h.t;
  b.mIntersection.mPoint = vec(h.point);
  b.mIntersection.mCosIncidence = h.cs;
  b.mIntersection.mValid = h.what == kIntersect;
  b.mBarycentric = vec(h.bary);
  b.mNormal = vec(h.normal);
  b.mWhat = static_cast<BezierIntersection::What>(h.what);
  return b;
}

}  // namespace bzr_host

namespace bzr {
namespace host {

static_assert(sizeof(BezierTriangle) == bzr_host::kWords * 4, "66-word records");

BezierIntersection patchIntersect(BezierTriangle const &patch, Ray const &ray, bool limitNone) {
  using namespace bzr_host;
  return to_reference(patch_intersect(PatchView{reinterpret_cast<const float *>(&patch)}, v3(ray.mStart),
                                      v3(ray.mDirection), limitNone));
}

BezierIntersection meshIntersect(BezierTriangle const *patches, std::size_t n, Ray const &ray, uint32_t *patch) {
  using namespace bzr_host;
  uint32_t p;
  const Hit h = mesh_intersect(reinterpret_cast<const float *>(patches), n, v3(ray.mStart), v3(ray.mDirection), p);
  if (patch) *patch = p;
  return to_reference(h);
}

std::pair<Ray, RefractionResult> lensRefract(BezierTriangle const *patches, std::size_t n, float ri, Ray const &ray,
                                             RefractionResult expected) {
  using namespace bzr_host;
  const f3 s = v3(ray.mStart), d = v3(ray.mDirection);
  uint32_t p;
  const Hit h = mesh_intersect(reinterpret_cast<const float *>(patches), n, s, d, p);
  f3 os, od;
  const uint32_t st = refract_hit(h, ri, s, d, static_cast<uint32_t>(expected), os, od);
  Ray out;
  if (st == BZR_RR_NONE) {  // the input ray, as the batch path returns it
    os = s;
    od = d;
  }
  out.mStart = vec(os);
  out.mDirection = vec(od);
  return {out, static_cast<RefractionResult>(st)};
}

}  // namespace host
}  // namespace bzr
