// patch_math.hpp -- device arithmetic of the hot path, one ray per lane.
//
// Every function evaluates in IEEE binary32 with the operation order of the
// reference (Eigen 3.3 fixed-size semantics, see include/bzr/bzr.hpp) and must
// be compiled with -ffp-contract=off: the results are then bit-identical to
// the CPU oracle (oracle/bzr_oracle.c), which tests/test_gpu_parity.py checks.
//   plane_ray        reference/3dGeomUtil.h:279-296 (+ deviations D1/D2)
//   interpolate      reference/bezierTriangle.cpp:105-121
//   surface_normal   reference/bezierTriangle.cpp:197-233
//   patch_intersect  reference/bezierTriangle.cpp:123-195
#pragma once
#include <hip/hip_runtime.h>
#include <cfloat>
#include <cstdint>

namespace bzr_dev {

// Correctly rounded binary32 division and square root.  HIP compiles `/` and
// __builtin_sqrtf correctly rounded by default (-fhip-fp32-correctly-rounded-divide-sqrt);
// note __fsqrt_rn is NOT: it maps to the approximate __ocml_native_sqrt_f32 in ROCm 7.2.
__device__ __forceinline__ float div_rn(float a, float b) { return a / b; }
__device__ __forceinline__ float sqrt_rn(float a) { return __builtin_sqrtf(a); }

struct f3 {
  float x, y, z;
};
__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 scale(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + (a.y * b.y + a.z * b.z); }
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
  return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ f3 normalized(f3 a) {
  float z = dot(a, a);
  if (z > 0.0f) {
    float s = sqrt_rn(z);
    return mk(div_rn(a.x, s), div_rn(a.y, s), div_rn(a.z, s));
  }
  return a;
}
__device__ __forceinline__ float norm(f3 a) { return sqrt_rn(dot(a, a)); }

// Patch record = the reference's BezierTriangle, 66 words (include/bzr.h bzr_patch).
namespace rec {
constexpr int kUnder = 0;     // n.xyz, c
constexpr int kDivider = 4;   // 3 x (n.xyz, c)
constexpr int kNeigh = 16;    // 3 x u32
constexpr int kCp = 19;       // 10 x xyz
constexpr int kMinv = 49;     // 3x3 col-major
constexpr int kHin = 58;
constexpr int kHout = 59;
constexpr int kDirA = 60;
constexpr int kDirB = 63;
constexpr int kWords = 66;
}  // namespace rec

// Two interchangeable patch sources for the math below (same accessors, same arithmetic):
//   Patch          the record held in registers (per-lane patches)
//   PatchView<P>   reads the record at its point of use through P; with a constant-address-space
//                  P (uniform_patch) the words are scalar loads, so a wave-uniform record occupies
//                  SGPRs only while in use instead of all 66 words at once
struct Patch {  // registers holding one record
  f3 n_;
  float c_;
  f3 dn_[3];
  float dc_[3];
  f3 cp_[10];
  float m_[9];  // col-major
  float hin_, hout_;
  f3 da_, db_;
  __device__ __forceinline__ f3 n() const { return n_; }
  __device__ __forceinline__ float c() const { return c_; }
  __device__ __forceinline__ f3 dn(int k) const { return dn_[k]; }
  __device__ __forceinline__ float dc(int k) const { return dc_[k]; }
  __device__ __forceinline__ f3 cp(int k) const { return cp_[k]; }
  __device__ __forceinline__ float m(int k) const { return m_[k]; }
  __device__ __forceinline__ float hin() const { return hin_; }
  __device__ __forceinline__ float hout() const { return hout_; }
  __device__ __forceinline__ f3 da() const { return da_; }
  __device__ __forceinline__ f3 db() const { return db_; }
};

template <typename Ptr>
struct PatchView {
  Ptr r;
  __device__ __forceinline__ f3 v3(int o) const { return mk(r[o], r[o + 1], r[o + 2]); }
  __device__ __forceinline__ f3 n() const { return v3(0); }
  __device__ __forceinline__ float c() const { return r[3]; }
  __device__ __forceinline__ f3 dn(int k) const { return v3(rec::kDivider + 4 * k); }
  __device__ __forceinline__ float dc(int k) const { return r[rec::kDivider + 4 * k + 3]; }
  __device__ __forceinline__ f3 cp(int k) const { return v3(rec::kCp + 3 * k); }
  __device__ __forceinline__ float m(int k) const { return r[rec::kMinv + k]; }
  __device__ __forceinline__ float hin() const { return r[rec::kHin]; }
  __device__ __forceinline__ float hout() const { return r[rec::kHout]; }
  __device__ __forceinline__ f3 da() const { return v3(rec::kDirA); }
  __device__ __forceinline__ f3 db() const { return v3(rec::kDirB); }
};

__device__ __forceinline__ Patch load_patch(const float *__restrict__ r) {
  Patch p;
  p.n_ = mk(r[0], r[1], r[2]);
  p.c_ = r[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    p.dn_[k] = mk(r[rec::kDivider + 4 * k], r[rec::kDivider + 4 * k + 1], r[rec::kDivider + 4 * k + 2]);
    p.dc_[k] = r[rec::kDivider + 4 * k + 3];
  }
#pragma unroll
  for (int k = 0; k < 10; ++k) p.cp_[k] = mk(r[rec::kCp + 3 * k], r[rec::kCp + 3 * k + 1], r[rec::kCp + 3 * k + 2]);
#pragma unroll
  for (int k = 0; k < 9; ++k) p.m_[k] = r[rec::kMinv + k];
  p.hin_ = r[rec::kHin];
  p.hout_ = r[rec::kHout];
  p.da_ = mk(r[rec::kDirA], r[rec::kDirA + 1], r[rec::kDirA + 2]);
  p.db_ = mk(r[rec::kDirB], r[rec::kDirB + 1], r[rec::kDirB + 2]);
  return p;
}

typedef __attribute__((address_space(4))) const float const_float;
// View of record `index` for a wave-uniform index (constant address space: scalar loads).
__device__ __forceinline__ PatchView<const const_float *> uniform_patch(const float *base, uint32_t index) {
  return PatchView<const const_float *>{(const const_float *)(uintptr_t)(base + (size_t)rec::kWords * index)};
}

template <typename P>
__device__ __forceinline__ f3 matvec(const P &p, f3 v) {  // Eigen row redux over the col-major M
  return mk(p.m(0) * v.x + (p.m(3) * v.y + p.m(6) * v.z), p.m(1) * v.x + (p.m(4) * v.y + p.m(7) * v.z),
            p.m(2) * v.x + (p.m(5) * v.y + p.m(8) * v.z));
}

// Plane::intersect(start, dir) with D1 (point for any t) and D2 (point = start when |cos| < eps)
__device__ __forceinline__ bool plane_ray(f3 n, float c, f3 start, f3 dir, f3 &point, float &cs, float &t) {
  cs = dot(dir, n);
  if (fabsf(cs) >= 0.00001f) {
    t = div_rn(c - dot(n, start), cs);
    point = add(start, scale(dir, t));
    return t > 0.0f;
  }
  t = 0.0f;
  point = start;
  return false;
}

__device__ __forceinline__ float plane_distance(f3 n, float c, f3 p) { return dot(p, n) - c; }
__device__ __forceinline__ f3 plane_project(f3 n, float c, f3 p) { return sub(p, scale(n, dot(p, n) - c)); }

template <typename P>
__device__ __forceinline__ f3 interpolate(const P &p, f3 b) {
  float q0 = b.x * b.x, q1 = b.y * b.y, q2 = b.z * b.z;
#define c(k) p.cp(k)
#define BZR_IP(F)                                                                                      \
  (((((c(0).F * b.x) * q0 + (c(1).F * b.y) * q1) + (c(2).F * b.z) * q2) +                             \
    3.0f * ((((((c(3).F * b.y) * q0 + (c(4).F * b.x) * q1) + (c(5).F * b.z) * q1) + (c(6).F * b.y) * q2) + \
             (c(7).F * b.x) * q2) +                                                                    \
            (c(8).F * b.z) * q0)) +                                                                    \
   (((c(9).F * b.x) * b.y) * b.z) * 6.0f)
  return mk(BZR_IP(x), BZR_IP(y), BZR_IP(z));
#undef BZR_IP
#undef c
}

template <typename P>
__device__ __forceinline__ f3 surface_normal(const P &p, f3 b) {
  float q0 = b.x * b.x, q1 = b.y * b.y, q2 = b.z * b.z;
#define c(k) p.cp(k)
  // control point slots: 300=0 030=1 003=2 210=3 120=4 021=5 012=6 102=7 201=8 111=9
#define BZR_K0(F) (((c(0).F * q0 + c(7).F * q2) + c(4).F * q1) + 2.0f * (((c(8).F * b.x) * b.z + (c(3).F * b.x) * b.y) + (c(9).F * b.z) * b.y))
#define BZR_K1(F) (((c(1).F * q1 + c(6).F * q2) + c(3).F * q0) + 2.0f * (((c(9).F * b.x) * b.z + (c(4).F * b.x) * b.y) + (c(5).F * b.y) * b.z))
#define BZR_K2(F) (((c(2).F * q2 + c(8).F * q0) + c(5).F * q1) + 2.0f * (((c(7).F * b.x) * b.z + (c(6).F * b.y) * b.z) + (c(9).F * b.x) * b.y))
  f3 k0 = mk(BZR_K0(x), BZR_K0(y), BZR_K0(z));
  f3 k1 = mk(BZR_K1(x), BZR_K1(y), BZR_K1(z));
  f3 k2 = mk(BZR_K2(x), BZR_K2(y), BZR_K2(z));
#undef BZR_K0
#undef BZR_K1
#undef BZR_K2
#undef c
  const f3 da = p.da(), db = p.db();
  f3 ca = mk((da.x * k0.x + da.y * k1.x) + da.z * k2.x, (da.x * k0.y + da.y * k1.y) + da.z * k2.y,
             (da.x * k0.z + da.y * k1.z) + da.z * k2.z);
  f3 cb = mk((db.x * k0.x + db.y * k1.x) + db.z * k2.x, (db.x * k0.y + db.y * k1.y) + db.z * k2.y,
             (db.x * k0.z + db.y * k1.z) + db.z * k2.z);
  return normalized(cross(ca, cb));
}

struct Hit {
  float t;
  f3 point;
  float cs;
  f3 bary;
  f3 normal;
  uint32_t what;  // 0..2 follow side, 3 none, 4 intersect
};

#ifndef BZR_NEWTON_ITERS
#define BZR_NEWTON_ITERS 4
#endif
constexpr uint32_t kFollow2 = 2u, kNone = 3u, kIntersect = 4u;

// BezierTriangle::intersect (reference/bezierTriangle.cpp:123-195).  limitNone: 0 = cThis, 1 = cNone.
// kGated: the caller has already evaluated the planar gate (:124-131) with this same arithmetic and
// it passed (the culled pipeline's candidates), so its early returns are skipped -- same result bits.
template <bool kGated = false, typename P>
__device__ __forceinline__ Hit patch_intersect(const P &p, f3 s, f3 d, bool limitNone) {
  Hit h;
  h.t = 0.0f;
  h.point = mk(0.0f, 0.0f, 0.0f);
  h.cs = 0.0f;
  h.bary = h.point;
  h.normal = h.point;
  h.what = kNone;
  f3 ip;
  float ic, it;
  bool valid = plane_ray(p.n(), p.c(), s, d, ip, ic, it);
  if (!kGated) {
    if (!(valid && fabsf(it) > -p.hin() && fabsf(it) > p.hout())) return h;
    f3 b0 = matvec(p, ip);
    if (!(limitNone || (b0.x >= 0.0f && b0.x <= 1.0f && b0.y >= 0.0f && b0.y <= 1.0f && b0.z >= 0.0f && b0.z <= 1.0f)))
      return h;
  }
  float din = div_rn(p.hin(), ic), dout = div_rn(p.hout(), ic);
  float closer = it + (ic > 0.0f ? din : dout);
  float further = it + (ic > 0.0f ? dout : din);
  // secant start between the two bounding heights
  f3 por = add(s, scale(d, closer));
  f3 b = matvec(p, plane_project(p.n(), p.c(), por));
  f3 q = interpolate(p, b);
  float diffc = fabsf(plane_distance(p.n(), p.c(), por)) - fabsf(plane_distance(p.n(), p.c(), q));
  por = add(s, scale(d, further));
  b = matvec(p, plane_project(p.n(), p.c(), por));
  q = interpolate(p, b);
  float difff = fabsf(plane_distance(p.n(), p.c(), por)) - fabsf(plane_distance(p.n(), p.c(), q));
  float den = diffc - difff;
  float middle = fabsf(den) < 0.000001f ? div_rn(closer + further, 2.0f)
                                        : div_rn(diffc * further - difff * closer, den);
  f3 pdir = p.n();
  for (int i = 0; i < BZR_NEWTON_ITERS; ++i) {  // csRootSearchIterations
    h.t = middle;
    por = add(s, scale(d, middle));
    f3 pp;
    float pc, pt;
    plane_ray(p.n(), p.c(), por, pdir, pp, pc, pt);
    h.bary = matvec(p, pp);
    h.normal = surface_normal(p, h.bary);
    h.point = interpolate(p, h.bary);
    pdir = normalized(sub(h.point, pp));
    middle = div_rn(dot(sub(h.point, s), h.normal), dot(d, h.normal));
  }
  f3 rel = sub(h.point, s);
  f3 perp = sub(rel, scale(d, dot(rel, d)));
  if (norm(perp) > 0.01f || h.t < (further - closer) * 1.0f) {
    h.what = kNone;
    return h;
  }
  uint32_t out = plane_distance(p.dn(0), p.dc(0), h.point) < 0.0f ? 1u : 0u;
  out |= plane_distance(p.dn(1), p.dc(1), h.point) < 0.0f ? 2u : 0u;
  out |= plane_distance(p.dn(2), p.dc(2), h.point) < 0.0f ? 4u : 0u;
  if (out == 1u) h.what = 0u;
  else if (out == 2u) h.what = 1u;
  else if (out == 4u) h.what = 2u;
  else {
    h.what = kIntersect;
    h.cs = dot(d, h.normal);
  }
  return h;
}

}  // namespace bzr_dev
