// patch_math.hpp -- device arithmetic of the hot path, one ray per lane.
//
// The exact:: arithmetic (patch_math_body.inc) evaluates in IEEE binary32 with the
// operation order of the reference (Eigen 3.3 fixed-size semantics, see
// include/bzr/bzr.hpp) and must be compiled with -ffp-contract=off: the results are
// then bit-identical to the CPU oracle (oracle/bzr_oracle.c), which
// tests/test_gpu_parity.py checks.  fast:: is the same text with contraction and
// approximate div/sqrt, used after the (always exact) planar gate in BZR_MODE_FAST.
//   plane_ray        reference/3dGeomUtil.h:279-296 (+ deviations D1/D2)
//   interpolate      reference/bezierTriangle.cpp:105-121
//   surface_normal   reference/bezierTriangle.cpp:197-233
//   patch_intersect  reference/bezierTriangle.cpp:123-195
#pragma once
#include <hip/hip_runtime.h>
#include <cfloat>
#include <cstdint>

namespace bzr_dev {

struct f3 {
  float x, y, z;
};
__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
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
// BZR_NEWTON_UNROLL (default 1): unroll the 4 Newton iterations (+1.7 % fused cfg4, +0.7 % staged cfg2/cfg3).
#ifndef BZR_NEWTON_UNROLL
#define BZR_NEWTON_UNROLL 1
#endif
constexpr uint32_t kFollow2 = 2u, kNone = 3u, kIntersect = 4u;
// BZR_PASS_FLAT (default 0): patch_intersect's gate without the early return (see there).
#ifndef BZR_PASS_FLAT
#define BZR_PASS_FLAT 0
#endif

// Correctly rounded binary32 division and square root.  HIP compiles `/` and
// __builtin_sqrtf correctly rounded by default (-fhip-fp32-correctly-rounded-divide-sqrt);
// note __fsqrt_rn is NOT: it maps to the approximate __ocml_native_sqrt_f32 in ROCm 7.2.
namespace exact {
__device__ __forceinline__ float div_rn(float a, float b) { return a / b; }
__device__ __forceinline__ float sqrt_rn(float a) { return __builtin_sqrtf(a); }

// The two sequences above, as LLVM lowers them for gfx950, minus their range handling:
//   sqrt: v_sqrt_f32, then the neighbours s -/+ 1 ulp are tested with fma residuals; LLVM first scales
//         z < 2^-96 by 2^32 and passes 0 / inf / NaN through (v_cmp_class);
//   a/b:  v_div_scale (num, den), v_rcp_f32, one Newton step of the reciprocal, q = num*y, two fma
//         corrections (the second is v_div_fmas), v_div_fixup (signs, zeros, inf/NaN, overflow).
// Where v_div_scale scales nothing and v_div_fixup passes the quotient through, the plain fma chain is
// the same instructions on the same values, so it returns the same correctly rounded bits.  V_DIV_SCALE
// scales when: num or den is 0; exp(num) - exp(den) >= 96; den is denormal; 1/den or num/den is
// denormal; |num| < 2^-103.  unit_or_self() takes the plain chain only when |a_k| >= 2^-100 for every k and
// 2^-96 <= z <= 2^40 (so s = sqrt(z) is in [2^-48, 2^20] and |a_k| / s >= 2^-120 is normal; |a_k| <= ~s):
// none of those cases, no sqrt scaling, no special value.  The three quotients share the divisor, so
// they share the reciprocal: 1 sqrt + 3 + 3 x 5 instructions instead of 1 + 3 x 11.
__device__ __forceinline__ float sqrt_unscaled(float z) {
  const float s = __builtin_amdgcn_sqrtf(z);
  const float lo = __uint_as_float(__float_as_uint(s) - 1u), hi = __uint_as_float(__float_as_uint(s) + 1u);
  const float rlo = __builtin_fmaf(-lo, s, z), rhi = __builtin_fmaf(-hi, s, z);
  const float t = rlo <= 0.0f ? lo : s;
  return rhi > 0.0f ? hi : t;
}
__device__ __forceinline__ float div_unscaled(float a, float b, float y) {  // y: the refined 1/b
  float q = a * y;
  float r = __builtin_fmaf(-b, q, a);
  q = __builtin_fmaf(r, y, q);
  r = __builtin_fmaf(-b, q, a);
  return __builtin_fmaf(r, y, q);
}
// newton_tail's acceptance test norm(perp) > 0.01f (reference/bezierTriangle.cpp:165) without the square
// root: RN(sqrt(z)) is monotone in z, so RN(sqrt(z)) > 0.01f exactly when z > 0x38d1b718 (1.00000005e-4f),
// the largest float whose correctly rounded square root is <= 0.01f -- checked over all 2^32 float bit
// patterns, NaN and negatives included (tests/test_sqrt_threshold.py repeats it on a sample).
__device__ __forceinline__ bool sqrt_above_hundredth(float z) { return z > __uint_as_float(0x38d1b718u); }
#ifndef BZR_UNIT_SHARED
#define BZR_UNIT_SHARED 1
#endif
// Eigen normalized() with z = a.a: a / sqrt(z) when z > 0, else a unchanged.
__device__ __forceinline__ f3 unit_or_self(f3 a, float z) {
#if BZR_UNIT_SHARED
  // the plain chain for every lane; lanes outside the guard (z <= 0 among them) redo it with the full
  // sequences or keep a (the branch is rarely taken, and the common path needs no copies at the join)
  const float s = sqrt_unscaled(z);
  const float y0 = __builtin_amdgcn_rcpf(s);
  const float y = __builtin_fmaf(__builtin_fmaf(-s, y0, 1.0f), y0, y0);
  f3 r = mk(div_unscaled(a.x, s, y), div_unscaled(a.y, s, y), div_unscaled(a.z, s, y));
  const float m = fminf(fminf(fabsf(a.x), fabsf(a.y)), fabsf(a.z));
  if (!(m >= 0x1p-100f && z >= 0x1p-96f && z <= 0x1p40f)) {
    r = a;
    if (z > 0.0f) {
      const float sr = sqrt_rn(z);
      r = mk(div_rn(a.x, sr), div_rn(a.y, sr), div_rn(a.z, sr));
    }
  }
  return r;
#else
  if (!(z > 0.0f)) return a;
  float s = sqrt_rn(z);
  return mk(div_rn(a.x, s), div_rn(a.y, s), div_rn(a.z, s));
#endif
}
// BZR_DIV_HEIGHTS (default 1): newton_tail's two bracket quotients din = hIn / cos and dout = hOut / cos
// (reference/bezierTriangle.cpp:132-133) share their divisor, so they share one refined reciprocal and take the
// plain fma chain (div_unscaled) -- 3 + 2 x 5 VALU instead of 2 x 11 -- when it provably returns the correctly
// rounded quotient: the heights are record constants with 2^-40 <= |h| < 2^41 (an exponent test, on the scalar
// unit when the record sits in SGPRs) and every lane's |cos| lies in [2^-20, 2^20] (the planar gate that let the
// lane in already requires |cos| >= 1e-5), so V_DIV_SCALE scales nothing (no zero, no denormal divisor,
// reciprocal or quotient, exponent gap < 96, |num| >= 2^-103) and V_DIV_FIXUP passes the quotient through.
// Otherwise (a zero height, an extreme lane) both lanes' quotients take the full sequences.  Same bits either
// way (division sites).
#ifndef BZR_DIV_HEIGHTS
#define BZR_DIV_HEIGHTS 1
#endif
__device__ __forceinline__ bool height_in_range(float h) {
  const uint32_t e = (__float_as_uint(h) >> 23) & 0xFFu;  // biased exponent: 2^-40 <= |h| < 2^41
  return e - (127u - 40u) <= 80u;
}
__device__ __forceinline__ void div_heights(float hin, float hout, float ic, float &din, float &dout) {
#if BZR_DIV_HEIGHTS
  const bool ok = height_in_range(hin) && height_in_range(hout) && fabsf(ic) >= 0x1p-20f && fabsf(ic) <= 0x1p20f;
  if (__all(ok)) {
    const float y0 = __builtin_amdgcn_rcpf(ic);
    const float y = __builtin_fmaf(__builtin_fmaf(-ic, y0, 1.0f), y0, y0);
    din = div_unscaled(hin, ic, y);
    dout = div_unscaled(hout, ic, y);
    return;
  }
#endif
  din = div_rn(hin, ic);
  dout = div_rn(hout, ic);
}
#include "patch_math_body.inc"
}  // namespace exact

// BZR_MODE_FAST: contracted FMA, v_rcp_f32 / v_sqrt_f32 / v_rsq_f32 (about 1 ulp each).
namespace fast {
#pragma clang fp contract(fast)
__device__ __forceinline__ float div_rn(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }
__device__ __forceinline__ float sqrt_rn(float a) { return __builtin_amdgcn_sqrtf(a); }
__device__ __forceinline__ bool sqrt_above_hundredth(float z) { return sqrt_rn(z) > 0.01f; }
__device__ __forceinline__ f3 unit_or_self(f3 a, float z) {
  if (!(z > 0.0f)) return a;
  float r = __builtin_amdgcn_rsqf(z);
  return mk(a.x * r, a.y * r, a.z * r);
}
__device__ __forceinline__ void div_heights(float hin, float hout, float ic, float &din, float &dout) {
  din = div_rn(hin, ic);
  dout = div_rn(hout, ic);
}
#include "patch_math_body.inc"
#pragma clang fp contract(off)
}  // namespace fast

// Everything outside the Newton stage evaluates exactly.  (No arithmetic function is declared in
// bzr_dev itself, so argument-dependent lookup on f3 / Patch never mixes the two namespaces.)
using namespace exact;

// BezierTriangle::intersect (reference/bezierTriangle.cpp:123-195).  limitNone: 0 = cThis, 1 = cNone.
// kGated: the caller has already evaluated the planar gate (:124-131) with this same arithmetic and
// it passed (the culled pipeline's candidates), so its early returns are skipped -- same result bits.
// kFast: the gate stays exact (same candidates as the reference), the rest runs in fast::.
template <bool kGated = false, bool kFast = false, typename P>
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
  (void)valid;
#if BZR_PASS_FLAT
  if (!kGated) {
    // Branch-free form: every lane of the call runs the Newton tail and lanes whose gate fails get the
    // kNone record afterwards -- the same bits for the lanes that pass, and no divergent branch, so the
    // record's scalar loads need not wait inside one (they batch ahead of the arithmetic).
    const f3 b0 = matvec(p, ip);
    const bool in = (b0.x >= 0.0f) & (b0.x <= 1.0f) & (b0.y >= 0.0f) & (b0.y <= 1.0f) & (b0.z >= 0.0f) & (b0.z <= 1.0f);
    const bool ok = valid & (fabsf(it) > -p.hin()) & (fabsf(it) > p.hout()) & (limitNone | in);
    Hit r;
    if constexpr (kFast) r = fast::newton_tail(p, s, d, ic, it);
    else r = newton_tail(p, s, d, ic, it);
    return ok ? r : h;
  }
#endif
  if (!kGated) {
    if (!(valid && fabsf(it) > -p.hin() && fabsf(it) > p.hout())) return h;
    f3 b0 = matvec(p, ip);
    if (!(limitNone || (b0.x >= 0.0f && b0.x <= 1.0f && b0.y >= 0.0f && b0.y <= 1.0f && b0.z >= 0.0f && b0.z <= 1.0f)))
      return h;
  }
  if constexpr (kFast) return fast::newton_tail(p, s, d, ic, it);
  else return newton_tail(p, s, d, ic, it);
}

}  // namespace bzr_dev
