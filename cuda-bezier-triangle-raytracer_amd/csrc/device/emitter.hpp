// emitter.hpp -- the illumination pipeline's ray source and target (device side).
//
// Emitter: UniformHemisphere::getRandom's distribution (reference/hostUtil.cpp:16-29): cos(incidence)
// uniform in [0,1), turn uniform in [0, 2*pi), direction (cos, sin*cos(turn), sin*sin(turn)), and its
// patch numbering (reference/hostUtil.cpp:3-14) -- drawn from a counter-based generator so any ray
// range is independent of the others.  Every step is plain binary32 arithmetic (the turn's cos/sin
// by fixed polynomials), compiled with -ffp-contract=off: the oracle's restatement
// (oracle/illum_oracle.c) reproduces the rays bit for bit.
// Target: Plane::intersect (reference/3dGeomUtil.h:279-296) with the target plane, then binning.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "bzr.h"
#include "patch_math.hpp"

namespace bzr_dev {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {  // splitmix64 finaliser
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// two 24-bit uniforms in [0,1) for (seed, key, stream)
__device__ __forceinline__ void uniform2(uint64_t seed, uint64_t key, uint32_t stream, float &u, float &v) {
  const uint64_t h = mix64(seed + 0x9E3779B97F4A7C15ull * (2ull * key + stream + 1ull));
  u = (float)(uint32_t)(h >> 40) * 0x1p-24f;
  v = (float)(uint32_t)((h >> 16) & 0xFFFFFFull) * 0x1p-24f;
}
// (cos, sin) of 2*pi*u, u in [0,1): quadrant reduction, then Taylor polynomials on [0, pi/2)
__device__ __forceinline__ void sincos_turn(float u, float &c, float &s) {
  const float x = u * 4.0f;
  const int q = (int)x;
  const float t = (x - (float)q) * 1.57079632679489662f;
  const float t2 = t * t;
  const float sp =
      t * (1.0f + t2 * (-1.66666667e-1f + t2 * (8.33333333e-3f + t2 * (-1.98412698e-4f + t2 * (2.75573192e-6f +
                                                                                            t2 * -2.50521084e-8f)))));
  const float cp =
      1.0f + t2 * (-0.5f + t2 * (4.16666667e-2f + t2 * (-1.38888889e-3f + t2 * (2.48015873e-5f +
                                                                                  t2 * (-2.75573192e-7f + t2 * 2.08767570e-9f)))));
  switch (q & 3) {
    case 0: c = cp; s = sp; break;
    case 1: c = -sp; s = cp; break;
    case 2: c = -cp; s = -sp; break;
    default: c = sp; s = -cp; break;
  }
}

// Hemisphere patch numbering of UniformHemisphere(belts): belt i spans incidence [i, i+1) * pi/2/belts
// and holds count[i] patches of equal turn width, numbered from first[i].  cos_lo[i] = cos(i * width)
// (i >= 1): the incidence is in belt >= i exactly when cos(incidence) <= cos_lo[i].
struct BeltTable {
  const float *cos_lo;
  const uint32_t *count, *first;
  uint32_t belts;
};

__device__ __forceinline__ uint32_t hemisphere_patch(const BeltTable &bt, float cos_inc, float turn_frac) {
  uint32_t belt = 0;
  for (uint32_t i = 1; i < bt.belts; ++i) belt += cos_inc <= bt.cos_lo[i] ? 1u : 0u;
  const uint32_t cnt = bt.count[belt];
  uint32_t k = (uint32_t)(turn_frac * (float)cnt);
  if (k >= cnt) k = cnt - 1u;
  return bt.first[belt] + k;
}

// Ray `j` of the emitter: origin on the emitter rectangle, unit direction, hemisphere patch index.
__device__ __forceinline__ void emit_ray(const bzr_emitter &em, const BeltTable &bt, uint64_t j, f3 &o, f3 &d,
                                         uint32_t &patch) {
  const uint64_t per_part = (uint64_t)em.points_per_part * em.rays_per_point;
  const uint64_t point = j / em.rays_per_point;
  const uint64_t part = (j / per_part) % ((uint64_t)em.parts_u * em.parts_v);
  const uint32_t pu = (uint32_t)(part % em.parts_u), pv = (uint32_t)(part / em.parts_u);
  float a, b;
  uniform2(em.seed, point, 1u, a, b);
  a = ((float)pu + a) / (float)em.parts_u;
  b = ((float)pv + b) / (float)em.parts_v;
  o = mk((em.origin[0] + em.edge_u[0] * a) + em.edge_v[0] * b, (em.origin[1] + em.edge_u[1] * a) + em.edge_v[1] * b,
         (em.origin[2] + em.edge_u[2] * a) + em.edge_v[2] * b);
  float ci, tf;
  uniform2(em.seed, j, 0u, ci, tf);
  float ct, st;
  sincos_turn(tf, ct, st);
  const float si = sqrt_rn(1.0f - ci * ci);
  d = normalized(mk(ci, si * ct, si * st));
  patch = hemisphere_patch(bt, ci, tf);
}

// false when the ray cannot meet the sphere (centre c, radius r): its start is outside and it points
// away or passes by.  In double: the discriminant cancels badly in binary32 for far starts.
__device__ __forceinline__ bool may_hit_sphere(f3 s, f3 d, const float sphere[4]) {
  const double ox = (double)s.x - sphere[0], oy = (double)s.y - sphere[1], oz = (double)s.z - sphere[2];
  const double r = sphere[3];
  const double cc = ox * ox + oy * oy + oz * oz - r * r;
  if (cc <= 0.0) return true;  // starts inside
  const double bb = ox * d.x + oy * d.y + oz * d.z;
  if (bb >= 0.0) return false;
  return bb * bb - cc >= 0.0;
}

// Target cell of a ray leaving the last lens, or -1: Plane::intersect (valid iff t > 0, D1) with the
// plane (n, c) through the target, then (u, v) coordinates / cell sizes.
__device__ __forceinline__ int32_t target_cell(const bzr_target &tg, f3 n, float c, float cell_u, float cell_v, f3 s,
                                               f3 d) {
  f3 p;
  float cs, t;
  if (!plane_ray(n, c, s, d, p, cs, t)) return -1;
  const f3 rel = sub(p, mk(tg.origin[0], tg.origin[1], tg.origin[2]));
  const float a = dot(rel, mk(tg.axis_u[0], tg.axis_u[1], tg.axis_u[2]));
  const float b = dot(rel, mk(tg.axis_v[0], tg.axis_v[1], tg.axis_v[2]));
  if (!(a >= 0.0f && a < tg.size_u && b >= 0.0f && b < tg.size_v)) return -1;
  uint32_t iu = (uint32_t)(a / cell_u), iv = (uint32_t)(b / cell_v);
  if (iu >= tg.bins_u) iu = tg.bins_u - 1u;
  if (iv >= tg.bins_v) iv = tg.bins_v - 1u;
  return (int32_t)(iv * tg.bins_u + iu);
}

}  // namespace bzr_dev
