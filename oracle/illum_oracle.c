/*
 * illum_oracle.c -- TEST INFRASTRUCTURE ONLY (part of liboracle.so, see bzr_oracle.h).
 *
 * CPU restatement of the illumination pipeline's two ends, the checker for libbzr's bzr_emit /
 * bzr_illuminate (DESIGN.md section f):
 *   - UniformHemisphere (reference/hostUtil.cpp:3-29) exactly as the reference runs it:
 *     std::ranlux24_base (subtract_with_carry_engine<uint_fast32_t, 24, 10, 24>, default seed
 *     19780503 through linear_congruential_engine<uint_fast32_t, 40014, 0, 2147483563>),
 *     std::uniform_real_distribution<float> via libstdc++'s generate_canonical<float, 24>, and the
 *     C double acos / sin / cos the reference's ::acos(float) calls bind (see orc_hemisphere_random);
 *   - the counter-based emitter (the reference's sampling formulas from a splitmix64 stream) and the
 *     target-plane binning, in the same binary32 operation order as the device code.
 * Build with -ffp-contract=off (oracle/Makefile).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "bzr_oracle.h"

/* ---------------------------------------------------------------- UniformHemisphere */
static const float kPi = 3.14159265358979323846f; /* cgPi, reference/3dGeomUtil.h:19 */

struct orc_hemisphere {
  /* ranlux24_base */
  uint32_t x[24];
  uint32_t carry;
  uint32_t p;
  /* UniformHemisphere */
  float belt_width;
  uint32_t belts;
  float *patch_width;
  uint32_t *so_far;
  uint32_t patch_count;
};

static void ranlux_seed(orc_hemisphere *h, uint32_t value) {
  uint64_t lcg = (value == 0u ? 19780503u : value) % 2147483563u; /* linear_congruential_engine seed */
  if (lcg == 0u) lcg = 1u;
  for (int i = 0; i < 24; ++i) {
    lcg = (40014u * lcg) % 2147483563u;
    h->x[i] = (uint32_t)(lcg & 0xFFFFFFu); /* sum mod 2^24 */
  }
  h->carry = h->x[23] == 0u ? 1u : 0u;
  h->p = 0u;
}

static uint32_t ranlux_next(orc_hemisphere *h) { /* subtract with carry, r = 24, s = 10, w = 24 */
  int ps = (int)h->p - 10;
  if (ps < 0) ps += 24;
  uint32_t xi;
  if (h->x[ps] >= h->x[h->p] + h->carry) {
    xi = h->x[ps] - h->x[h->p] - h->carry;
    h->carry = 0u;
  } else {
    xi = (1u << 24) - h->x[h->p] - h->carry + h->x[ps];
    h->carry = 1u;
  }
  h->x[h->p] = xi;
  h->p = (h->p + 1u) % 24u;
  return xi;
}

static float canonical(orc_hemisphere *h) { /* generate_canonical<float, 24>: one draw, range 2^24 */
  float ret = (float)ranlux_next(h) * 1.0f / 16777216.0f;
  if (ret >= 1.0f) ret = nextafterf(1.0f, 0.0f);
  return ret;
}

orc_hemisphere *orc_hemisphere_create(uint32_t belts) { /* reference/hostUtil.cpp:3-14 */
  orc_hemisphere *h = (orc_hemisphere *)calloc(1, sizeof(orc_hemisphere));
  if (!h) return NULL;
  ranlux_seed(h, 19780503u);
  h->belts = belts;
  h->belt_width = kPi / 2.0f / (float)belts;
  h->patch_width = (float *)calloc(belts ? belts : 1, sizeof(float));
  h->so_far = (uint32_t *)calloc(belts ? belts : 1, sizeof(uint32_t));
  h->patch_count = 0u;
  for (uint32_t i = 0; i < belts; ++i) {
    uint32_t now = (uint32_t)ceil((double)(4.0f * (float)belts) * sin((double)((2.0f * (float)i + 1.0f) / (4.0f * (float)belts) * kPi)));
    h->patch_width[i] = kPi * 2.0f / (float)now;
    h->so_far[i] = h->patch_count;
    h->patch_count += now;
  }
  return h;
}

void orc_hemisphere_free(orc_hemisphere *h) {
  if (!h) return;
  free(h->patch_width);
  free(h->so_far);
  free(h);
}

uint32_t orc_hemisphere_patch_count(const orc_hemisphere *h) { return h->patch_count; }

/* UniformHemisphere::getRandom (reference/hostUtil.cpp:16-29) -> direction, patch index.
 * `::acos(float)` etc. in the reference bind C's double functions (its include chain, Eigen's
 * <cmath>, puts no float overloads in the global namespace), and `beltRadius * ::cos(turn)` is a
 * double product rounded once to float on assignment.  uniform_real_distribution<float> returns
 * canonical * (b - a) + a. */
uint32_t orc_hemisphere_random(orc_hemisphere *h, float dir[3]) {
  const float incidence = (float)acos((double)(canonical(h) * (1.0f - 0.0f) + 0.0f));
  const float belt_radius = (float)sin((double)incidence);
  const float turn = canonical(h) * (kPi * 2.0f - 0.0f) + 0.0f;
  float d[3] = {(float)cos((double)incidence), (float)((double)belt_radius * cos((double)turn)),
                (float)((double)belt_radius * sin((double)turn))};
  const float z = d[0] * d[0] + (d[1] * d[1] + d[2] * d[2]); /* Vector::normalize (Eigen) */
  if (z > 0.0f) {
    const float s = sqrtf(z);
    for (int k = 0; k < 3; ++k) d[k] = d[k] / s;
  }
  memcpy(dir, d, sizeof(d));
  const uint32_t belt = (uint32_t)(incidence / h->belt_width);
  return h->so_far[belt] + (uint32_t)(turn / h->patch_width[belt]);
}

/* ---------------------------------------------------------------- counter-based emitter */
static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static void uniform2(uint64_t seed, uint64_t key, uint32_t stream, float *u, float *v) {
  const uint64_t h = mix64(seed + 0x9E3779B97F4A7C15ull * (2ull * key + stream + 1ull));
  *u = (float)(uint32_t)(h >> 40) * 0x1p-24f;
  *v = (float)(uint32_t)((h >> 16) & 0xFFFFFFull) * 0x1p-24f;
}

static void sincos_turn(float u, float *c, float *s) {
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
    case 0: *c = cp; *s = sp; break;
    case 1: *c = -sp; *s = cp; break;
    case 2: *c = -cp; *s = -sp; break;
    default: *c = sp; *s = -cp; break;
  }
}

int orc_emit(const orc_emitter *em, uint64_t first, uint32_t n, float *rays_soa, uint32_t *patch) {
  if (!em->parts_u || !em->parts_v || !em->points_per_part || !em->rays_per_point || !em->belts) return 1;
  const uint32_t belts = em->belts;
  const float width = kPi / 2.0f / (float)belts;
  float *cos_lo = (float *)malloc(belts * sizeof(float));
  uint32_t *count = (uint32_t *)malloc(belts * sizeof(uint32_t)), *firsts = (uint32_t *)malloc(belts * sizeof(uint32_t));
  uint32_t so_far = 0;
  for (uint32_t i = 0; i < belts; ++i) {
    count[i] = (uint32_t)ceil((double)(4.0f * (float)belts) * sin((double)((2.0f * (float)i + 1.0f) / (4.0f * (float)belts) * kPi)));
    firsts[i] = so_far;
    so_far += count[i];
    cos_lo[i] = i ? cosf((float)i * width) : 1.0f;
  }
  const uint64_t per_part = (uint64_t)em->points_per_part * em->rays_per_point;
  for (uint32_t r = 0; r < n; ++r) {
    const uint64_t j = first + r;
    const uint64_t point = j / em->rays_per_point;
    const uint64_t part = (j / per_part) % ((uint64_t)em->parts_u * em->parts_v);
    const uint32_t pu = (uint32_t)(part % em->parts_u), pv = (uint32_t)(part / em->parts_u);
    float a, b;
    uniform2(em->seed, point, 1u, &a, &b);
    a = ((float)pu + a) / (float)em->parts_u;
    b = ((float)pv + b) / (float)em->parts_v;
    float o[3];
    for (int k = 0; k < 3; ++k) o[k] = (em->origin[k] + em->edge_u[k] * a) + em->edge_v[k] * b;
    float ci, tf, ct, st;
    uniform2(em->seed, j, 0u, &ci, &tf);
    sincos_turn(tf, &ct, &st);
    const float si = sqrtf(1.0f - ci * ci);
    float d[3] = {ci, si * ct, si * st};
    const float z = d[0] * d[0] + (d[1] * d[1] + d[2] * d[2]);
    if (z > 0.0f) {
      const float s = sqrtf(z);
      for (int k = 0; k < 3; ++k) d[k] = d[k] / s;
    }
    for (int k = 0; k < 3; ++k) {
      rays_soa[(size_t)k * n + r] = o[k];
      rays_soa[(size_t)(3 + k) * n + r] = d[k];
    }
    if (patch) {
      uint32_t belt = 0;
      for (uint32_t i = 1; i < belts; ++i) belt += ci <= cos_lo[i] ? 1u : 0u;
      uint32_t k = (uint32_t)(tf * (float)count[belt]);
      if (k >= count[belt]) k = count[belt] - 1u;
      patch[r] = firsts[belt] + k;
    }
  }
  free(cos_lo);
  free(count);
  free(firsts);
  return 0;
}

/* ---------------------------------------------------------------- target plane */
void orc_land(const orc_target *tg, const float *rays_soa, const uint32_t *status, uint32_t n, uint32_t *hist,
              uint64_t *exited, uint64_t *landed) {
  const float *au = tg->axis_u, *av = tg->axis_v;
  float pn[3] = {au[1] * av[2] - au[2] * av[1], au[2] * av[0] - au[0] * av[2], au[0] * av[1] - au[1] * av[0]};
  const float z = pn[0] * pn[0] + (pn[1] * pn[1] + pn[2] * pn[2]);
  if (z > 0.0f) {
    const float s = sqrtf(z);
    for (int k = 0; k < 3; ++k) pn[k] = pn[k] / s;
  }
  const float pc = pn[0] * tg->origin[0] + (pn[1] * tg->origin[1] + pn[2] * tg->origin[2]);
  const float cell_u = tg->size_u / (float)tg->bins_u, cell_v = tg->size_v / (float)tg->bins_v;
  const oplane pl = {{pn[0], pn[1], pn[2]}, pc};
  for (uint32_t r = 0; r < n; ++r) {
    if (status[r] != 2u) continue; /* RefractionResult::cOutside */
    ++*exited;
    const ov3 s = {rays_soa[r], rays_soa[(size_t)n + r], rays_soa[(size_t)2 * n + r]};
    const ov3 d = {rays_soa[(size_t)3 * n + r], rays_soa[(size_t)4 * n + r], rays_soa[(size_t)5 * n + r]};
    ov3 p;
    float cs, t;
    if (!orc_plane_intersect_ray(pl, s, d, &p, &cs, &t)) continue;
    const ov3 rel = {p.x - tg->origin[0], p.y - tg->origin[1], p.z - tg->origin[2]};
    const float a = rel.x * au[0] + (rel.y * au[1] + rel.z * au[2]);
    const float b = rel.x * av[0] + (rel.y * av[1] + rel.z * av[2]);
    if (!(a >= 0.0f && a < tg->size_u && b >= 0.0f && b < tg->size_v)) continue;
    uint32_t iu = (uint32_t)(a / cell_u), iv = (uint32_t)(b / cell_v);
    if (iu >= tg->bins_u) iu = tg->bins_u - 1u;
    if (iv >= tg->bins_v) iv = tg->bins_v - 1u;
    ++hist[(size_t)iv * tg->bins_u + iu];
    ++*landed;
  }
}
