/*
 * bzr_oracle.c -- TEST INFRASTRUCTURE ONLY (see bzr_oracle.h for the contract,
 * the pinning status and the two documented deviations D1/D2).
 *
 * Plain-C restatement of balazs-bamer/cuda-bezier-triangle-raytracer @ v1.
 * Every function cites the reference lines it restates.  Compile with
 * -O2 -ffp-contract=off (x86-64 SSE scalar maths, no FMA), which is how the
 * reference's own CMake build (-O2, reference/CMakeLists.txt:8) evaluates.
 */
#include "bzr_oracle.h"

#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static char g_err[256];

const char *orc_last_error(void) { return g_err; }
static int fail(const char *msg) { snprintf(g_err, sizeof g_err, "%s", msg); return -1; }

/* ========================================================================== *
 * Eigen surface.  The reference does all vector maths through Eigen 3.3
 * fixed-size float types (reference/3dGeomUtil.h:23-27).  The evaluation order
 * below is what Eigen produces for them with no vectorisation (size 3 is not a
 * packet multiple):
 *   redux (dot, squaredNorm, sum, mat*vec row):  a0 + (a1 + a2)
 *   normalized():  z = squaredNorm(); z > 0 ? v / sqrt(z) : v
 *   inverse():     cofactor expansion, det = c00*m00 + (c10*m10 + c20*m20),
 *                  inv(i,j) = cof(j,i) * (1/det)
 *   cross():       (a1 b2 - a2 b1, a2 b0 - a0 b2, a0 b1 - a1 b0)
 * Coefficient-wise expressions are evaluated left to right per component.
 * ========================================================================== */
static inline ov3 v3(float x, float y, float z) { ov3 r = {x, y, z}; return r; }
static inline ov3 vadd(ov3 a, ov3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline ov3 vsub(ov3 a, ov3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline ov3 vmul(ov3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
static inline ov3 vdiv(ov3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
static inline ov3 vneg(ov3 a) { return v3(-a.x, -a.y, -a.z); }
static inline float vdot(ov3 a, ov3 b) { return a.x * b.x + (a.y * b.y + a.z * b.z); }
static inline float vsq(ov3 a) { return a.x * a.x + (a.y * a.y + a.z * a.z); }
static inline float vnorm(ov3 a) { return sqrtf(vsq(a)); }
static inline ov3 vcross(ov3 a, ov3 b) {
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline ov3 vnormalized(ov3 a) {
  float z = vsq(a);
  if (z > 0.0f) { float s = sqrtf(z); return vdiv(a, s); }
  return a;
}
static inline int veq(ov3 a, ov3 b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
static inline float vget(ov3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
static inline float fmin_std(float a, float b) { return (b < a) ? b : a; }   /* std::min */
static inline float fmax_std(float a, float b) { return (a < b) ? b : a; }   /* std::max */

/* col-major m(i,j) = m[j*3+i] */
#define M(m, i, j) ((m)[(j) * 3 + (i)])
ov3 orc_matvec(const float m[9], ov3 v) {
  return v3(M(m, 0, 0) * v.x + (M(m, 0, 1) * v.y + M(m, 0, 2) * v.z),
            M(m, 1, 0) * v.x + (M(m, 1, 1) * v.y + M(m, 1, 2) * v.z),
            M(m, 2, 0) * v.x + (M(m, 2, 1) * v.y + M(m, 2, 2) * v.z));
}
static inline float cof3(const float m[9], int i, int j) {
  int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
  return M(m, i1, j1) * M(m, i2, j2) - M(m, i1, j2) * M(m, i2, j1);
}
static void inverse3(const float m[9], float r[9]) {
  float c0 = cof3(m, 0, 0), c1 = cof3(m, 1, 0), c2 = cof3(m, 2, 0);
  float det = c0 * M(m, 0, 0) + (c1 * M(m, 1, 0) + c2 * M(m, 2, 0));
  float invdet = 1.0f / det;
  M(r, 0, 0) = c0 * invdet; M(r, 0, 1) = c1 * invdet; M(r, 0, 2) = c2 * invdet;
  M(r, 1, 0) = cof3(m, 0, 1) * invdet;
  M(r, 1, 1) = cof3(m, 1, 1) * invdet;
  M(r, 2, 0) = cof3(m, 0, 2) * invdet;
  M(r, 2, 1) = cof3(m, 1, 2) * invdet;
  M(r, 1, 2) = cof3(m, 2, 1) * invdet;
  M(r, 2, 2) = cof3(m, 2, 2) * invdet;
}

/* ========================================================================== *
 * L1 geometry, reference/3dGeomUtil.h
 * ========================================================================== */
static const float kGeneralEps = 1.0e-5f;          /* cgGeneralEpsilon :20 */
static const float kRayPlaneEps = 0.00001f;        /* csRayPlaneIntersectionEpsilon :219 */

static inline ov3 tri_normal(ov3 a, ov3 b, ov3 c) { return vcross(vsub(b, a), vsub(c, a)); } /* util::getNormal :38 */

oplane orc_plane_from_1proportion_2points(float prop, ov3 p0, ov3 p1) {         /* :233-238 */
  oplane r;
  r.n = vnormalized(vsub(p1, p0));
  r.c = vdot(r.n, vadd(vmul(p1, prop), vmul(p0, 1.0f - prop)));
  return r;
}
oplane orc_plane_from_3points(ov3 p0, ov3 p1, ov3 p2) {                          /* :241-246 */
  oplane r;
  r.n = vnormalized(vcross(vsub(p1, p0), vsub(p2, p0)));
  r.c = vdot(r.n, p0);
  return r;
}
oplane orc_plane_from_1vector_2points(ov3 dir, ov3 p0, ov3 p1) {                 /* :252-257 */
  oplane r;
  r.n = vnormalized(vcross(dir, vsub(p1, p0)));
  r.c = vdot(r.n, p0);
  return r;
}
oplane orc_plane_from_2vectors_1point(ov3 d0, ov3 d1, ov3 p) {                   /* :260-265 */
  oplane r;
  r.n = vnormalized(vcross(d0, d1));
  r.c = vdot(r.n, p);
  return r;
}
ov3 orc_plane_intersect3(oplane a, oplane b, oplane c) {                         /* :268-276 */
  float m[9], inv[9];
  M(m, 0, 0) = a.n.x; M(m, 0, 1) = a.n.y; M(m, 0, 2) = a.n.z;   /* rows = normals */
  M(m, 1, 0) = b.n.x; M(m, 1, 1) = b.n.y; M(m, 1, 2) = b.n.z;
  M(m, 2, 0) = c.n.x; M(m, 2, 1) = c.n.y; M(m, 2, 2) = c.n.z;
  inverse3(m, inv);
  return orc_matvec(inv, v3(a.c, b.c, c.c));
}
/* :279-296 with deviations D1 (point written for any t) and D2 (point = start when |cos| < eps) */
int orc_plane_intersect_ray(oplane pl, ov3 start, ov3 dir, ov3 *point, float *cos_inc, float *t) {
  float cs = vdot(dir, pl.n);
  *cos_inc = cs;
  if (fabsf(cs) >= kRayPlaneEps) {
    float d = (pl.c - vdot(pl.n, start)) / cs;
    *t = d;
    *point = vadd(start, vmul(dir, d));
    return d > 0.0f;
  }
  *t = 0.0f;
  *point = start;
  return 0;
}
ov3 orc_plane_project(oplane pl, ov3 p) { return vsub(p, vmul(pl.n, vdot(p, pl.n) - pl.c)); } /* :303 */
float orc_plane_distance(oplane pl, ov3 p) { return vdot(p, pl.n) - pl.c; }                 /* :307 */
static void plane_make_distance_positive(oplane *pl, ov3 p) {                               /* :310-317 */
  if (orc_plane_distance(*pl, p) < 0.0f) { pl->n = vneg(pl->n); pl->c = -pl->c; }
}

void orc_barycentric_inverse(ov3 v0, ov3 v1, ov3 v2, float out[9]) {             /* :70-77 */
  float m[9];
  M(m, 0, 0) = v0.x; M(m, 0, 1) = v1.x; M(m, 0, 2) = v2.x;   /* columns = vertices */
  M(m, 1, 0) = v0.y; M(m, 1, 1) = v1.y; M(m, 1, 2) = v2.y;
  M(m, 2, 0) = v0.z; M(m, 2, 1) = v1.z; M(m, 2, 2) = v2.z;
  inverse3(m, out);
}

ov3 orc_get_aperpendicular(ov3 v) {                                               /* :80-95 */
  const float eps = 1e-10f;
  ov3 r; r.x = 0.0f;
  if (fabsf(v.y) < eps && fabsf(v.z) < eps) { r.y = 1.0f; r.z = 0.0f; }
  else {
    float den = sqrtf(v.y * v.y + v.z * v.z);
    r.y = -v.z / den;
    r.z = v.y / den;
  }
  return r;
}

/* util::divide (:98-122): uniform subdivision into D*D triangles, emitted in the
 * reference's order through a callback. */
typedef void (*tri_sink)(void *ctx, ov3 a, ov3 b, ov3 c);
static void util_divide(ov3 t0, ov3 t1, ov3 t2, int32_t D, tri_sink sink, void *ctx) {
  float fd = (float)D;
  ov3 v01 = vdiv(vsub(t1, t0), fd);
  ov3 v02 = vdiv(vsub(t2, t0), fd);
  ov3 line = t0;
  ov3 b0 = line;
  ov3 b1 = (D > 1) ? vadd(b0, v01) : t1;
  ov3 b2 = (D > 1) ? vadd(b0, v02) : t2;
  for (int32_t i = 0; i < D - 1; ++i) {
    for (int32_t j = 0; j < D - i - 1; ++j) {
      sink(ctx, b0, b1, b2);
      ov3 b1n = vadd(b1, v02);
      sink(ctx, b1, b1n, b2);
      b1 = b1n;
      b0 = b2;
      b2 = vadd(b2, v02);
    }
    sink(ctx, b0, b1, b2);
    line = vadd(line, v01);
    b0 = line;
    b1 = vadd(b0, v01);
    b2 = vadd(b0, v02);
  }
  sink(ctx, b0, t1, b2);
}

uint32_t orc_to_which_side(ov3 s, ov3 e) {                                        /* :137-164 */
  uint32_t result = 3u;
  float den = s.x - e.x + s.y - e.y;
  if (fabsf(den) > kGeneralEps) {
    float ratio = ((s.x - 1.0f) * e.y - s.y * (e.x - 1.0f)) / den;
    float dir = (s.x + s.y - 1.0f) / den;
    result = (ratio > -kGeneralEps && ratio < 1.0f + kGeneralEps && dir > 0.0f) ? 0u : result;
  }
  den = s.y - e.y + s.z - e.z;
  if (fabsf(den) > kGeneralEps) {
    float ratio = ((s.y - 1.0f) * e.z - s.z * (e.y - 1.0f)) / den;
    float dir = (s.y + s.z - 1.0f) / den;
    result = (ratio > -kGeneralEps && ratio < 1.0f + kGeneralEps && dir > 0.0f) ? 1u : result;
  }
  den = s.z - e.z + s.x - e.x;
  if (fabsf(den) > kGeneralEps) {
    float ratio = ((s.z - 1.0f) * e.x - s.x * (e.z - 1.0f)) / den;
    float dir = (s.z + s.x - 1.0f) / den;
    result = (ratio > -kGeneralEps && ratio < 1.0f + kGeneralEps && dir > 0.0f) ? 2u : result;
  }
  return result;
}

oray orc_ray_make(ov3 start, ov3 dir) { oray r; r.start = start; r.dir = vnormalized(dir); return r; } /* :176-178 */

static inline ov3 ray_perp(const oray *r, ov3 p) {                                /* :182-184 */
  ov3 d = vsub(p, r->start);
  return vsub(d, vmul(r->dir, vdot(d, r->dir)));
}
float orc_ray_average_error_squared(const oray *r, const ov3 *pts, uint32_t n) {  /* :199-205 */
  float sum = 0.0f;
  for (uint32_t i = 0; i < n; ++i) sum += vsq(ray_perp(r, pts[i]));
  return n == 0 ? 0.0f : sum / (float)n;
}

/* ========================================================================== *
 * Minimal containers with the iteration orders of the libstdc++ containers the
 * reference uses (all that matters for bit parity of the preprocessing):
 *   - std::unordered_map<Vertex,...>  : used only for lookups / first-seen index
 *   - std::unordered_multimap equal_range: newest element first
 *   - std::unordered_set<uint32_t> iteration: emulated (uset_*) below
 *   - std::multimap<float,...>: stable ascending order (equal keys keep insertion order)
 * ========================================================================== */
/* vertex -> index hash map (exact float equality; +0 and -0 compare equal) */
typedef struct { ov3 *key; uint32_t *val; int32_t *slot; uint32_t n, cap, nslot; } vmap;
static uint32_t vhash(ov3 v) {
  uint32_t h = 2166136261u;
  float c[3] = {v.x, v.y, v.z};
  for (int i = 0; i < 3; ++i) {
    float f = c[i] == 0.0f ? 0.0f : c[i];
    uint32_t b; memcpy(&b, &f, 4);
    h = (h ^ b) * 16777619u;
    h ^= h >> 15;
  }
  return h;
}
static int vmap_init(vmap *m, uint32_t expect) {
  m->n = 0; m->cap = expect ? expect : 16;
  m->nslot = 1; while (m->nslot < 2 * m->cap) m->nslot <<= 1;
  m->key = (ov3 *)malloc(sizeof(ov3) * m->cap);
  m->val = (uint32_t *)malloc(sizeof(uint32_t) * m->cap);
  m->slot = (int32_t *)malloc(sizeof(int32_t) * m->nslot);
  if (!m->key || !m->val || !m->slot) return -1;
  for (uint32_t i = 0; i < m->nslot; ++i) m->slot[i] = -1;
  return 0;
}
static void vmap_free(vmap *m) { free(m->key); free(m->val); free(m->slot); memset(m, 0, sizeof *m); }
static int32_t vmap_find(const vmap *m, ov3 k) {
  uint32_t mask = m->nslot - 1, s = vhash(k) & mask;
  while (m->slot[s] >= 0) {
    if (veq(m->key[m->slot[s]], k)) return m->slot[s];
    s = (s + 1) & mask;
  }
  return -1;
}
static int vmap_grow(vmap *m) {
  uint32_t ncap = m->cap * 2;
  ov3 *k = (ov3 *)realloc(m->key, sizeof(ov3) * ncap);
  if (!k) return -1;
  m->key = k;
  uint32_t *v = (uint32_t *)realloc(m->val, sizeof(uint32_t) * ncap);
  if (!v) return -1;
  m->val = v;
  m->cap = ncap;
  uint32_t ns = m->nslot * 2;
  int32_t *sl = (int32_t *)malloc(sizeof(int32_t) * ns);
  if (!sl) return -1;
  for (uint32_t i = 0; i < ns; ++i) sl[i] = -1;
  for (uint32_t e = 0; e < m->n; ++e) {
    uint32_t s = vhash(m->key[e]) & (ns - 1);
    while (sl[s] >= 0) s = (s + 1) & (ns - 1);
    sl[s] = (int32_t)e;
  }
  free(m->slot); m->slot = sl; m->nslot = ns;
  return 0;
}
/* inserts if absent; returns entry index */
static int32_t vmap_insert(vmap *m, ov3 k, uint32_t val) {
  int32_t e = vmap_find(m, k);
  if (e >= 0) return e;
  if (m->n == m->cap && vmap_grow(m)) return -1;
  uint32_t mask = m->nslot - 1, s = vhash(k) & mask;
  while (m->slot[s] >= 0) s = (s + 1) & mask;
  m->key[m->n] = k; m->val[m->n] = val; m->slot[s] = (int32_t)m->n;
  return (int32_t)m->n++;
}

/* Emulation of GCC 11 libstdc++ std::unordered_set<uint32_t> (identity hash,
 * max_load_factor 1, prime rehash policy) for its ITERATION ORDER, which the
 * reference's getInitialFaceIndex depends on for ties (reference/mesh.cpp:224-239).
 * Validated against the real container by tests/test_oracle_containers.py. */
static const uint32_t kBucketChain[] = {13u, 29u, 59u, 127u, 257u, 541u, 1109u, 2357u, 5087u,
                                        10273u, 20753u, 42043u, 85229u, 172933u, 351061u, 712697u};
typedef struct { uint32_t *key; int32_t *next; int32_t *bucket; uint32_t n, cap, nb; int32_t head; int chain; } uset;
#define USET_BB (-2)   /* bucket points at _M_before_begin */
static void uset_init(uset *s) { memset(s, 0, sizeof *s); s->nb = 1; s->head = -1; s->chain = -1; }
static void uset_free(uset *s) { free(s->key); free(s->next); free(s->bucket); memset(s, 0, sizeof *s); }
static int uset_rehash(uset *s, uint32_t nb) {
  int32_t *nbk = (int32_t *)malloc(sizeof(int32_t) * nb);
  if (!nbk) return -1;
  for (uint32_t i = 0; i < nb; ++i) nbk[i] = -1;
  int32_t p = s->head;
  s->head = -1;
  uint32_t bbegin_bkt = 0;
  while (p >= 0) {
    int32_t nxt = s->next[p];
    uint32_t b = s->key[p] % nb;
    if (nbk[b] == -1) {
      s->next[p] = s->head;
      s->head = p;
      nbk[b] = USET_BB;
      if (s->next[p] >= 0) nbk[bbegin_bkt] = p;
      bbegin_bkt = b;
    } else {
      int32_t before = nbk[b];
      int32_t *link = (before == USET_BB) ? &s->head : &s->next[before];
      s->next[p] = *link;
      *link = p;
    }
    p = nxt;
  }
  free(s->bucket);
  s->bucket = nbk;
  s->nb = nb;
  return 0;
}
static int uset_insert(uset *s, uint32_t k) {
  for (int32_t p = s->head; p >= 0; p = s->next[p]) if (s->key[p] == k) return 0;
  if (s->n + 1 > (s->chain < 0 ? 0u : s->nb)) {   /* _M_need_rehash with next_resize == n_bkt */
    s->chain++;
    if (s->chain >= (int)(sizeof kBucketChain / sizeof kBucketChain[0])) return fail("uset too large");
    if (uset_rehash(s, kBucketChain[s->chain])) return -1;
  }
  if (s->n == s->cap) {
    uint32_t nc = s->cap ? s->cap * 2 : 16;
    uint32_t *k2 = (uint32_t *)realloc(s->key, sizeof(uint32_t) * nc);
    int32_t *n2 = (int32_t *)realloc(s->next, sizeof(int32_t) * nc);
    if (!k2 || !n2) return -1;
    s->key = k2; s->next = n2; s->cap = nc;
  }
  int32_t node = (int32_t)s->n++;
  s->key[node] = k;
  uint32_t b = k % s->nb;
  if (s->bucket[b] != -1) {
    int32_t before = s->bucket[b];
    int32_t *link = (before == USET_BB) ? &s->head : &s->next[before];
    s->next[node] = *link;
    *link = node;
  } else {
    s->next[node] = s->head;
    s->head = node;
    if (s->next[node] >= 0) s->bucket[s->key[s->next[node]] % s->nb] = node;
    s->bucket[b] = USET_BB;
  }
  return 0;
}

/* exported for the container validation test */
uint32_t orc_debug_uset_order(const uint32_t *keys, uint32_t n, uint32_t *out);
uint32_t orc_debug_uset_order(const uint32_t *keys, uint32_t n, uint32_t *out) {
  uset s; uset_init(&s);
  for (uint32_t i = 0; i < n; ++i) uset_insert(&s, keys[i]);
  uint32_t c = 0;
  for (int32_t p = s.head; p >= 0; p = s.next[p]) out[c++] = s.key[p];
  uset_free(&s);
  return c;
}

/* ========================================================================== *
 * Mesh, reference/mesh.cpp
 * ========================================================================== */
void orc_mesh_init(omesh *m) { memset(m, 0, sizeof *m); }
static void mesh_clear_aux(omesh *m) {
  free(m->f2n); m->f2n = NULL; m->nf2n = 0;
  free(m->nrm_key); free(m->nrm_val); m->nrm_key = m->nrm_val = NULL; m->nnrm = 0;
}
void orc_mesh_free(omesh *m) { free(m->tri); mesh_clear_aux(m); memset(m, 0, sizeof *m); }
int orc_mesh_push(omesh *m, const otri *t) {
  if (m->n == m->cap) {
    uint32_t nc = m->cap ? m->cap * 2 : 64;
    otri *p = (otri *)realloc(m->tri, sizeof(otri) * nc);
    if (!p) return fail("out of memory");
    m->tri = p; m->cap = nc;
  }
  m->tri[m->n++] = *t;
  return 0;
}
int orc_mesh_copy(omesh *dst, const omesh *src) {
  orc_mesh_init(dst);
  for (uint32_t i = 0; i < src->n; ++i) if (orc_mesh_push(dst, &src->tri[i])) return -1;
  if (src->nf2n) {
    dst->f2n = (oneigh *)malloc(sizeof(oneigh) * src->nf2n);
    memcpy(dst->f2n, src->f2n, sizeof(oneigh) * src->nf2n);
    dst->nf2n = src->nf2n;
  }
  if (src->nnrm) {
    dst->nrm_key = (ov3 *)malloc(sizeof(ov3) * src->nnrm);
    dst->nrm_val = (ov3 *)malloc(sizeof(ov3) * src->nnrm);
    memcpy(dst->nrm_key, src->nrm_key, sizeof(ov3) * src->nnrm);
    memcpy(dst->nrm_val, src->nrm_val, sizeof(ov3) * src->nnrm);
    dst->nnrm = src->nnrm;
  }
  return 0;
}

static float envelope(int kind, float x) {
  if (kind == ORC_ENV_ELLIPSOID) return sqrtf(1.0f - x * x);           /* mesh.h:99 */
  float x2 = x * x;                                                     /* test.cpp:242-245, 336-339 */
  return sqrtf(1.0f - x2) + 0.7f * (expf(-4.0f) - expf(-4.0f * x2));
}

/* Mesh::makeSolidOfRevolution, reference/mesh.cpp:434-477 */
int orc_mesh_make_solid_of_revolution(omesh *m, int32_t sectors, int32_t belts, int env, ov3 size) {
  m->n = 0; mesh_clear_aux(m);
  const float pi = 3.14159265358979323846f;
  float half = pi / (float)sectors;
  float full = half * 2.0f;
  float belt_angle = pi / ((float)belts + 1.0f);
  float bias = 0.0f;
  float a_mid = belt_angle, a_down = 2.0f * belt_angle;
  float r_up = 0.0f;
  float r_mid = size.x * envelope(env, cosf(a_mid));
  float r_down = size.x * envelope(env, cosf(a_down));
  float z_up = size.z, z_mid = size.z * cosf(a_mid), z_down = size.z * cosf(a_down);
  for (int32_t belt = 0; belt < belts; ++belt) {
    float s_ud = bias + half, s_m1 = bias + 0.0f, s_m2 = bias + full;
    for (int32_t sector = 0; sector < sectors; ++sector) {
      ov3 c1 = v3(r_up * sinf(s_ud), size.y * r_up * cosf(s_ud), z_up);
      ov3 c2 = v3(r_mid * sinf(s_m1), size.y * r_mid * cosf(s_m1), z_mid);
      ov3 c3 = v3(r_mid * sinf(s_m2), size.y * r_mid * cosf(s_m2), z_mid);
      otri t = {{c1, c2, c3}};
      if (orc_mesh_push(m, &t)) return -1;
      c1 = v3(size.x * r_down * sinf(s_ud), size.y * r_down * cosf(s_ud), z_down);
      otri u = {{c2, c3, c1}};
      if (orc_mesh_push(m, &u)) return -1;
      s_ud += full;
      s_m1 = s_m2;
      s_m2 += full;
    }
    a_mid = a_down;
    a_down += belt_angle;
    r_up = r_mid;
    r_mid = r_down;
    r_down = size.x * envelope(env, cosf(a_down));
    z_up = z_mid;
    z_mid = z_down;
    z_down = size.z * cosf(a_down);
    bias += half;
  }
  return 0;
}
int orc_mesh_make_ellipsoid(omesh *m, int32_t sectors, int32_t belts, ov3 size) {
  return orc_mesh_make_solid_of_revolution(m, sectors, belts, ORC_ENV_ELLIPSOID, size);
}

/* Mesh::transform, reference/mesh.cpp:361-367: v = T*v + d */
void orc_mesh_transform(omesh *m, const float tr[9], ov3 disp) {
  for (uint32_t f = 0; f < m->n; ++f)
    for (int k = 0; k < 3; ++k) m->tri[f].v[k] = vadd(orc_matvec(tr, m->tri[f].v[k]), disp);
}

static void sink_push(void *ctx, ov3 a, ov3 b, ov3 c) { otri t = {{a, b, c}}; orc_mesh_push((omesh *)ctx, &t); }

/* Mesh::splitTriangles(int32_t), reference/mesh.cpp:389-395 */
int orc_mesh_split_divisor(omesh *m, int32_t divisor) {
  omesh r; orc_mesh_init(&r);
  for (uint32_t f = 0; f < m->n; ++f) util_divide(m->tri[f].v[0], m->tri[f].v[1], m->tri[f].v[2], divisor, sink_push, &r);
  free(m->tri); mesh_clear_aux(m);
  m->tri = r.tri; m->n = r.n; m->cap = r.cap;
  return 0;
}
/* Mesh::splitTriangles(float), reference/mesh.cpp:375-385 */
int orc_mesh_split_maxside(omesh *m, float max_side) {
  omesh r; orc_mesh_init(&r);
  for (uint32_t f = 0; f < m->n; ++f) {
    const otri *t = &m->tri[f];
    float s = vnorm(vsub(t->v[0], t->v[1]));
    s = fmax_std(s, vnorm(vsub(t->v[0], t->v[2])));
    s = fmax_std(s, vnorm(vsub(t->v[1], t->v[2])));
    int32_t d = (int32_t)ceilf(s / max_side);
    util_divide(t->v[0], t->v[1], t->v[2], d, sink_push, &r);
  }
  free(m->tri); mesh_clear_aux(m);
  m->tri = r.tri; m->n = r.n; m->cap = r.cap;
  return 0;
}

/* ---- standardizeVertices, reference/mesh.cpp:4-91 ---- */
typedef struct { float key; uint32_t seq; uint32_t face; uint32_t vtx; } proj_e;
static int proj_cmp(const void *a, const void *b) {
  const proj_e *x = (const proj_e *)a, *y = (const proj_e *)b;
  if (x->key < y->key) return -1;
  if (y->key < x->key) return 1;
  return x->seq < y->seq ? -1 : (x->seq > y->seq);
}
static float get_smallest_side(const omesh *m) {                                 /* :4-12 */
  float s = FLT_MAX;
  for (uint32_t f = 0; f < m->n; ++f)
    for (int i = 0; i < 3; ++i) s = fmin_std(s, vnorm(vsub(m->tri[f].v[i], m->tri[f].v[(i + 1) % 3])));
  return s;
}
int orc_mesh_standardize_vertices(omesh *m) {
  if (m->n == 0) return 0;
  float eps = get_smallest_side(m) * 0.2f;
  uint32_t nv = m->n * 3;
  proj_e *proj[3];
  uint32_t *ibeg[3], nint[3], maxima[3];
  for (int d = 0; d < 3; ++d) {
    proj[d] = (proj_e *)malloc(sizeof(proj_e) * nv);
    ibeg[d] = (uint32_t *)malloc(sizeof(uint32_t) * (nv + 1));
    for (uint32_t f = 0, s = 0; f < m->n; ++f)                                   /* projectVertices :14-22 */
      for (uint32_t k = 0; k < 3; ++k, ++s) {
        proj_e e = {vget(m->tri[f].v[k], d), s, f, k};
        proj[d][s] = e;
      }
    qsort(proj[d], nv, sizeof(proj_e), proj_cmp);
    /* makeProximityIntervals :24-54 */
    uint32_t mx = 0, counter = 0, start = 0, ni = 0;
    float sv = 0.0f;
    for (uint32_t i = 0; i < nv; ++i) {
      if (i > 0) {
        float now = proj[d][i].key;
        if (now - sv >= eps) {
          ibeg[d][ni++] = start;
          sv = now; start = i;
          mx = mx > counter ? mx : counter;
          counter = 1;
        } else {
          ++counter;
        }
      } else {
        start = 0; sv = proj[d][0].key; counter = 1;
      }
    }
    ibeg[d][ni++] = start;
    mx = mx > counter ? mx : counter;
    ibeg[d][ni] = nv;
    nint[d] = ni;
    maxima[d] = mx;
  }
  int best = 0;                                                                   /* std::min_element :85 */
  for (int d = 1; d < 3; ++d) if (maxima[d] < maxima[best]) best = d;
  float eps2 = eps * eps;
  for (uint32_t it = 0; it < nint[best]; ++it) {                                  /* standardizeInIntervals :56-70 */
    uint32_t b = ibeg[best][it], e = ibeg[best][it + 1];
    for (uint32_t i = b; i < e; ++i) {
      ov3 *v1 = &m->tri[proj[best][i].face].v[proj[best][i].vtx];
      for (uint32_t j = b; j < e; ++j) {
        ov3 *v2 = &m->tri[proj[best][j].face].v[proj[best][j].vtx];
        if (vsq(vsub(*v1, *v2)) < eps2 &&
            (v1->x < v2->x || (v1->x == v2->x && v1->y < v2->y) || (v1->x == v2->x && v1->y == v2->y && v1->z < v2->z)))
          *v1 = *v2;
      }
    }
  }
  for (int d = 0; d < 3; ++d) { free(proj[d]); free(ibeg[d]); }
  return 0;
}

uint32_t orc_mesh_unique_vertices(const omesh *m, ov3 *out) {                    /* getVertices :95-103 */
  vmap vm;
  if (vmap_init(&vm, m->n * 3 + 16)) return 0;
  for (uint32_t f = 0; f < m->n; ++f)
    for (int k = 0; k < 3; ++k) vmap_insert(&vm, m->tri[f].v[k], 0);
  uint32_t n = vm.n;
  if (out) memcpy(out, vm.key, sizeof(ov3) * n);
  vmap_free(&vm);
  return n;
}

/* ---- standardizeNormals, reference/mesh.cpp:107-357 ---- */
typedef struct {
  uint32_t (*fv)[3];      /* face2vertex */
  vmap vidx;              /* vertex -> index */
  /* edge -> faces, stored sorted by (lo, hi, insertion seq) */
  struct edge_e { uint32_t lo, hi, seq, face; } *edges;
  uint32_t nedges;
} topo;
static int edge_cmp(const void *a, const void *b) {
  const struct edge_e *x = (const struct edge_e *)a, *y = (const struct edge_e *)b;
  if (x->lo != y->lo) return x->lo < y->lo ? -1 : 1;
  if (x->hi != y->hi) return x->hi < y->hi ? -1 : 1;
  return x->seq < y->seq ? -1 : (x->seq > y->seq);
}
static int topo_build(const omesh *m, topo *t) {                                  /* createEdge2faceFace2vertex :118-153 */
  memset(t, 0, sizeof *t);
  t->fv = (uint32_t(*)[3])malloc(sizeof(uint32_t[3]) * (m->n ? m->n : 1));
  t->edges = (struct edge_e *)malloc(sizeof(struct edge_e) * (3 * m->n + 1));
  if (!t->fv || !t->edges || vmap_init(&t->vidx, m->n * 3 + 16)) return fail("out of memory");
  for (uint32_t f = 0; f < m->n; ++f) {
    for (int k = 0; k < 3; ++k) {
      int32_t e = vmap_insert(&t->vidx, m->tri[f].v[k], t->vidx.n);
      t->fv[f][k] = t->vidx.val[e];
    }
    for (int i = 0; i < 3; ++i) {
      uint32_t lo = t->fv[f][i], hi = t->fv[f][(i + 1) % 3];
      if (lo > hi) { uint32_t s = lo; lo = hi; hi = s; }
      struct edge_e ee = {lo, hi, t->nedges, f};
      t->edges[t->nedges++] = ee;
    }
  }
  qsort(t->edges, t->nedges, sizeof(struct edge_e), edge_cmp);
  return 0;
}
static void topo_free(topo *t) { free(t->fv); free(t->edges); vmap_free(&t->vidx); }
/* std::unordered_multimap::equal_range gives the newest element first; the
 * reference takes the first element that is not indexFace (skipping only a
 * leading indexFace).  Returns -1 on "Vertex on edge detected." */
static int64_t edge_other(const topo *t, uint32_t lo, uint32_t hi, uint32_t face) {
  uint32_t a = 0, b = t->nedges;
  while (a < b) {   /* lower bound of (lo,hi) */
    uint32_t mid = (a + b) / 2;
    const struct edge_e *e = &t->edges[mid];
    if (e->lo < lo || (e->lo == lo && e->hi < hi)) a = mid + 1; else b = mid;
  }
  uint32_t first = a, last = a;
  while (last < t->nedges && t->edges[last].lo == lo && t->edges[last].hi == hi) ++last;
  if (last == first) return -1;
  /* equal_range order = reverse insertion order: edges[last-1], edges[last-2], ... */
  int64_t idx = (int64_t)last - 1;
  if (t->edges[idx].face == face) {
    --idx;
    if (idx < (int64_t)first) return -1;
  }
  return t->edges[idx].face;
}
static int create_face2neighbour(omesh *m, const topo *t) {                       /* :185-222 */
  free(m->f2n);
  m->f2n = (oneigh *)malloc(sizeof(oneigh) * (m->n ? m->n : 1));
  m->nf2n = m->n;
  static const uint8_t resolve[3][3] = {{3, 0, 2}, {0, 3, 1}, {2, 1, 3}};
  for (uint32_t f = 0; f < m->n; ++f) {
    for (int k = 0; k < 3; ++k) {
      uint32_t a = t->fv[f][k], b = t->fv[f][(k + 1) % 3];
      uint32_t lo = a < b ? a : b, hi = a < b ? b : a;
      int64_t other = edge_other(t, lo, hi, f);
      if (other < 0) return fail("Vertex on edge detected.");
      m->f2n[f].fellow[k] = (uint32_t)other;
      int ia = 3, ib = 3;
      for (int q = 2; q >= 0; --q) { if (t->fv[other][q] == a) ia = q; if (t->fv[other][q] == b) ib = q; }
      m->f2n[f].start[k] = (ia < 3 && ib < 3) ? resolve[ia][ib] : 3;
    }
  }
  return 0;
}
static inline ov3 get_altitude(ov3 c1, ov3 c2, ov3 ind) {                         /* 3dGeomUtil.h:125-130 */
  ov3 cv = vsub(c2, c1), iv = vsub(ind, c1);
  float foot = vdot(cv, iv) / vsq(cv);
  return vsub(iv, vmul(cv, foot));
}
static uint32_t independent_from(const otri *target, const otri *other) {        /* :107-116 */
  for (uint32_t i = 0; i < 3; ++i)
    if (!veq(other->v[0], target->v[i]) && !veq(other->v[1], target->v[i]) && !veq(other->v[2], target->v[i])) return i;
  return 3u;
}
static void normalize_desired(otri *f, ov3 desired) {                             /* :241-248 */
  ov3 n = tri_normal(f->v[0], f->v[1], f->v[2]);
  if (vdot(desired, n) < 0.0f) { ov3 s = f->v[0]; f->v[0] = f->v[1]; f->v[1] = s; }
}
static void normalize_pair(const otri *kn, otri *un) {                            /* :250-282 */
  uint32_t ik = independent_from(kn, un), c1k = (ik + 1) % 3, c2k = (ik + 2) % 3;
  uint32_t iu = independent_from(un, kn), c1u = (iu + 1) % 3, c2u = (iu + 2) % 3;
  if (ik > 2 || iu > 2) return;   /* reference indexes out of bounds here (identical faces); unreachable on valid meshes */
  ov3 alt_k = get_altitude(kn->v[c1k], kn->v[c2k], kn->v[ik]);
  ov3 alt_u = get_altitude(un->v[c1u], un->v[c2u], un->v[iu]);
  float dot_alt = vdot(alt_k, alt_u);
  ov3 nk = tri_normal(kn->v[0], kn->v[1], kn->v[2]);
  ov3 nu = tri_normal(un->v[0], un->v[1], un->v[2]);
  float kdu = vdot(nk, nu);
  if (fabsf(kdu / (vnorm(nk) * vnorm(nu))) < 0.01f) {
    ov3 ni = vadd(un->v[iu], vmul(vsub(kn->v[ik], vdiv(vadd(kn->v[c1k], kn->v[c2k]), 2.0f)), 0.2f));
    otri nf = *un;
    nf.v[iu] = ni;
    alt_u = get_altitude(un->v[c1u], un->v[c2u], ni);
    dot_alt = vdot(alt_k, alt_u);
    nu = tri_normal(nf.v[0], nf.v[1], nf.v[2]);
    kdu = vdot(nk, nu);
  }
  if (dot_alt * kdu > 0.0f) { ov3 s = un->v[c1u]; un->v[c1u] = un->v[c2u]; un->v[c2u] = s; }
}
static int calc_normal_averages(omesh *m) {                                       /* :284-308 */
  vmap vm;
  if (vmap_init(&vm, m->n * 3 + 16)) return fail("out of memory");
  /* per unique vertex: list of (triangle) in insertion order -> iterate newest first */
  uint32_t nv3 = m->n * 3;
  uint32_t *cnt = NULL, *startv = NULL, *list = NULL, *vid = (uint32_t *)malloc(sizeof(uint32_t) * (nv3 + 1));
  for (uint32_t f = 0; f < m->n; ++f)
    for (int k = 0; k < 3; ++k) {
      int32_t e = vmap_insert(&vm, m->tri[f].v[k], 0);
      vid[f * 3 + k] = (uint32_t)e;
    }
  cnt = (uint32_t *)calloc(vm.n + 1, sizeof(uint32_t));
  startv = (uint32_t *)calloc(vm.n + 1, sizeof(uint32_t));
  list = (uint32_t *)malloc(sizeof(uint32_t) * (nv3 + 1));
  for (uint32_t i = 0; i < nv3; ++i) cnt[vid[i]]++;
  for (uint32_t v = 0; v < vm.n; ++v) startv[v + 1] = startv[v] + cnt[v];
  memset(cnt, 0, sizeof(uint32_t) * (vm.n + 1));
  for (uint32_t i = 0; i < nv3; ++i) list[startv[vid[i]] + cnt[vid[i]]++] = i / 3;
  free(m->nrm_key); free(m->nrm_val);
  m->nrm_key = (ov3 *)malloc(sizeof(ov3) * (vm.n + 1));
  m->nrm_val = (ov3 *)malloc(sizeof(ov3) * (vm.n + 1));
  m->nnrm = vm.n;
  for (uint32_t v = 0; v < vm.n; ++v) {
    ov3 vert = vm.key[v];
    ov3 sum = v3(0.0f, 0.0f, 0.0f);
    for (int64_t q = (int64_t)startv[v + 1] - 1; q >= (int64_t)startv[v]; --q) {   /* newest first */
      const otri *t = &m->tri[list[q]];
      uint32_t w = 0;
      while (w < 3 && !veq(t->v[w], vert)) ++w;
      ov3 sa = vsub(t->v[(w + 1) % 3], t->v[w]);
      ov3 sb = vsub(t->v[(w + 2) % 3], t->v[w]);
      float ca = vdot(sa, sb) / (vnorm(sa) * vnorm(sb));
      sum = vadd(sum, vmul(vnormalized(tri_normal(t->v[0], t->v[1], t->v[2])), acosf(ca)));
    }
    float z = vsq(sum);                              /* Vector::normalize() */
    if (z > 0.0f) sum = vdiv(sum, sqrtf(z));
    m->nrm_key[v] = vert;
    m->nrm_val[v] = sum;
  }
  free(cnt); free(startv); free(list); free(vid);
  vmap_free(&vm);
  return 0;
}
int orc_mesh_standardize_normals(omesh *m) {                                      /* :310-357 */
  if (m->n == 0) return 0;
  topo t;
  if (topo_build(m, &t)) return -1;
  /* getSmallestXstuff :155-183 */
  float sx = FLT_MAX;
  uint32_t sidx = 0;
  for (uint32_t f = 0; f < m->n; ++f)
    for (int k = 0; k < 3; ++k)
      if (m->tri[f].v[k].x < sx) { sx = m->tri[f].v[k].x; sidx = t.fv[f][k]; }
  uset faces; uset_init(&faces);
  for (uint32_t f = 0; f < m->n; ++f)
    for (int k = 0; k < 3; ++k)
      if (t.fv[f][k] == sidx) uset_insert(&faces, f);
  if (create_face2neighbour(m, &t)) { topo_free(&t); uset_free(&faces); return -1; }
  ov3 desired = v3(-1.0f, 0.0f, 0.0f);
  /* getInitialFaceIndex :224-239 (iterates the unordered_set) */
  float best = -FLT_MAX;
  uint32_t init = 0;
  for (int32_t p = faces.head; p >= 0; p = faces.next[p]) {
    uint32_t f = faces.key[p];
    ov3 n = vnormalized(tri_normal(m->tri[f].v[0], m->tri[f].v[1], m->tri[f].v[2]));
    float a = fabsf(vdot(desired, n));
    if (a > best) { best = a; init = f; }
  }
  uset_free(&faces);
  normalize_desired(&m->tri[init], desired);
  /* flood fill with a LIFO (std::list used via emplace_back/back/pop_back) */
  uint8_t *remaining = (uint8_t *)malloc(m->n);
  memset(remaining, 1, m->n);
  uint32_t cap = 1024, top = 0;
  uint32_t (*stk)[2] = (uint32_t(*)[2])malloc(sizeof(uint32_t[2]) * cap);
  for (int k = 0; k < 3; ++k) { stk[top][0] = init; stk[top][1] = m->f2n[init].fellow[k]; ++top; }
  remaining[init] = 0;
  while (top > 0) {
    --top;
    uint32_t kn = stk[top][0], un = stk[top][1];
    if (remaining[un]) normalize_pair(&m->tri[kn], &m->tri[un]);
    remaining[un] = 0;
    for (int k = 0; k < 3; ++k) {
      uint32_t f = m->f2n[un].fellow[k];
      if (remaining[f] && un != f) {
        if (top == cap) { cap *= 2; stk = (uint32_t(*)[2])realloc(stk, sizeof(uint32_t[2]) * cap); }
        stk[top][0] = un; stk[top][1] = f; ++top;
      }
    }
  }
  free(stk); free(remaining);
  topo_free(&t);
  if (topo_build(m, &t)) return -1;
  int rc = create_face2neighbour(m, &t);
  topo_free(&t);
  if (rc) return -1;
  return calc_normal_averages(m);
}

/* ---- STL I/O (reference/mesh.cpp:399-430 + the stl_reader submodule's file format) ---- */
int orc_mesh_read_stl(omesh *m, const char *path) {
  FILE *fp = fopen(path, "rb");
  if (!fp) return fail("cannot open STL file");
  fseek(fp, 0, SEEK_END);
  long sz = ftell(fp);
  fseek(fp, 0, SEEK_SET);
  unsigned char *buf = (unsigned char *)malloc((size_t)sz + 1);
  if (!buf || fread(buf, 1, (size_t)sz, fp) != (size_t)sz) { fclose(fp); free(buf); return fail("read error"); }
  fclose(fp);
  buf[sz] = 0;
  m->n = 0; mesh_clear_aux(m);
  uint32_t nt = 0;
  if (sz >= 84) memcpy(&nt, buf + 80, 4);
  if (sz >= 84 && (long)(84 + 50ull * nt) == sz) {        /* binary */
    for (uint32_t i = 0; i < nt; ++i) {
      const unsigned char *p = buf + 84 + 50ull * i + 12;
      float c[9]; memcpy(c, p, 36);
      otri t = {{v3(c[0], c[1], c[2]), v3(c[3], c[4], c[5]), v3(c[6], c[7], c[8])}};
      if (orc_mesh_push(m, &t)) { free(buf); return -1; }
    }
  } else {                                                 /* ASCII */
    char *s = (char *)buf;
    ov3 vs[3]; int k = 0;
    while ((s = strstr(s, "vertex")) != NULL) {
      s += 6;
      char *e;
      float x = strtof(s, &e); s = e;
      float y = strtof(s, &e); s = e;
      float z = strtof(s, &e); s = e;
      vs[k++] = v3(x, y, z);
      if (k == 3) { otri t = {{vs[0], vs[1], vs[2]}}; if (orc_mesh_push(m, &t)) { free(buf); return -1; } k = 0; }
    }
  }
  free(buf);
  return 0;
}
int orc_mesh_write_stl(const omesh *m, const char *path) {                       /* :419-430, %g == ostream default */
  FILE *fp = fopen(path, "w");
  if (!fp) return fail("cannot open output");
  fprintf(fp, "solid Exported from Blender-2.82 (sub 7)\n");
  for (uint32_t f = 0; f < m->n; ++f) {
    fprintf(fp, "facet normal 0.000000 0.000000 0.000000\nouter loop\n");
    for (int k = 0; k < 3; ++k) fprintf(fp, "vertex %g %g %g\n", m->tri[f].v[k].x, m->tri[f].v[k].y, m->tri[f].v[k].z);
    fprintf(fp, "endloop\nendfacet\n");
  }
  fprintf(fp, "endsolid Exported from Blender-2.82 (sub 7)\n");
  fclose(fp);
  return 0;
}

/* ========================================================================== *
 * BezierTriangle, reference/bezierTriangle.cpp
 * ========================================================================== */
enum { CP300 = 0, CP030 = 1, CP003 = 2, CP210 = 3, CP120 = 4, CP021 = 5, CP012 = 6, CP102 = 7, CP201 = 8, CP111 = 9 };

/* interpolate, :105-121 */
ov3 orc_patch_interpolate(const opatch *p, float b0, float b1, float b2) {
  float q0 = b0 * b0, q1 = b1 * b1, q2 = b2 * b2;
  const ov3 *c = p->cp;
  ov3 r;
  /* A + B + C + 3*(D + E + F + G + H + I) + J, left-associative, per component */
  for (int i = 0; i < 3; ++i) {
    float c0 = vget(c[0], i), c1 = vget(c[1], i), c2 = vget(c[2], i), c3 = vget(c[3], i), c4 = vget(c[4], i);
    float c5 = vget(c[5], i), c6 = vget(c[6], i), c7 = vget(c[7], i), c8 = vget(c[8], i), c9 = vget(c[9], i);
    float lin = ((c0 * b0) * q0 + (c1 * b1) * q1) + (c2 * b2) * q2;
    float side = (((((c3 * b1) * q0 + (c4 * b0) * q1) + (c5 * b2) * q1) + (c6 * b1) * q2) + (c7 * b0) * q2) + (c8 * b2) * q0;
    float v = (lin + 3.0f * side) + (((c9 * b0) * b1) * b2) * 6.0f;
    if (i == 0) r.x = v; else if (i == 1) r.y = v; else r.z = v;
  }
  return r;
}
static ov3 patch_interpolate_linear(const opatch *p, float b0, float b1, float b2) { /* :99-103 */
  return vadd(vadd(vmul(p->cp[0], b0), vmul(p->cp[1], b1)), vmul(p->cp[2], b2));
}

/* getNormal, :197-233 */
ov3 orc_patch_normal(const opatch *p, ov3 b) {
  float q0 = b.x * b.x, q1 = b.y * b.y, q2 = b.z * b.z;
  const ov3 *c = p->cp;
  float comp[3][3];
  for (int i = 0; i < 3; ++i) {
    float k0 = ((vget(c[CP300], i) * q0 + vget(c[CP102], i) * q2) + vget(c[CP120], i) * q1) +
               2.0f * (((vget(c[CP201], i) * b.x) * b.z + (vget(c[CP210], i) * b.x) * b.y) + (vget(c[CP111], i) * b.z) * b.y);
    float k1 = ((vget(c[CP030], i) * q1 + vget(c[CP012], i) * q2) + vget(c[CP210], i) * q0) +
               2.0f * (((vget(c[CP111], i) * b.x) * b.z + (vget(c[CP120], i) * b.x) * b.y) + (vget(c[CP021], i) * b.y) * b.z);
    float k2 = ((vget(c[CP003], i) * q2 + vget(c[CP201], i) * q0) + vget(c[CP021], i) * q1) +
               2.0f * (((vget(c[CP102], i) * b.x) * b.z + (vget(c[CP012], i) * b.y) * b.z) + (vget(c[CP111], i) * b.x) * b.y);
    comp[0][i] = k0; comp[1][i] = k1; comp[2][i] = k2;
  }
  ov3 ca, cb;
  ca.x = (p->dir_a.x * comp[0][0] + p->dir_a.y * comp[1][0]) + p->dir_a.z * comp[2][0];
  ca.y = (p->dir_a.x * comp[0][1] + p->dir_a.y * comp[1][1]) + p->dir_a.z * comp[2][1];
  ca.z = (p->dir_a.x * comp[0][2] + p->dir_a.y * comp[1][2]) + p->dir_a.z * comp[2][2];
  cb.x = (p->dir_b.x * comp[0][0] + p->dir_b.y * comp[1][0]) + p->dir_b.z * comp[2][0];
  cb.y = (p->dir_b.x * comp[0][1] + p->dir_b.y * comp[1][1]) + p->dir_b.z * comp[2][1];
  cb.z = (p->dir_b.x * comp[0][2] + p->dir_b.y * comp[1][2]) + p->dir_b.z * comp[2][2];
  return vnormalized(vcross(ca, cb));
}

/* constructor, :4-43 */
static void patch_construct(opatch *p, ov3 v0, ov3 v1, ov3 centroid, ov3 avg0, ov3 avg1, oplane between,
                            const uint32_t neigh[3]) {
  memset(p, 0, sizeof *p);
  memcpy(p->neigh, neigh, sizeof p->neigh);
  p->cp[CP300] = v0;
  p->cp[CP030] = v1;
  oplane common0 = {avg0, vdot(v0, avg0)};
  oplane common1 = {avg1, vdot(v1, avg1)};
  oplane perp0 = orc_plane_from_1proportion_2points(0.291f, v0, v1);
  oplane perp1 = orc_plane_from_1proportion_2points(0.291f, v1, v0);
  p->cp[CP210] = orc_plane_intersect3(common0, between, perp0);
  p->cp[CP120] = orc_plane_intersect3(common1, between, perp1);
  ov3 on = tri_normal(v0, v1, centroid);
  oplane par0 = orc_plane_from_1vector_2points(on, v0, centroid);
  oplane par1 = orc_plane_from_1vector_2points(on, v1, centroid);
  oplane ps0 = orc_plane_from_1proportion_2points(0.304f, v0, centroid);
  oplane ps1 = orc_plane_from_1proportion_2points(0.304f, v1, centroid);
  p->cp[CP201] = orc_plane_intersect3(common0, par0, ps0);
  p->cp[CP021] = orc_plane_intersect3(common1, par1, ps1);
  oplane perp_between = orc_plane_from_1vector_2points(between.n, p->cp[CP210], p->cp[CP120]);
  oplane half = orc_plane_from_1proportion_2points(0.5f, p->cp[CP210], p->cp[CP120]);
  oplane perp_median = orc_plane_from_1proportion_2points(0.2f, vdiv(vadd(v0, v1), 2.0f), centroid);
  p->cp[CP111] = orc_plane_intersect3(perp_between, half, perp_median);
  p->divider[0] = between;
  plane_make_distance_positive(&p->divider[0], p->cp[CP111]);
}
/* setMissingFields1, :45-60 */
static void patch_fields1(opatch *p, ov3 centroid, const opatch *next, const opatch *prev) {
  ov3 on = tri_normal(p->cp[CP300], p->cp[CP030], centroid);
  oplane two0 = orc_plane_from_3points(p->cp[CP201], p->cp[CP111], prev->cp[CP111]);
  oplane two1 = orc_plane_from_3points(p->cp[CP021], next->cp[CP111], p->cp[CP111]);
  oplane par0 = orc_plane_from_1vector_2points(on, p->cp[CP300], centroid);
  oplane par1 = orc_plane_from_1vector_2points(on, p->cp[CP030], centroid);
  oplane ps0 = orc_plane_from_1proportion_2points(0.304f, centroid, p->cp[CP300]);
  oplane ps1 = orc_plane_from_1proportion_2points(0.304f, centroid, p->cp[CP030]);
  p->cp[CP102] = orc_plane_intersect3(two0, par0, ps0);
  p->cp[CP012] = orc_plane_intersect3(two1, par1, ps1);
}
typedef struct { opatch *p; float hin, hout; } height_ctx;
static void height_sink(void *vctx, ov3 a, ov3 b, ov3 c) {
  height_ctx *h = (height_ctx *)vctx;
  ov3 bs[3] = {a, b, c};
  for (int i = 0; i < 3; ++i) {
    float d = orc_plane_distance(h->p->under, orc_patch_interpolate(h->p, bs[i].x, bs[i].y, bs[i].z));
    h->hin = fmin_std(h->hin, d);
    h->hout = fmax_std(h->hout, d);
  }
}
/* setMissingFields2, :62-86 */
static void patch_fields2(opatch *p, const opatch *next) {
  p->cp[CP003] = vdiv(vadd(vadd(p->cp[CP102], p->cp[CP012]), next->cp[CP012]), 3.0f);
  p->under = orc_plane_from_3points(p->cp[CP300], p->cp[CP030], p->cp[CP003]);
  orc_barycentric_inverse(p->cp[CP300], p->cp[CP030], p->cp[CP003], p->minv);
  height_ctx h = {p, 0.0f, 0.0f};
  util_divide(v3(1.0f, 0.0f, 0.0f), v3(0.0f, 1.0f, 0.0f), v3(0.0f, 0.0f, 1.0f), 5, height_sink, &h);
  p->h_in = h.hin * 1.33333333f;
  p->h_out = h.hout * 1.33333333f;
  p->dir_a = v3(1.0f, 0.0f, -1.0f);
  p->dir_b = orc_matvec(p->minv, vcross(vsub(p->cp[CP003], p->cp[CP300]), p->under.n));
}
/* setMissingFields3, :88-97 */
static void patch_fields3(opatch *p, const opatch *next, const opatch *prev) {
  p->divider[1] = orc_plane_from_1vector_2points(vadd(p->under.n, next->under.n), p->cp[CP030], p->cp[CP003]);
  p->divider[2] = orc_plane_from_1vector_2points(vadd(p->under.n, prev->under.n), p->cp[CP300], p->cp[CP003]);
  plane_make_distance_positive(&p->divider[1], p->cp[CP111]);
  plane_make_distance_positive(&p->divider[2], p->cp[CP111]);
}

/* ========================================================================== *
 * BezierMesh, reference/bezierMesh.cpp
 * ========================================================================== */
static int32_t normal_lookup(const omesh *m, const vmap *vm, ov3 v) {
  int32_t e = vmap_find(vm, v);
  (void)m;
  return e;
}
/* ctor :4-34 + setMissingFields :36-51 */
int orc_bezier_build(const omesh *m, opatch *out) {
  if (m->nf2n != m->n) return fail("mesh not standardized (no face neighbours)");
  vmap vm;
  if (vmap_init(&vm, m->nnrm + 16)) return fail("out of memory");
  for (uint32_t i = 0; i < m->nnrm; ++i) vmap_insert(&vm, m->nrm_key[i], i);
  for (uint32_t f = 0; f < m->n; ++f) {
    const oneigh *ng = &m->f2n[f];
    const otri *t = &m->tri[f];
    ov3 centroid = vdiv(vadd(vadd(t->v[0], t->v[1]), t->v[2]), 3.0f);
    ov3 normal = vnormalized(tri_normal(t->v[0], t->v[1], t->v[2]));
    for (uint32_t k = 0; k < 3; ++k) {
      ov3 a = t->v[k], b = t->v[(k + 1) % 3];
      int32_t ea = normal_lookup(m, &vm, a), eb = normal_lookup(m, &vm, b);
      if (ea < 0 || eb < 0) { vmap_free(&vm); return fail("std::out_of_range: vertex normal missing"); }
      const otri *nt = &m->tri[ng->fellow[k]];
      oplane between = orc_plane_from_1vector_2points(vadd(normal, vnormalized(tri_normal(nt->v[0], nt->v[1], nt->v[2]))), a, b);
      uint32_t base = f * 3u;
      uint32_t nn[3] = {3u * ng->fellow[k] + ng->start[k], base + (k + 1u) % 3u, base + (k + 2u) % 3u};
      patch_construct(&out[base + k], a, b, centroid, m->nrm_val[vm.val[ea]], m->nrm_val[vm.val[eb]], between, nn);
    }
  }
  vmap_free(&vm);
  uint32_t np = m->n * 3;
  for (int pass = 1; pass <= 3; ++pass) {
    ov3 centroid = v3(0, 0, 0);
    for (uint32_t i = 0; i < np; ++i) {
      uint32_t sub = i % 3u, base = i - sub;
      const opatch *next = &out[base + (sub + 1u) % 3u];
      const opatch *prev = &out[base + (sub + 2u) % 3u];
      if (sub == 0) {
        const otri *t = &m->tri[base / 3u];
        centroid = vdiv(vadd(vadd(t->v[0], t->v[1]), t->v[2]), 3.0f);
      }
      if (pass == 1) patch_fields1(&out[i], centroid, next, prev);
      else if (pass == 2) patch_fields2(&out[i], next);
      else patch_fields3(&out[i], next, prev);
    }
  }
  return 0;
}

typedef struct { const opatch *p; uint32_t np; omesh *out; } interp_ctx;
static void interp_sink(void *vctx, ov3 a, ov3 b, ov3 c) {                         /* :55-66 */
  interp_ctx *x = (interp_ctx *)vctx;
  for (uint32_t i = 0; i < x->np; ++i) {
    const opatch *p = &x->p[i];
    otri t = {{orc_patch_interpolate(p, a.x, a.y, a.z), orc_patch_interpolate(p, b.x, b.y, b.z),
               orc_patch_interpolate(p, c.x, c.y, c.z)}};
    orc_mesh_push(x->out, &t);
  }
}
int orc_bezier_interpolate_mesh(const opatch *p, uint32_t np, int32_t divisor, omesh *out) {
  orc_mesh_init(out);
  interp_ctx x = {p, np, out};
  util_divide(v3(1.0f, 0.0f, 0.0f), v3(0.0f, 1.0f, 0.0f), v3(0.0f, 0.0f, 1.0f), divisor, interp_sink, &x);
  return 0;
}

/* BezierMesh::interpolate(index, b0, b1, b2), :200-204 */
static ov3 split_point(const opatch *p, float b0, float b1, float b2) {
  const float f = 0.7f;
  return vadd(vmul(orc_patch_interpolate(p, b0, b1, b2), f), vmul(patch_interpolate_linear(p, b0, b1, b2), 1.0f - f));
}
static float perimeter(const otri *t) {                                           /* 3dGeomUtil.h:43-45 */
  return (vnorm(vsub(t->v[0], t->v[1])) + vnorm(vsub(t->v[1], t->v[2]))) + vnorm(vsub(t->v[2], t->v[0]));
}
static void push3(omesh *m, ov3 a, ov3 b, ov3 c) { otri t = {{a, b, c}}; orc_mesh_push(m, &t); }
/* splitThickBezierTriangles :79-134 and append{2,3,4}split :144-198 */
int orc_bezier_split_thick(const opatch *p, uint32_t np, const omesh *orig, omesh *out) {
  static const uint8_t mask[3] = {1, 2, 4};
  static const uint8_t count[8] = {1, 2, 2, 3, 2, 3, 3, 4};
  static const float ratios[3] = {0.25f, 0.5f, 0.75f};
  uint32_t no = np / 3u;
  if (orig->nf2n != no) return fail("neighbour table size mismatch");
  uint8_t *split = (uint8_t *)calloc(no + 1, 1);
  for (uint32_t o = 0; o < no; ++o) {
    uint32_t s = o * 3u;
    otri t = {{p[s].cp[0], p[s + 1].cp[0], p[s + 2].cp[0]}};
    oplane pl = orc_plane_from_3points(t.v[0], t.v[1], t.v[2]);
    float mx = fabsf(orc_plane_distance(pl, p[o * 3u].cp[CP003]));
    for (uint32_t i = 0; i < 3u; ++i)
      for (int r = 0; r < 3; ++r)
        mx = fmax_std(mx, fabsf(orc_plane_distance(pl, orc_patch_interpolate(&p[s + i], ratios[r], 1.0f - ratios[r], 0.0f))));
    if (mx / perimeter(&t) > 0.03f) {
      split[o] = 7;
      for (int side = 0; side < 3; ++side) split[orig->f2n[o].fellow[side]] |= mask[orig->f2n[o].start[side]];
    }
  }
  orc_mesh_init(out);
  for (uint32_t o = 0; o < no; ++o) {
    uint32_t base = o * 3u;
    otri t = {{p[base].cp[0], p[base + 1].cp[0], p[base + 2].cp[0]}};
    uint8_t sp = split[o];
    uint32_t c = count[sp];
    if (c == 1) {
      orc_mesh_push(out, &t);
    } else if (c == 2) {
      static const uint8_t idx2[8] = {3, 0, 1, 3, 2, 3, 3, 3};
      uint32_t i2 = idx2[sp], ia = (i2 + 1) % 3, ib = (i2 + 2) % 3;
      ov3 sv = split_point(&p[base + i2], 0.5f, 0.5f, 0.0f);
      push3(out, t.v[ia], t.v[ib], sv);
      push3(out, t.v[ib], t.v[i2], sv);
    } else if (c == 3) {
      static const uint8_t idx1[8] = {3, 3, 3, 2, 3, 1, 0, 3};
      uint32_t i1 = idx1[sp], ia = (i1 + 1) % 3, ib = (i1 + 2) % 3;
      ov3 sb = split_point(&p[base + ib], 0.5f, 0.5f, 0.0f);
      ov3 sa = split_point(&p[base + ia], 0.5f, 0.5f, 0.0f);
      push3(out, t.v[ib], sb, sa);
      if (vnorm(vsub(t.v[ia], sb)) < vnorm(vsub(t.v[i1], sa))) {
        push3(out, t.v[ia], sa, sb);
        push3(out, t.v[i1], t.v[ia], sb);
      } else {
        push3(out, t.v[ia], sa, t.v[i1]);
        push3(out, t.v[i1], sa, sb);
      }
    } else {
      ov3 mid[3];
      for (uint32_t i = 0; i < 3; ++i) mid[i] = split_point(&p[base + i], 0.5f, 0.5f, 0.0f);
      push3(out, mid[0], mid[1], mid[2]);
      for (uint32_t i = 0; i < 3; ++i) push3(out, t.v[i], mid[i], mid[(i + 2) % 3]);
    }
  }
  free(split);
  return 0;
}

/* ========================================================================== *
 * Hot path
 * ========================================================================== */
/* BezierTriangle::intersect, reference/bezierTriangle.cpp:123-195 */
ohit orc_patch_intersect(const opatch *p, const oray *r, int limit) {
  ohit res;
  memset(&res, 0, sizeof res);
  res.patch = ~0u;
  ov3 ip; float ic, it;
  int valid = orc_plane_intersect_ray(p->under, r->start, r->dir, &ip, &ic, &it);
  if (!(valid && fabsf(it) > -p->h_in && fabsf(it) > p->h_out)) { res.what = ORC_NONE; return res; }
  ov3 bary = orc_matvec(p->minv, ip);
  if (!(limit == ORC_LIMIT_NONE ||
        (bary.x >= 0.0f && bary.x <= 1.0f && bary.y >= 0.0f && bary.y <= 1.0f && bary.z >= 0.0f && bary.z <= 1.0f))) {
    res.what = ORC_NONE;
    return res;
  }
  float d_in = p->h_in / ic, d_out = p->h_out / ic;
  float closer = it + (ic > 0.0f ? d_in : d_out);
  float further = it + (ic > 0.0f ? d_out : d_in);
  ov3 por = vadd(r->start, vmul(r->dir, closer));
  ov3 b = orc_matvec(p->minv, orc_plane_project(p->under, por));
  ov3 q = orc_patch_interpolate(p, b.x, b.y, b.z);
  float diff_c = fabsf(orc_plane_distance(p->under, por)) - fabsf(orc_plane_distance(p->under, q));
  por = vadd(r->start, vmul(r->dir, further));
  b = orc_matvec(p->minv, orc_plane_project(p->under, por));
  q = orc_patch_interpolate(p, b.x, b.y, b.z);
  float diff_f = fabsf(orc_plane_distance(p->under, por)) - fabsf(orc_plane_distance(p->under, q));
  float middle;
  float den = diff_c - diff_f;
  if (fabsf(den) < 0.000001f) middle = (closer + further) / 2.0f;
  else middle = (diff_c * further - diff_f * closer) / den;
  ov3 pdir = p->under.n;
  for (uint32_t i = 0; i < 4u; ++i) {
    res.t = middle;
    por = vadd(r->start, vmul(r->dir, middle));
    ov3 pp; float pc, pt;
    orc_plane_intersect_ray(p->under, por, pdir, &pp, &pc, &pt);
    res.bary = orc_matvec(p->minv, pp);
    res.normal = orc_patch_normal(p, res.bary);
    res.point = orc_patch_interpolate(p, res.bary.x, res.bary.y, res.bary.z);
    pdir = vnormalized(vsub(res.point, pp));
    middle = vdot(vsub(res.point, r->start), res.normal) / vdot(r->dir, res.normal);
  }
  if (vnorm(ray_perp(r, res.point)) > 0.01f || res.t < (further - closer) * 1.0f) {
    res.what = ORC_NONE;
  } else {
    uint32_t out = (orc_plane_distance(p->divider[0], res.point) < 0.0f ? 1u : 0u);
    out |= (orc_plane_distance(p->divider[1], res.point) < 0.0f ? 2u : 0u);
    out |= (orc_plane_distance(p->divider[2], res.point) < 0.0f ? 4u : 0u);
    if (out == 1u) res.what = ORC_FOLLOW0;
    else if (out == 2u) res.what = ORC_FOLLOW1;
    else if (out == 4u) res.what = ORC_FOLLOW2;
    else {
      res.what = ORC_INTERSECT;
      res.cos_inc = vdot(r->dir, res.normal);
    }
  }
  return res;
}

/* Work counters (planar tests, Newton runs incl. follow-side retries) for the roofline's
 * algorithmic flop count; updated once per BezierMesh::intersect call. */
static uint64_t g_cnt_tests, g_cnt_newton, g_cnt_follow, g_cnt_segments;
void orc_counters(uint64_t out[4]) { out[0] = g_cnt_tests; out[1] = g_cnt_newton; out[2] = g_cnt_follow; out[3] = g_cnt_segments; }
void orc_counters_reset(void) { g_cnt_tests = g_cnt_newton = g_cnt_follow = g_cnt_segments = 0; }

static int planar_candidate(const opatch *p, const oray *r) {
  ov3 ip; float ic, it;
  int valid = orc_plane_intersect_ray(p->under, r->start, r->dir, &ip, &ic, &it);
  if (!(valid && fabsf(it) > -p->h_in && fabsf(it) > p->h_out)) return 0;
  ov3 b = orc_matvec(p->minv, ip);
  return b.x >= 0.0f && b.x <= 1.0f && b.y >= 0.0f && b.y <= 1.0f && b.z >= 0.0f && b.z <= 1.0f;
}

/* BezierMesh::intersect, reference/bezierMesh.cpp:206-227 */
ohit orc_mesh_intersect(const opatch *p, uint32_t np, const oray *r) {
  uint64_t newton = 0, follow = 0;
  ohit best;
  memset(&best, 0, sizeof best);
  best.t = FLT_MAX;
  best.what = ORC_NONE;
  best.patch = ~0u;
  for (uint32_t i = 0; i < np; ++i) {
    if (!planar_candidate(&p[i], r)) continue;   /* same gate as the first lines of orc_patch_intersect */
    ++newton;
    ohit c = orc_patch_intersect(&p[i], r, ORC_LIMIT_THIS);
    uint32_t src = i;
    if (c.what <= ORC_FOLLOW2) {
      src = p[i].neigh[c.what];
      ++follow;
      c = orc_patch_intersect(&p[src], r, ORC_LIMIT_NONE);
    }
    if (c.what == ORC_INTERSECT && c.t < best.t) { best = c; best.patch = src; }
  }
#pragma omp atomic
  g_cnt_tests += np;
#pragma omp atomic
  g_cnt_newton += newton;
#pragma omp atomic
  g_cnt_follow += follow;
#pragma omp atomic
  g_cnt_segments += 1;
  return best;
}

/* BezierLens::refract, reference/bezierLens.cpp:4-34 */
uint32_t orc_lens_refract(const opatch *p, uint32_t np, float ri, const oray *r, uint32_t expected, oray *out) {
  uint32_t st;
  ohit h = orc_mesh_intersect(p, np, r);
  out->start = r->start;
  out->dir = r->dir;
  if (h.what == ORC_INTERSECT) {
    st = h.cos_inc < 0.0f ? ORC_RR_INSIDE : ORC_RR_OUTSIDE;
    out->start = h.point;
    float eta = st == ORC_RR_INSIDE ? 1.0f / ri : ri;
    float s2 = eta * eta * (1.0f - h.cos_inc * h.cos_inc);
    if (s2 < 0.99f) {
      if (s2 > 1e-12f) {
        float sgn = st == ORC_RR_INSIDE ? 1.0f : -1.0f;
        ov3 n = vmul(h.normal, sgn);
        float c1 = fabsf(h.cos_inc);
        float c2 = sqrtf(1.0f - s2);
        out->dir = vnormalized(vadd(vmul(r->dir, eta), vmul(n, eta * c1 - c2)));
      }
      /* else: direction unchanged */
    } else {
      st = ORC_RR_NONE;
    }
  } else {
    st = ORC_RR_NONE;
  }
  return st == expected ? st : ORC_RR_NONE;
}

/* ---- batch drivers ---- */
static inline oray ray_from_soa(const float *s, uint32_t n, uint32_t i) {
  oray r;
  r.start = v3(s[i], s[n + i], s[2 * n + i]);
  r.dir = v3(s[3 * n + i], s[4 * n + i], s[5 * n + i]);
  return r;
}
static inline void ray_to_soa(float *s, uint32_t n, uint32_t i, const oray *r) {
  s[i] = r->start.x; s[n + i] = r->start.y; s[2 * n + i] = r->start.z;
  s[3 * n + i] = r->dir.x; s[4 * n + i] = r->dir.y; s[5 * n + i] = r->dir.z;
}
static void set_threads(int threads) {
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#else
  (void)threads;
#endif
}
void orc_intersect_batch(const opatch *p, uint32_t np, const float *rays, uint32_t n, float *hits, int threads) {
  set_threads(threads);
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t ii = 0; ii < (int64_t)n; ++ii) {
    uint32_t i = (uint32_t)ii;
    oray r = ray_from_soa(rays, n, i);
    ohit h = orc_mesh_intersect(p, np, &r);
    float f[11] = {h.t, h.point.x, h.point.y, h.point.z, h.cos_inc, h.bary.x, h.bary.y, h.bary.z,
                   h.normal.x, h.normal.y, h.normal.z};
    if (h.what != ORC_INTERSECT) { for (int k = 1; k < 11; ++k) f[k] = 0.0f; }
    for (int k = 0; k < 11; ++k) hits[(size_t)k * n + i] = f[k];
    memcpy(&hits[(size_t)11 * n + i], &h.what, 4);
    memcpy(&hits[(size_t)12 * n + i], &h.patch, 4);
  }
}
void orc_refract_batch(const opatch *p, uint32_t np, float ri, const float *rays, const uint32_t *expected,
                       uint32_t n, float *out_rays, uint32_t *out_status, int threads) {
  set_threads(threads);
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t ii = 0; ii < (int64_t)n; ++ii) {
    uint32_t i = (uint32_t)ii;
    oray r = ray_from_soa(rays, n, i), o;
    uint32_t st = orc_lens_refract(p, np, ri, &r, expected[i], &o);
    if (st == ORC_RR_NONE) o = r;
    ray_to_soa(out_rays, n, i, &o);
    out_status[i] = st;
  }
}
void orc_trace_chain_batch(const opatch *const *lp, const uint32_t *lnp, const float *ri, uint32_t nlens,
                           const float *rays, uint32_t n, float *out_rays, uint32_t *out_status,
                           uint32_t *out_seg, int threads) {
  set_threads(threads);
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t ii = 0; ii < (int64_t)n; ++ii) {
    uint32_t i = (uint32_t)ii;
    oray r = ray_from_soa(rays, n, i);
    uint32_t st = ORC_RR_NONE, seg = 0;
    int alive = 1;
    for (uint32_t l = 0; l < nlens && alive; ++l) {
      for (uint32_t j = 0; j < 2u && alive; ++j) {
        oray o;
        ++seg;
        st = orc_lens_refract(lp[l], lnp[l], ri[l], &r, j == 0 ? ORC_RR_INSIDE : ORC_RR_OUTSIDE, &o);
        if (st == ORC_RR_NONE) alive = 0;
        else r = o;
      }
    }
    ray_to_soa(out_rays, n, i, &r);
    out_status[i] = st;
    out_seg[i] = seg;
  }
}

/* the planar gate matrix: out[r * np + i] = 1 iff ray r passes patch i's gate (cThis) */
void orc_planar_gate_batch(const opatch *p, uint32_t np, const float *rays, uint32_t n, uint8_t *out, int threads) {
  set_threads(threads);
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t rr = 0; rr < (int64_t)n; ++rr) {
    oray r = ray_from_soa(rays, n, (uint32_t)rr);
    for (uint32_t i = 0; i < np; ++i) out[(size_t)rr * np + i] = (uint8_t)planar_candidate(&p[i], &r);
  }
}

/* ========================================================================== *
 * measureApproximation, reference/test.cpp:429-460
 * ========================================================================== */
int orc_measure_approximation(uint32_t steps, int32_t sectors, int32_t belts, ov3 size, int32_t divisor, float *out_error) {
  omesh e; orc_mesh_init(&e);
  if (orc_mesh_make_ellipsoid(&e, sectors, belts, size)) return -1;
  orc_mesh_standardize_vertices(&e);
  if (orc_mesh_standardize_normals(&e)) { orc_mesh_free(&e); return -1; }
  for (uint32_t s = 0; s < steps; ++s) {
    opatch *p = (opatch *)malloc(sizeof(opatch) * e.n * 3);
    if (orc_bezier_build(&e, p)) { free(p); orc_mesh_free(&e); return -1; }
    omesh nx;
    orc_bezier_split_thick(p, e.n * 3, &e, &nx);
    free(p);
    orc_mesh_free(&e);
    e = nx;
    orc_mesh_standardize_vertices(&e);
    if (orc_mesh_standardize_normals(&e)) { orc_mesh_free(&e); return -1; }
  }
  opatch *p = (opatch *)malloc(sizeof(opatch) * e.n * 3);
  if (orc_bezier_build(&e, p)) { free(p); orc_mesh_free(&e); return -1; }
  omesh pl;
  orc_bezier_interpolate_mesh(p, e.n * 3, divisor, &pl);
  free(p);
  orc_mesh_standardize_vertices(&pl);
  uint32_t nv = orc_mesh_unique_vertices(&pl, NULL);
  ov3 *vs = (ov3 *)malloc(sizeof(ov3) * (nv + 1));
  orc_mesh_unique_vertices(&pl, vs);
  float sum = 0.0f;
  for (uint32_t i = 0; i < nv; ++i) {
    ov3 v = vs[i];
    float x = v.x / size.x, y = v.y / size.y, z = v.z / size.z;
    float rr = sqrtf(x * x + y * y + z * z);                   /* Spherical ctor, 3dGeomUtil.h:344-347 */
    float incl = acosf(z / rr);
    float azim = atan2f(y, x);
    ov3 eth = v3(size.x * sinf(incl) * cosf(azim), size.y * sinf(incl) * sinf(azim), size.z * cosf(incl));
    sum += vsq(vsub(v, eth)) / vsq(eth);
  }
  *out_error = sum / (float)nv;
  free(vs);
  orc_mesh_free(&pl);
  orc_mesh_free(&e);
  return 0;
}
