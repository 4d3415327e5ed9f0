/*
 * bzr_oracle.h -- TEST INFRASTRUCTURE ONLY.  CPU restatement (plain C11) of the
 * reference Bezier-triangle ray tracer, used as the parity checker for the HIP
 * product path.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library.  The product (libbzr.so) never links
 * or calls it.
 *
 * Reference restated: balazs-bamer/cuda-bezier-triangle-raytracer @ v1,
 *   reference/3dGeomUtil.h, mesh.{h,cpp}, bezierTriangle.{h,cpp},
 *   bezierMesh.{h,cpp}, bezierLens.{h,cpp}, test.cpp (measureApproximation).
 *
 * Arithmetic contract: IEEE binary32, no FP contraction (build with
 * -ffp-contract=off), Eigen 3.3 evaluation order for the fixed-size 3-vector
 * and 3x3 operations the reference uses (see bzr_oracle.c, "Eigen surface").
 *
 * Pinning status (see DESIGN.md section "Oracle"):
 *   - pinned by the reference's own known answers: the 7 measureApproximation
 *     KATs (reference/test.cpp:515-521; construction + interpolate, 1e-3 rel)
 *     and the googleTest L1 geometry cases (reference/googleTest.cpp:46-353);
 *   - the hot path (BezierTriangle::intersect / BezierMesh::intersect /
 *     BezierLens::refract) has NO known answer in the reference and the
 *     reference cannot be built here (Eigen3 absent, no network): hot-path
 *     parity against the reference itself is PARTIALLY PINNED -- by the
 *     reference's refraction harness (reference/test.cpp:330-427, 22 inside /
 *     22 outside events, tests/test_reference_harness.py) and the statistics
 *     SURVEY.md section 8 recorded from the reference; the golden fixtures in
 *     tests/golden/ are generated from this oracle (regression pins).
 *
 * Documented deviations from the reference (both are undefined behaviour there):
 *   D1  Plane::intersect(start, dir) (reference/3dGeomUtil.h:279-296) writes
 *       mPoint only when distance > 0; the oracle writes start + t*dir whenever
 *       |cos| >= 1e-5 (mValid keeps its t > 0 rule).  SURVEY.md section 0.2.
 *   D2  when |cos| < 1e-5 mPoint is still unset in the reference; the oracle
 *       returns mPoint = start (only reachable inside the Newton loop when the
 *       projection direction degenerates to the zero vector).
 */
#ifndef BZR_ORACLE_H
#define BZR_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { float x, y, z; } ov3;
typedef struct { ov3 v[3]; } otri;
typedef struct { ov3 n; float c; } oplane;

/* Byte-identical to the reference BezierTriangle (reference/bezierTriangle.h:64-80):
 * 264 bytes, trivially copyable, align 4.  The matrix is Eigen column-major. */
typedef struct {
  oplane   under;          /* mUnderlyingPlane            @0   */
  oplane   divider[3];     /* mNeighbourDividerPlanes     @16  */
  uint32_t neigh[3];       /* mNeighbours                 @64  */
  ov3      cp[10];         /* mControlPoints              @76  */
  float    minv[9];        /* mBarycentricInverse (col-major) @196 */
  float    h_in;           /* mHeightInside               @232 */
  float    h_out;          /* mHeightOutside              @236 */
  ov3      dir_a;          /* mBezierDerivativeDirectionVectorA @240 */
  ov3      dir_b;          /* mBezierDerivativeDirectionVectorB @252 */
} opatch;

/* reference/mesh.h:27-30 */
typedef struct {
  uint32_t fellow[3];
  uint8_t  start[3];
} oneigh;

typedef struct {
  otri    *tri;
  uint32_t n, cap;
  oneigh  *f2n;        /* filled by orc_mesh_standardize_normals */
  uint32_t nf2n;
  ov3     *nrm_key;    /* vertex -> average normal map (reference/mesh.h:38) */
  ov3     *nrm_val;
  uint32_t nnrm;
} omesh;

/* Result of BezierTriangle::intersect / BezierMesh::intersect
 * (reference/bezierTriangle.h:7-20) plus the winning patch index. */
typedef struct {
  float    t;            /* mIntersection.mDistance */
  ov3      point;        /* mIntersection.mPoint */
  float    cos_inc;      /* mIntersection.mCosIncidence */
  ov3      bary;         /* mBarycentric */
  ov3      normal;       /* mNormal */
  uint32_t what;         /* 0..2 follow side, 3 none, 4 intersect */
  uint32_t patch;        /* index of the patch that produced the hit; ~0u on miss */
} ohit;

enum { ORC_FOLLOW0 = 0, ORC_FOLLOW1 = 1, ORC_FOLLOW2 = 2, ORC_NONE = 3, ORC_INTERSECT = 4 };
enum { ORC_LIMIT_THIS = 0, ORC_LIMIT_NONE = 1 };                 /* LimitPlaneIntersection */
enum { ORC_RR_NONE = 0, ORC_RR_INSIDE = 1, ORC_RR_OUTSIDE = 2 }; /* RefractionResult */
enum { ORC_ENV_ELLIPSOID = 0, ORC_ENV_TESTLENS = 1 };            /* envelope functions */

typedef struct { ov3 start, dir; } oray;

/* ---- error reporting: preprocessing "throws" are reported as non-zero status ---- */
const char *orc_last_error(void);

/* ---- Mesh (reference/mesh.{h,cpp}) ---- */
void     orc_mesh_init(omesh *m);
void     orc_mesh_free(omesh *m);
int      orc_mesh_copy(omesh *dst, const omesh *src);
int      orc_mesh_push(omesh *m, const otri *t);
int      orc_mesh_make_solid_of_revolution(omesh *m, int32_t sectors, int32_t belts, int envelope, ov3 size);
int      orc_mesh_make_ellipsoid(omesh *m, int32_t sectors, int32_t belts, ov3 size);
int      orc_mesh_standardize_vertices(omesh *m);
int      orc_mesh_standardize_normals(omesh *m);          /* returns -1 on "Vertex on edge detected." */
void     orc_mesh_transform(omesh *m, const float tr[9] /* col-major */, ov3 disp);
int      orc_mesh_split_divisor(omesh *m, int32_t divisor);
int      orc_mesh_split_maxside(omesh *m, float max_side);
int      orc_mesh_read_stl(omesh *m, const char *path);
int      orc_mesh_write_stl(const omesh *m, const char *path);
uint32_t orc_mesh_unique_vertices(const omesh *m, ov3 *out /* may be NULL */);

/* ---- BezierMesh (reference/bezierMesh.{h,cpp}) ---- */
/* Builds 3*m->n patches; m must be standardized. Returns -1 if a vertex normal is missing. */
int      orc_bezier_build(const omesh *m, opatch *out);
int      orc_bezier_interpolate_mesh(const opatch *p, uint32_t np, int32_t divisor, omesh *out);
int      orc_bezier_split_thick(const opatch *p, uint32_t np, const omesh *orig, omesh *out);
ov3      orc_patch_interpolate(const opatch *p, float b0, float b1, float b2);
ov3      orc_patch_normal(const opatch *p, ov3 bary);

/* ---- hot path ---- */
oray     orc_ray_make(ov3 start, ov3 dir);                 /* Ray ctor normalises (3dGeomUtil.h:176-178) */
ohit     orc_patch_intersect(const opatch *p, const oray *r, int limit);
ohit     orc_mesh_intersect(const opatch *p, uint32_t np, const oray *r);
/* BezierLens::refract; returns status, writes *out (start/dir unspecified when status == NONE) */
uint32_t orc_lens_refract(const opatch *p, uint32_t np, float ri, const oray *r, uint32_t expected, oray *out);

/* ---- batch drivers (OpenMP) for fixtures and the CPU baseline ---- */
/* rays_soa: 6*n floats (ox[n], oy[n], oz[n], dx[n], dy[n], dz[n]); directions used verbatim.
 * hits_soa: 13*n words, field-major: t, px,py,pz, cos, bx,by,bz, nx,ny,nz, what(u32), patch(u32). */
void     orc_intersect_batch(const opatch *p, uint32_t np, const float *rays_soa, uint32_t n,
                             float *hits_soa, int threads);
/* Refraction chain (reference/test.cpp:376-401): per lens refract(INSIDE) then refract(OUTSIDE);
 * a NONE terminates.  out_rays_soa 6*n (ray after the last successful refraction, input ray if none),
 * out_status n (last status), out_segments n (number of BezierMesh::intersect calls made). */
void     orc_trace_chain_batch(const opatch *const *lens_patches, const uint32_t *lens_np, const float *ri,
                               uint32_t nlens, const float *rays_soa, uint32_t n,
                               float *out_rays_soa, uint32_t *out_status, uint32_t *out_segments, int threads);
/* Single refract call over a batch with per-ray expected status. */
void     orc_refract_batch(const opatch *p, uint32_t np, float ri, const float *rays_soa, const uint32_t *expected,
                           uint32_t n, float *out_rays_soa, uint32_t *out_status, int threads);

/* test hook: out[r * np + i] = 1 iff ray r passes patch i's planar gate (cThis) */
void     orc_planar_gate_batch(const opatch *p, uint32_t np, const float *rays_soa, uint32_t n, uint8_t *out, int threads);
/* work counters since the last reset: planar tests, Newton runs, follow-side retries, intersect calls */
void     orc_counters(uint64_t out[4]);
void     orc_counters_reset(void);

/* ---- reference/test.cpp:429-460 measureApproximation (the 7 published KATs) ---- */
int      orc_measure_approximation(uint32_t split_steps, int32_t sectors, int32_t belts, ov3 size,
                                   int32_t divisor, float *out_error);

/* ---- L1 geometry (reference/3dGeomUtil.h), exported for the googleTest restatement ---- */
oplane   orc_plane_from_1proportion_2points(float prop, ov3 p0, ov3 p1);
oplane   orc_plane_from_3points(ov3 p0, ov3 p1, ov3 p2);
oplane   orc_plane_from_1vector_2points(ov3 dir, ov3 p0, ov3 p1);
oplane   orc_plane_from_2vectors_1point(ov3 d0, ov3 d1, ov3 p);
ov3      orc_plane_intersect3(oplane a, oplane b, oplane c);
/* Plane::intersect(start, dir) with D1/D2; valid (0/1) returned, point/cos/t written */
int      orc_plane_intersect_ray(oplane pl, ov3 start, ov3 dir, ov3 *point, float *cos_inc, float *t);
ov3      orc_plane_project(oplane pl, ov3 p);
float    orc_plane_distance(oplane pl, ov3 p);
void     orc_barycentric_inverse(ov3 v0, ov3 v1, ov3 v2, float out_colmajor[9]);
ov3      orc_matvec(const float m_colmajor[9], ov3 v);
uint32_t orc_to_which_side(ov3 start, ov3 end);
ov3      orc_get_aperpendicular(ov3 v);
float    orc_ray_average_error_squared(const oray *r, const ov3 *pts, uint32_t n);

/* ---- illumination ends (illum_oracle.c) ---- */
/* Same layouts as libbzr's bzr_emitter / bzr_target (include/bzr.h). */
typedef struct {
  float origin[3], edge_u[3], edge_v[3];
  uint32_t parts_u, parts_v, points_per_part, rays_per_point, belts;
  uint64_t seed;
} orc_emitter;
typedef struct {
  float origin[3], axis_u[3], axis_v[3];
  float size_u, size_v;
  uint32_t bins_u, bins_v;
} orc_target;
typedef struct orc_hemisphere orc_hemisphere;   /* UniformHemisphere (reference/hostUtil.h:8-24) */
orc_hemisphere *orc_hemisphere_create(uint32_t belts);
void     orc_hemisphere_free(orc_hemisphere *h);
uint32_t orc_hemisphere_patch_count(const orc_hemisphere *h);
uint32_t orc_hemisphere_random(orc_hemisphere *h, float dir[3]);
int      orc_emit(const orc_emitter *em, uint64_t first, uint32_t n, float *rays_soa, uint32_t *patch);
void     orc_land(const orc_target *tg, const float *rays_soa, const uint32_t *status, uint32_t n, uint32_t *hist,
                  uint64_t *exited, uint64_t *landed);

#ifdef __cplusplus
}
#endif
#endif
