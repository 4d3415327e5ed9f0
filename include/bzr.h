/*
 * bzr.h -- C ABI of the MI355X-native Bezier-triangle ray tracer (libbzr.so).
 *
 * The reference (balazs-bamer/cuda-bezier-triangle-raytracer @ v1) has no FFI;
 * its boundary is the C++ class API it exports for this path:
 *   BezierMesh::intersect(Ray)          reference/bezierMesh.h:37, bezierMesh.cpp:206-227
 *   BezierTriangle::intersect(Ray, lim) reference/bezierTriangle.h:105, bezierTriangle.cpp:123-195
 *   BezierLens::refract(Ray, expected)  reference/bezierLens.h:27, bezierLens.cpp:4-34
 *   the refraction-chain driver loop    reference/test.cpp:376-401
 * plus the host preprocessing that produces the patch records
 *   Mesh                                reference/mesh.h:18-133
 *   BezierMesh::BezierMesh(Mesh)        reference/bezierMesh.cpp:4-51
 * Every entry point below is the batch form of one of those, with plain
 * pointers and sizes.  The C++ drop-in classes in include/bzr/bzr.hpp forward
 * to it; INTEGRATION.md shows the binding a maintainer adds.
 *
 * Conventions
 *   - Every call returns bzr_status (0 = ok).  Nothing throws across the ABI.
 *     bzr_last_error() returns the calling thread's last error text.
 *   - Rays are SoA: rays_soa[k*n + i], k = 0..5 -> ox, oy, oz, dx, dy, dz.
 *     Directions are used as given (the reference's Ray ctor normalises;
 *     normalise on the caller side exactly as Ray(start, dir) does).
 *   - Hits are SoA, 13 words per ray: hits_soa[k*n + i] with k =
 *       0 t   1 px  2 py  3 pz  4 cos  5 b0  6 b1  7 b2  8 nx  9 ny  10 nz
 *       11 what (uint32: 0..2 follow side, 3 none, 4 intersect)
 *       12 patch (uint32: index of the patch hit, 0xFFFFFFFF on a miss)
 *     On a miss t = FLT_MAX and fields 1..10 are 0 (the reference leaves them
 *     uninitialised).
 *   - Pointer residency is selected per call by BZR_DEVICE_PTRS; host-pointer
 *     calls are synchronous, device-pointer calls are asynchronous on the
 *     context's stream until bzr_sync().
 *   - Numerics: BZR_MODE_PARITY (default) is IEEE binary32 with the
 *     reference's operation order and no contraction, bit-identical to the CPU
 *     oracle.  BZR_MODE_FAST keeps the planar gate exact (same candidate
 *     patches as the reference) and runs the Newton stage with FMA contraction
 *     and the hardware's approximate reciprocal / square root; it meets the
 *     SURVEY 8c fast-mode gates (hit/miss >= 99.5 %, t within 1e-5 relative on
 *     >= 99 % of same-patch hits) but is not bit-exact.  FAST needs the culled
 *     path: FAST | BZR_ACCEL_NONE returns BZR_ERR_INVALID_ARGUMENT.
 *   - Scan strategy: by default each lens mesh carries a BVH over the regions
 *     where each patch's planar gate can pass, and only those patches reach
 *     the Newton stage -- the output bits are the brute-force scan's.
 *     BZR_ACCEL_NONE runs the reference's brute-force scan itself (A/B testing).
 *     Patches with no proven bound on where their float gate can pass (planes
 *     through ~the origin whose M is rounding-dominated, non-finite records)
 *     are not in the BVH: every wave tests them (the always list).
 *   - Flags are checked first: unknown bits, BZR_PIPELINE_STAGED together with
 *     BZR_PIPELINE_FUSED, or FAST | ACCEL_NONE return BZR_ERR_INVALID_ARGUMENT.
 */
#ifndef BZR_H
#define BZR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BZR_ABI_VERSION 2

typedef int32_t bzr_status;
enum {
  BZR_OK = 0,
  BZR_ERR_INVALID_ARGUMENT = 1,
  BZR_ERR_HIP = 2,
  BZR_ERR_OUT_OF_MEMORY = 3,
  BZR_ERR_PREPROCESS = 4,   /* a reference preprocessing "throw" (e.g. "Vertex on edge detected.") */
  BZR_ERR_NO_DEVICE = 5,
  BZR_ERR_CAPACITY = 6      /* a compact multi-GPU gather had more survivors than its capacity (bzr_tiled_sync) */
};

enum {
  BZR_HOST_PTRS = 0u,
  BZR_DEVICE_PTRS = 1u,
  BZR_MODE_PARITY = 0u,
  BZR_MODE_FAST = 2u,
  BZR_ACCEL_NONE = 4u,  /* brute-force patch scan instead of the (bit-identical) BVH-culled path */
  /* Culled-path pipeline (same output bits either way; neither flag = automatic choice):
   *   fused   one kernel per call (k_trace): each wave walks the BVH and runs the Newton stage for its own
   *           rays with patch-uniform records -- no per-pair HBM traffic; best when a wave's rays meet
   *           few distinct patches (dense ray grids, many rays per patch)
   *   staged  traverse -> bucket pairs by patch -> Newton -> resolve -> finish per segment; full-wave
   *           Newton passes whatever the ray coherence, at 3-12x the algorithmic HBM bytes
   * automatic: fused when n >= 256 x the largest lens's patch count (and always for meshes of 2^25 patches
   * or more, which the staged encoding cannot hold), else staged.  The 256 is tuned for callers that keep
   * two or three frames in flight (bench.py, bzr_tiled with several slots): there the fused path wins from
   * ~256 rays per patch up.  A caller that traces ONE frame at a time and waits for it sees the fused
   * frame's tail (its slowest waves) undiluted; the fused path dispatches a context's repeated same-size
   * calls longest-tile-first from the previous calls' costs, which shortens that tail (cfg2 lone frames
   * 0.62 -> 0.40 ms), and lone cfg2 frames now run as fast fused as staged (0.395 vs 0.392 ms, 341 rays per
   * patch).  The first call of a size, or calls of changing sizes, run in input order. */
  BZR_PIPELINE_STAGED = 8u,
  BZR_PIPELINE_FUSED = 16u,
  /* Ray records in the reference's layout: rays / out_rays are [n][6] (per ray start xyz, direction xyz --
   * `Ray` of reference/3dGeomUtil.h:168, 24 bytes) instead of [6][n].  Host or device pointers alike; the library
   * transposes on the device (48 bytes per ray each way, HBM-bound), so a C++ caller hands its std::vector<Ray>
   * over with no host-side conversion.  Accepted by bzr_intersect (rays), bzr_refract, bzr_trace_chain,
   * bzr_trace_tiled, bzr_tiled_set_rays (rays) and bzr_tiled_trace (out_rays); other calls reject it.  Other
   * arrays (hits, status, segments, expected) keep their layouts. */
  BZR_RAYS_AOS = 32u
};

enum { BZR_WHAT_FOLLOW0 = 0, BZR_WHAT_FOLLOW1 = 1, BZR_WHAT_FOLLOW2 = 2, BZR_WHAT_NONE = 3, BZR_WHAT_INTERSECT = 4 };
enum { BZR_LIMIT_THIS = 0, BZR_LIMIT_NONE = 1 };                       /* BezierTriangle::LimitPlaneIntersection */
enum { BZR_RR_NONE = 0, BZR_RR_INSIDE = 1, BZR_RR_OUTSIDE = 2 };       /* RefractionResult */
enum { BZR_HIT_FIELDS = 13, BZR_RAY_FIELDS = 6 };

/* One cubic Bezier patch, byte-identical to the reference's BezierTriangle
 * (reference/bezierTriangle.h:64-80; Eigen column-major 3x3): 264 bytes. */
typedef struct bzr_patch {
  float    under_n[3], under_c;        /* mUnderlyingPlane                  @0   */
  float    divider[3][4];              /* mNeighbourDividerPlanes (n, c)    @16  */
  uint32_t neigh[3];                   /* mNeighbours                       @64  */
  float    cp[10][3];                  /* mControlPoints                    @76  */
  float    minv[9];                    /* mBarycentricInverse, col-major    @196 */
  float    h_in, h_out;                /* mHeightInside / mHeightOutside    @232 */
  float    dir_a[3], dir_b[3];         /* derivative direction vectors      @240 */
} bzr_patch;

typedef struct bzr_ctx bzr_ctx;         /* one HIP device + one stream; one host thread at a time */
typedef struct bzr_mesh bzr_mesh;       /* immutable device copy of a patch array */
typedef struct bzr_trimesh bzr_trimesh; /* host triangle mesh (reference Mesh) */

/* ---- library ---- */
int32_t     bzr_abi_version(void);
const char *bzr_last_error(void);
bzr_status  bzr_device_count(int32_t *count);

/* ---- context ---- */
bzr_status bzr_ctx_create(int32_t hip_device, bzr_ctx **out);
bzr_status bzr_ctx_destroy(bzr_ctx *ctx);
/* Launch on a caller-owned hipStream_t (NULL = the HIP null stream);
 * bzr_ctx_use_own_stream() goes back to the context's own non-blocking stream.  Work already queued
 * on the previous stream is ordered before later launches (an event hand-off, no host wait): the
 * hand-off records an event on the previous stream, so a caller stream must stay alive while it is
 * bound and until the next bzr_ctx_set_stream / bzr_ctx_use_own_stream / bzr_ctx_destroy returns.
 * Device-pointer calls launch on the bound stream and return before the kernels finish: inputs must
 * be ready on that stream, and outputs are valid on it (or after bzr_sync). */
bzr_status bzr_ctx_set_stream(bzr_ctx *ctx, void *hip_stream);
bzr_status bzr_ctx_use_own_stream(bzr_ctx *ctx);
bzr_status bzr_ctx_get_stream(bzr_ctx *ctx, void **hip_stream);
bzr_status bzr_sync(bzr_ctx *ctx);

/* ---- measurement: per-kernel HIP-event timing on the context's stream ---- */
enum {
  BZR_KERNEL_TRAVERSE = 0,        /* BVH walk + planar gate -> candidate pairs, per-patch histogram */
  BZR_KERNEL_BUCKET = 1,          /* prefix sum + scatter of the pairs into patch-major order */
  BZR_KERNEL_NEWTON = 2,          /* Newton stage per pair, patch-uniform waves */
  BZR_KERNEL_FOLLOW = 3,          /* k_resolve: follow-side neighbour retries + the overflow rays' full scans */
  BZR_KERNEL_FINISH = 4,          /* winner -> BezierIntersection / refraction */
  BZR_KERNEL_OVERFLOW = 5,        /* (unused since the full scans run inside k_resolve; id kept) */
  BZR_KERNEL_INTERSECT_SCAN = 6,  /* brute force (BZR_ACCEL_NONE) */
  BZR_KERNEL_REFRACT_SCAN = 7,
  BZR_KERNEL_CHAIN_SCAN = 8,
  BZR_KERNEL_PATCH = 9,
  BZR_KERNEL_NEWTON_LANE = 10,    /* Newton stage for fragmented pair chunks, one patch record per lane */
  BZR_KERNEL_TRACE = 11,          /* fused culled path: BVH walk + gate + Newton + winner (+ refraction chain) */
  BZR_KERNEL_COUNT = 12
};
/* While enabled, every launch is bracketed by hipEvents on the context's stream. */
bzr_status bzr_ctx_timing(bzr_ctx *ctx, int32_t enable);
/* Synchronises, returns the summed milliseconds and launch counts per kernel id since the last
 * report, and resets them. */
bzr_status bzr_ctx_timing_report(bzr_ctx *ctx, float ms[BZR_KERNEL_COUNT], uint32_t calls[BZR_KERNEL_COUNT]);

/* ---- measurement: work counters of the culled path (device-side, accumulated per segment) ---- */
enum {
  BZR_COUNTER_SEGMENTS = 0,      /* rays traced (one BezierMesh::intersect each) */
  BZR_COUNTER_PAIRS = 1,         /* (ray, patch) pairs that passed the planar gate: Newton runs */
  BZR_COUNTER_FOLLOWS = 2,       /* follow-side retries on a neighbour patch: Newton runs */
  BZR_COUNTER_OVERFLOW_RAYS = 3, /* rays resolved by the in-order full scan */
  BZR_COUNTER_LANE_CHUNKS = 4,   /* staged path: 64-pair chunks spanning many patches, one record per lane */
  BZR_COUNTER_NODE_VISITS = 5,   /* fused path: BVH nodes fetched (per wave, 128 B each) */
  BZR_COUNTER_LEAF_FETCHES = 6,  /* fused path: leaf gate records fetched (per wave, 64 B each) */
  BZR_COUNTER_GATE_TESTS = 7,    /* fused path: planar gates evaluated (per ray: lanes whose box test hit a fetched leaf) */
  BZR_COUNTER_NEWTON_ROUNDS = 8, /* fused path: patch-uniform Newton passes (per wave; cThis + follow-side) */
  BZR_COUNTER_ROUNDS_ODD = 9,    /* fused path: the passes of odd chain segments (refract(OUTSIDE): a lens's back surface) */
  BZR_COUNTER_RUNS_ODD = 10,     /* fused path: their Newton runs (pairs + follow retries) */
  BZR_COUNTER_DIRTY_ROWS = 11,   /* staged intersect: hit rows two improving pairs wrote concurrently (evaluated again) */
  BZR_COUNTER_COUNT = 12
};
/* While enabled, each culled segment adds its counts on the device (one tiny kernel per segment). */
bzr_status bzr_ctx_counters(bzr_ctx *ctx, int32_t enable);
/* Synchronises, returns the counts accumulated since the last report, and resets them. */
bzr_status bzr_ctx_counters_report(bzr_ctx *ctx, uint64_t counts[BZR_COUNTER_COUNT]);

/* ---- device mesh: BezierMesh's patch vector (reference/bezierMesh.h:17) ---- */
/* Copies n records of `stride` bytes (stride >= sizeof(bzr_patch)) from host memory. */
bzr_status bzr_mesh_create(bzr_ctx *ctx, const void *patches, uint32_t n, uint32_t stride, bzr_mesh **out);
bzr_status bzr_mesh_destroy(bzr_mesh *mesh);
bzr_status bzr_mesh_size(const bzr_mesh *mesh, uint32_t *n);

/* ---- hot path ---- */
/* BezierMesh::intersect over a ray batch (reference/bezierMesh.cpp:206-227). */
bzr_status bzr_intersect(bzr_ctx *ctx, const bzr_mesh *mesh, const float *rays_soa, uint32_t n,
                         float *hits_soa, uint32_t flags);
/* One hit in the reference's BezierIntersection layout (reference/bezierTriangle.h:7-21 with
 * Intersection of reference/3dGeomUtil.h:209-214): 52 bytes, `valid` is the bool mValid in its first
 * byte (the other three bytes zero). */
typedef struct bzr_hit_record {
  uint32_t valid;             /* mIntersection.mValid (what == BZR_WHAT_INTERSECT)   @0  */
  float    point[3];          /* mIntersection.mPoint                                @4  */
  float    cos_incidence;     /* mIntersection.mCosIncidence                         @16 */
  float    distance;          /* mIntersection.mDistance (FLT_MAX on a miss)          @20 */
  float    bary[3];           /* mBarycentric                                        @24 */
  float    normal[3];         /* mNormal                                             @36 */
  uint32_t what;              /* mWhat (BZR_WHAT_*)                                  @48 */
} bzr_hit_record;
/* bzr_intersect with the hits written as n bzr_hit_record (the drop-in's BezierIntersection array, no
 * host-side conversion; the records are built on the device, 52 B per ray) and the hit patch indices in
 * patch_index [n] (may be NULL; 0xFFFFFFFF on a miss).  Same values as bzr_intersect's rows; flags as
 * bzr_intersect's, BZR_RAYS_AOS included. */
bzr_status bzr_intersect_records(bzr_ctx *ctx, const bzr_mesh *mesh, const float *rays, uint32_t n,
                                 bzr_hit_record *records, uint32_t *patch_index, uint32_t flags);
/* BezierTriangle::intersect for (patch, ray, limit) triples (reference/bezierTriangle.cpp:123-195).
 * The `patch` field of the output is the input patch index. */
bzr_status bzr_patch_intersect(bzr_ctx *ctx, const bzr_mesh *mesh, const uint32_t *patch_index,
                               const uint32_t *limit, const float *rays_soa, uint32_t n,
                               float *hits_soa, uint32_t flags);
/* BezierLens::refract (reference/bezierLens.cpp:4-34); expected may be NULL (then every ray expects
 * `expected_all`).  out_rays_soa: the refracted ray (start = hit point) when status != NONE,
 * the input ray otherwise. */
bzr_status bzr_refract(bzr_ctx *ctx, const bzr_mesh *mesh, float refractive_index, const float *rays_soa,
                       const uint32_t *expected, uint32_t expected_all, uint32_t n,
                       float *out_rays_soa, uint32_t *out_status, uint32_t flags);
/* The reference refraction chain (reference/test.cpp:376-401): for each lens, refract(INSIDE) then
 * refract(OUTSIDE); a NONE terminates the ray.  out_rays_soa: ray after the last successful
 * refraction (input ray if none); out_status: last status (OUTSIDE = passed every lens);
 * out_segments (may be NULL): BezierMesh::intersect calls made for the ray. */
bzr_status bzr_trace_chain(bzr_ctx *ctx, const bzr_mesh *const *lenses, const float *refractive_index,
                           uint32_t nlens, const float *rays_soa, uint32_t n, float *out_rays_soa,
                           uint32_t *out_status, uint32_t *out_segments, uint32_t flags);
/* Multi-GPU refraction chain in ONE process (C/C++ hosts without torch.distributed):
 * image-plane tiles are dealt round-robin to the contexts, one per device.  Tile k is the rays
 * [k * tile_rays, (k + 1) * tile_rays) of the SoA input (callers order rays tile-major, e.g. 64x64-pixel
 * tiles of 4096 rays); context d traces tiles d, d + nctx, ... through its own copy of the lenses,
 * lenses[d * nlens + l] living on ctxs[d]'s device, and the results are gathered to ctxs[0]'s device on
 * the device side (RCCL when the contexts' devices are distinct, peer copies otherwise) and land in the
 * outputs in input order (same bits as one bzr_trace_chain over all rays).  A one-frame bzr_tiled plan
 * (below) created and destroyed per call: host pointers, or with BZR_DEVICE_PTRS rays and outputs on
 * ctxs[0]'s device.  Synchronous either way; the mode / pipeline flags pass through.  Callers tracing
 * many frames keep a plan instead (the RCCL communicator and the buffers are set up once). */
bzr_status bzr_trace_tiled(bzr_ctx *const *ctxs, uint32_t nctx, const bzr_mesh *const *lenses,
                           const float *refractive_index, uint32_t nlens, const float *rays_soa, uint32_t n,
                           uint32_t tile_rays, float *out_rays_soa, uint32_t *out_status,
                           uint32_t *out_segments, uint32_t flags);

/* ---- multi-GPU frames from one process, gathered on the device (one host thread drives
 * every device, ncclCommInitAll, grouped ncclSend / ncclRecv to device 0) ---- */
typedef struct bzr_tiled bzr_tiled;
enum { BZR_GATHER_AUTO = 0, BZR_GATHER_RCCL = 1, BZR_GATHER_PEER = 2, BZR_GATHER_DIRECT = 3 };
/* A frame plan over ndev devices and nslot frame slots: ctxs[s * ndev + d] is slot s's context on list
 * device d (every slot lists the same devices in the same order; all contexts distinct).  The frame is n
 * rays in tile-major order; device d traces tiles d, d + ndev, ... (its share).  The plan owns each
 * device's share buffers per slot and device 0's receive buffers.  transport: BZR_GATHER_RCCL (one RCCL
 * communicator per device, ncclCommInitAll; needs distinct devices), BZR_GATHER_PEER (hipMemcpyPeerAsync;
 * any device list, including several list entries on one device), BZR_GATHER_DIRECT (ndev == 1 only: the
 * one device traces straight into the caller's outputs -- no pack, no gather, no unpack, no share
 * buffers), BZR_GATHER_AUTO (DIRECT for one device, RCCL when several devices are distinct, PEER
 * otherwise).  Not thread-safe; the contexts must not be used by other threads meanwhile. */
bzr_status bzr_tiled_create(bzr_ctx *const *ctxs, uint32_t ndev, uint32_t nslot, uint32_t n, uint32_t tile_rays,
                            int32_t transport, bzr_tiled **out);
bzr_status bzr_tiled_destroy(bzr_tiled *plan);
/* transport chosen; share_rays[ndev] (may be NULL): rays per device; npad (may be NULL): columns of a
 * packed share (the largest share, in whole tiles) -- each device sends 28 * npad bytes per frame. */
bzr_status bzr_tiled_info(const bzr_tiled *plan, int32_t *transport, uint32_t *share_rays, uint32_t *npad);
/* The frame's input rays [6][n] (host memory, or with BZR_DEVICE_PTRS ctxs[0]'s device memory) into every
 * device's share.  Waits for the frames in flight first (they read the previous rays).  The frame lands on
 * device 0 once (host: one H2D copy, then the call waits for it so the host buffer may be reused; device:
 * one D2D copy, which must find the source complete and unchanged until bzr_tiled_sync); device 0 extracts
 * each device's share and sends it there (one peer copy per other device, (ndev - 1) / ndev of the frame
 * in all), queued on ctxs[0]'s stream and ordered before the next bzr_tiled_trace without a host wait.
 * With one device the frame is the share: one copy, nothing extracted.  The rays stay resident for every
 * following frame.  BZR_RAYS_AOS: the rays are [n][6] records, transposed on device 0 after the copy. */
bzr_status bzr_tiled_set_rays(bzr_tiled *plan, const float *rays_soa, uint32_t flags);
/* Device d's share input [6][share_rays[d]] (device memory on device d), for callers that generate rays
 * on the devices: write it (ordered before the next bzr_tiled_trace, e.g. then bzr_tiled_sync). */
bzr_status bzr_tiled_share_rays(bzr_tiled *plan, uint32_t device_index, float **rays_soa);
/* One frame on slot (frame number mod nslot): every device traces its share through
 * lenses[d * nlens + l] (refract(INSIDE) then refract(OUTSIDE) per lens, as bzr_trace_chain), packs it
 * (28 B per ray), the packed shares are gathered to device 0, which writes out_rays_soa [6][n],
 * out_status [n] and out_segments [n] (may be NULL) in input order.  BZR_DEVICE_PTRS: outputs on ctxs[0]'s
 * device; the call returns once the frame is queued (no host wait), frames on different slots overlap,
 * and the outputs are ready on bzr_tiled_stream's stream (or after bzr_tiled_sync) -- keep one set of
 * outputs per frame in flight.  Host pointers: synchronous, and a compact frame with more survivors than
 * the capacity returns BZR_ERR_CAPACITY at once.  Mode / pipeline flags pass through.  BZR_RAYS_AOS: out_rays
 * as [n][6] records (device 0 transposes the frame's rays on the stream that produced them, 48 B per ray). */
bzr_status bzr_tiled_trace(bzr_tiled *plan, const bzr_mesh *const *lenses, const float *refractive_index,
                           uint32_t nlens, float *out_rays_soa, uint32_t *out_status, uint32_t *out_segments,
                           uint32_t flags);
/* Device 0's gather stream: the outputs of the last bzr_tiled_trace are complete in its order. */
bzr_status bzr_tiled_stream(bzr_tiled *plan, void **hip_stream);
/* Waits for every frame queued; returns BZR_ERR_CAPACITY if a compact frame since the last sync had more
 * survivors than the capacity (that frame's outputs are incomplete). */
bzr_status bzr_tiled_sync(bzr_tiled *plan);
/* What each device sends per frame (bzr_pack_frame's layouts): BZR_PACK_RAYS (default; 28 B per ray of the
 * share, npad columns) or BZR_PACK_COMPACT: one status/segment byte per ray, the survivor count and the
 * final rays of at most `cap` survivors (the rays that refracted at least once; 0 < cap <= npad) -- device
 * 0 returns the others' primary rays from its copy of the frame, so the compact layout needs
 * bzr_tiled_set_rays.  Synchronises first.  A BZR_GATHER_DIRECT plan gathers nothing: it keeps the layout,
 * which has no effect on its frames. */
bzr_status bzr_tiled_set_layout(bzr_tiled *plan, int32_t layout, uint32_t cap);
/* Traces one frame (rays layout, synchronous), counts each device's survivors and switches to the compact
 * layout with cap = the largest count + 1/64 + 64 (at most npad); cap_out (may be NULL) gets it. */
bzr_status bzr_tiled_calibrate(bzr_tiled *plan, const bzr_mesh *const *lenses, const float *refractive_index,
                               uint32_t nlens, uint32_t flags, uint32_t *cap_out);
/* BezierMesh::interpolate(divisor) on the device (reference/bezierMesh.cpp:55-66): the tessellated
 * surface, divisor^2 sub-triangles of every patch, in the reference's order (sub-triangle outer,
 * patch inner).  out_xyz: divisor^2 * n_patches triangles x 3 vertices x 3 floats.  divisor >= 1.
 * Bit-identical to the host bzr_bezier_interpolate of the same patches. */
bzr_status bzr_mesh_interpolate(bzr_ctx *ctx, const bzr_mesh *mesh, int32_t divisor, float *out_xyz,
                                uint32_t flags);

/* ---- illumination: emitter -> lens chain -> target plane (reference README.md:159-194) ---- */
/* A rectangular emitter (origin + a*edge_u + b*edge_v, a, b in [0,1)) divided into parts_u x
 * parts_v parts; rays are numbered part by part, points_per_part points per part, rays_per_point
 * rays per point.  Directions are uniform over the hemisphere around +x, sampled as
 * UniformHemisphere::getRandom does (reference/hostUtil.cpp:16-29: cos(incidence) uniform in
 * [0,1), turn uniform in [0, 2*pi)) from a counter-based generator (splitmix64 of seed and ray
 * index), so any ray range can be generated independently; `belts` sets the hemisphere patch
 * numbering of UniformHemisphere(belts) (reference/hostUtil.cpp:3-14). */
typedef struct bzr_emitter {
  float origin[3], edge_u[3], edge_v[3];
  uint32_t parts_u, parts_v, points_per_part, rays_per_point, belts;
  uint64_t seed;
} bzr_emitter;
/* The illuminated rectangle: origin + a*axis_u + b*axis_v (unit, orthogonal axes), a in
 * [0, size_u), b in [0, size_v), bins_u x bins_v counting cells (row-major, u fastest).  A ray that
 * leaves the last lens (status OUTSIDE) lands where Plane::intersect (reference/3dGeomUtil.h:279-296)
 * meets the plane through origin with normal axis_u x axis_v. */
typedef struct bzr_target {
  float origin[3], axis_u[3], axis_v[3];
  float size_u, size_v;
  uint32_t bins_u, bins_v;
} bzr_target;
enum { BZR_ILLUM_EMITTED = 0, BZR_ILLUM_CULLED = 1, BZR_ILLUM_EXITED = 2, BZR_ILLUM_LANDED = 3 };
/* Rays first .. first+n-1 of the emitter: rays_soa [6][n] (unit directions), hemisphere patch
 * index per ray (may be NULL). */
bzr_status bzr_emit(bzr_ctx *ctx, const bzr_emitter *em, uint64_t first, uint32_t n, float *rays_soa,
                    uint32_t *patch_index, uint32_t flags);
/* Emits `total_rays` rays, drops those that miss the first lens's bounding sphere (Ritter's sphere
 * over the gate-region boxes: a ray that misses it cannot pass any planar gate, so dropping it is
 * exact), traces the rest through the refraction chain and adds one count per landed ray to
 * hist[bins_v][bins_u] (accumulates: zero it first).  stats (may be NULL) gets the BZR_ILLUM_*
 * counts.  Synchronous; hist may be host or device memory per `flags`. */
bzr_status bzr_illuminate(bzr_ctx *ctx, const bzr_mesh *const *lenses, const float *refractive_index,
                          uint32_t nlens, const bzr_emitter *em, uint64_t total_rays, const bzr_target *target,
                          uint32_t *hist, uint64_t stats[4], uint32_t flags);
/* The bounding sphere bzr_illuminate culls with: center xyz, radius. */
bzr_status bzr_mesh_bounding_sphere(const bzr_mesh *mesh, float out[4]);

/* ---- multi-GPU frames: a rank's results into its gather buffer (bzr_amd/frame.py) ---- */
/* No reference counterpart: the reference is single-process (its refraction chain loop,
 * reference/test.cpp:376-401, keeps the results in host vectors); this is the step between
 * bzr_trace_chain and the per-frame gather of a sharded image. */
enum { BZR_PACK_IMAGE = 0, BZR_PACK_RAYS = 1, BZR_PACK_COMPACT = 2 };
/* One chain frame's outputs (bzr_trace_chain: rays_soa [6][n], status [n], segments [n]; device
 * pointers) into `packed` (device) on the context's stream, without a host sync.  npad >= n is the
 * padded per-rank column count of the gather buffer.
 *   BZR_PACK_IMAGE    packed[npad] words: word i = status | segments << 8 (rays_soa may be NULL)
 *   BZR_PACK_RAYS     packed[7][npad]: the 6 ray rows, then the word row
 *   BZR_PACK_COMPACT  npad / 4 words of bytes, byte i = (status & 3) | segments << 2; then the
 *                     survivor count (uint32); then 6 rows of cap + 1 floats holding the rays of the
 *                     survivors (segments >= 2 or status != 0) in ray order.  0 < cap <= npad, npad a
 *                     multiple of 4; survivors past cap are counted but not written (the reader checks
 *                     count <= cap).
 * Columns >= n (and the last column of each compact row) are not written.  With n = 0 the input
 * pointers may be NULL. */
bzr_status bzr_pack_frame(bzr_ctx *ctx, int32_t layout, const float *rays_soa, const uint32_t *status,
                          const uint32_t *segments, uint32_t n, uint32_t npad, uint32_t cap, void *packed);

/* ---- host preprocessing (reference Mesh / BezierMesh construction) ---- */
enum { BZR_ENVELOPE_ELLIPSOID = 0, BZR_ENVELOPE_TESTLENS = 1 };
bzr_status bzr_trimesh_create(bzr_trimesh **out);
bzr_status bzr_trimesh_destroy(bzr_trimesh *m);
bzr_status bzr_trimesh_copy(const bzr_trimesh *src, bzr_trimesh **out);
bzr_status bzr_trimesh_size(const bzr_trimesh *m, uint32_t *n);
bzr_status bzr_trimesh_get(const bzr_trimesh *m, float *xyz /* 9*n */);
bzr_status bzr_trimesh_set(bzr_trimesh *m, const float *xyz, uint32_t n);
bzr_status bzr_trimesh_make_solid_of_revolution(bzr_trimesh *m, int32_t sectors, int32_t belts, int32_t envelope,
                                                float sx, float sy, float sz);
bzr_status bzr_trimesh_make_ellipsoid(bzr_trimesh *m, int32_t sectors, int32_t belts, float sx, float sy, float sz);
bzr_status bzr_trimesh_read_stl(bzr_trimesh *m, const char *path);
bzr_status bzr_trimesh_write_stl(const bzr_trimesh *m, const char *path);
bzr_status bzr_trimesh_transform(bzr_trimesh *m, const float transform_colmajor[9], const float displacement[3]);
bzr_status bzr_trimesh_split(bzr_trimesh *m, int32_t divisor);
bzr_status bzr_trimesh_split_maxside(bzr_trimesh *m, float max_side);
bzr_status bzr_trimesh_standardize_vertices(bzr_trimesh *m);
bzr_status bzr_trimesh_standardize_normals(bzr_trimesh *m);
/* Face neighbours after standardize_normals: 3 fellow indices + 3 common-side starts per face. */
bzr_status bzr_trimesh_neighbours(const bzr_trimesh *m, uint32_t *fellow /* 3*n */, uint8_t *start /* 3*n */);
/* BezierMesh(Mesh): writes 3*n patches. */
bzr_status bzr_bezier_build(const bzr_trimesh *m, bzr_patch *out);
/* BezierMesh::splitThickBezierTriangles -> new (unstandardized) triangle mesh */
bzr_status bzr_bezier_split_thick(const bzr_trimesh *m, bzr_trimesh *out);
/* BezierMesh::interpolate(divisor) -> tessellated triangle mesh */
bzr_status bzr_bezier_interpolate(const bzr_trimesh *m, int32_t divisor, bzr_trimesh *out);

#ifdef __cplusplus
}
#endif
#endif
