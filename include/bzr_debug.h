/*
 * bzr_debug.h -- test hooks of libbzr.so (not part of the drop-in boundary).
 */
#ifndef BZR_DEBUG_H
#define BZR_DEBUG_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
/* The culling boxes the BVH is built from, by patch index: boxes[6*i] = lo.xyz, hi.xyz of the region
 * where patch i's planar gate can pass for ray origins with |s|_inf <= *s_max.  Returns 0 on success. */
int32_t bzr_debug_gate_boxes(const void *patches, uint32_t n, uint32_t stride, float *boxes, float *s_max);
/* The same for one BVH tier: 0 = far (as above), 1 = near (bvh.hpp kTierNear; tighter boxes, valid for
 * origins |s|_inf <= *s_max, which is 8x the mesh's control-point span). */
int32_t bzr_debug_gate_boxes_tier(const void *patches, uint32_t n, uint32_t stride, int32_t tier, float *boxes,
                                  float *s_max);
/* Patches without a proven gate region (rounding-dominated, or non-finite records): they are not in the
 * tier's tree and every wave-segment gate-tests them (bvh.hpp Bvh::always).  *count = their number; out
 * (optional, *count words) = their indices, ascending.  Their gate boxes above are the always-hit box.
 * Returns 0 on success. */
int32_t bzr_debug_always_list(const void *patches, uint32_t n, uint32_t stride, int32_t tier, uint32_t *out,
                              uint32_t *count);
/* The always list's wedge pre-test (bvh.cpp always_wedge), 8 floats per always-listed patch in list order:
 * w.xyz, L, H, B, C, 0.  A lane whose float plane point p~ = s + d (num x rcp(cs)) has w.p~ outside
 * [L - B|p~| - C(|s|+|p~|), H + B|p~| + C(|s|+|p~|)] cannot pass that patch's gate. */
int32_t bzr_debug_always_wedges(const void *patches, uint32_t n, uint32_t stride, int32_t tier, float *out);
/* The oriented gate-region boxes of one tier's wide-patch subtree (bvh.hpp Bvh4ObbNode), by patch index:
 * out[16*i] = centre xyz, axes u v w (xyz each), half extents (3), then 1.0f if patch i is a wide patch
 * (its parent node tests this box) or 0.0f (16 zeros: the patch is AABB-culled).  Returns 0 on success. */
int32_t bzr_debug_gate_obbs(const void *patches, uint32_t n, uint32_t stride, int32_t tier, float *out);
/* The bounding sphere bzr_illuminate culls with (Ritter over the gate boxes): centre xyz, radius. */
int32_t bzr_debug_bounding_sphere(const void *patches, uint32_t n, uint32_t stride, float out[4]);
/* Host replay of the device BVH walk (same 4-wide trees and wave-uniform tier choice, same float slab and
 * oriented-box tests -- 1/x where the device uses v_rcp_f32) over `nr` rays in SoA
 * [6, nr], grouped in waves of 64 consecutive rays.  hits (optional, nr x n bytes): hits[r*n + b] = 1
 * when ray r reaches patch b's leaf box -- a superset of the patches whose planar gate it passes.
 * stats[0] node visits (per wave), [1] leaf records fetched (per wave), [2] leaf-box hits (per ray),
 * [3] waves.  Returns 0 on success. */
int32_t bzr_debug_traverse(const void *patches, uint32_t n, uint32_t stride, const float *rays, uint32_t nr,
                           uint8_t *hits, uint64_t stats[4]);
/* Host replay of the wave-bundle walk (trace.hip BZR_TRACE_BUNDLE: batches of up to 16 nodes tested against
 * the wave's ray bundle) beside the per-lane walk, waves of 64 consecutive rays; waves whose direction spread
 * exceeds max_spread take the per-lane walk.  stats[0] waves, [1] bundle batches, [2] leaves (bundle or
 * per-lane walk), [3] per-lane node visits, [4] per-lane leaves, [5] per-lane leaves the bundle walk missed
 * (0: conservative), [6] child slots tested, [7] deepest work stack, [8] waves on the per-lane walk, [9]
 * batches after which the work stack exceeded 64, [10] bundle-walk leaves the leaf pre-test keeps, [11] leaves it
 * rejected although some lane's exact planar gate passes (0: conservative).  Returns 0 on success. */
int32_t bzr_debug_traverse_bundle(const void *patches, uint32_t n, uint32_t stride, const float *rays, uint32_t nr,
                                  float max_spread, uint64_t stats[12]);
/* Device check of the exact normalized() (Eigen a / sqrt(a.a)): `a` is device memory [3][n], `out` device
 * memory [6][n]: rows 0-2 the product's normalized(a), rows 3-5 the same with the compiler's correctly
 * rounded sqrt and one division per component.  Asynchronous on the context's stream.  ctx is a
 * bzr_ctx* (bzr.h). */
int32_t bzr_debug_unit(void *ctx, const float *a, uint32_t n, float *out);
/* Device check of newton_tail's bracket quotients hIn / cos, hOut / cos (patch_math.hpp div_heights: one shared
 * reciprocal where proven): `a` device memory [3][n] (hIn, hOut, cos), `out` device memory [4][n]: rows 0-1 the
 * product's quotients, rows 2-3 one correctly rounded division each.  Asynchronous on the context's stream. */
int32_t bzr_debug_div_heights(void *ctx, const float *a, uint32_t n, float *out);
/* Per-wave timing of the fused kernel: while set, every fused call (k_trace, one 64-ray wave per 64
 * consecutive rays) of `n` <= 64 * waves rays writes clock[2w] = the wave's start (s_memtime ticks) and
 * clock[2w+1] = its duration, for wave w = ray index / 64.  `clock` is device memory; NULL turns it off.
 * ctx is a bzr_ctx* (bzr.h). */
int32_t bzr_debug_wave_clock(void *ctx, unsigned long long *clock, uint32_t waves);
/* The same with the constant 100 MHz clock beside it (a diagnostic of the shader clock the chip holds,
 * MI355X_MICROARCH.md "DVFS give-back" item 6): clock[4w] = start, [4w+1] = duration (s_memtime ticks),
 * [4w+2] = start, [4w+3] = duration (s_memrealtime ticks); the wave's clock is [4w+1] / [4w+3] x 100 MHz. */
int32_t bzr_debug_wave_clock_rate(void *ctx, unsigned long long *clock, uint32_t waves);
#ifdef __cplusplus
}
#endif
#endif
