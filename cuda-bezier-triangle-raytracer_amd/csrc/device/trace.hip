// trace.hip -- CDNA4 kernels of the hot path + the device half of the C ABI.
//
// Reference semantics (one ray per lane, IEEE binary32, reference operation order):
//   BezierMesh::intersect      reference/bezierMesh.cpp:206-227
//   BezierTriangle::intersect  reference/bezierTriangle.cpp:123-195
//   BezierLens::refract        reference/bezierLens.cpp:4-34
//   refraction chain driver    reference/test.cpp:376-401
//
// Two interchangeable scan strategies, identical output bits (tests/test_gpu_parity.py):
//   culled (default)  k_traverse walks the lens BVH (bvh.cpp) wave-uniformly: node and patch
//                     boxes are fetched with scalar loads, each lane slab-tests its own ray, the
//                     wave descends while any lane hits (ballot), and lanes whose ray passes a
//                     patch's exact planar gate append that patch to their candidate list.
//                     k_resolve_* then runs the Newton stage over each ray's candidates and keeps
//                     the (t, patch index) lexicographic minimum -- the same winner as the
//                     reference's in-order strict-< scan.  Lists that overflow, stacks that
//                     overflow and rays beyond the boxes' validity radius fall back to the full
//                     in-order scan inside k_resolve_*, so every ray gets the reference result.
//   brute force       (BZR_ACCEL_NONE) the reference's own scan: every patch's 64-byte planar
//                     record fetched once per wave with scalar loads, Newton for passing lanes.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <functional>

#include <cstdio>
#include <cstring>
#include <new>
#include <type_traits>
#include <string>
#include <vector>

#include "../host/bvh.hpp"
#include "bzr.h"
#include "ctx.hpp"
#include "patch_math.hpp"
#include "emitter.hpp"

using namespace bzr_dev;

// ------------------------------------------------------------------ errors
namespace {
thread_local std::string t_error;
bzr_status set_error(bzr_status s, const std::string &msg) {
  t_error = msg;
  return s;
}
#define BZR_HIP(call)                                                                                     \
  do {                                                                                                    \
    hipError_t e_ = (call);                                                                               \
    if (e_ != hipSuccess) return set_error(BZR_ERR_HIP, std::string(#call ": ") + hipGetErrorString(e_)); \
  } while (0)
}  // namespace

extern "C" const char *bzr_last_error(void) { return t_error.c_str(); }
extern "C" int32_t bzr_abi_version(void) { return BZR_ABI_VERSION; }
// the host half of the library reports its errors through here
extern "C" void bzr_internal_set_error(const char *msg) { t_error = msg ? msg : ""; }

// ------------------------------------------------------------ device mesh
struct bzr_mesh {
  int device;
  uint32_t n;
  float4 *planar;   // 4 float4 per patch: n.xyz c | hin hout M00 M01 | M02 M10 M11 M12 | M20 M21 M22 0
  float *full;      // 66 words per patch (bzr_patch)
  bzr_host::Bvh4Node *nodes;  // 4-wide BVH over the patches' gate-region boxes (bvh.cpp), far tier
  float4 *leaf;     // 4 float4 per BVH leaf slot: the planar record, patch index in the last word
  bzr_host::Bvh4Node *nodes_near;  // the near tier's tree and leaf slots (bvh.hpp kTierNear)
  float4 *leaf_near;
  bzr_host::Bvh4ObbNode *obb;       // both tiers' wide-patch subtrees (oriented boxes, bvh.hpp)
  bzr_host::Bvh4ObbNode *obb_near;
  float4 *kids;      // the far tree's children AoS (2 float4 per child: lo.xyz ref, hi.xyz 0): the bundle walk's
  float4 *kids_near; // per-lane child records (kids_of), and the near tree's
  float4 *wide;      // two levels per node for k_traverse's bundle walk (BZR_TRAV_WIDE, wide_of): node i's 16
  float4 *wide_near; // grandchild slots, 2 float4 each as in kids
  float4 *always;   // 8 float4 per always-tested patch (bvh.hpp Bvh::always): planar record with the patch index
                    // in its last word, then the wedge pre-test (always_wedge: w.xyz L H B C 0) and 8 pad words
  uint32_t n_always;
  uint32_t nnodes;
  float s_max;      // far tier: origins beyond take the full scan
  float s_near;     // near tier: waves whose rays all start within it walk the tighter tree
  float sphere[4];  // Ritter sphere over the gate-region boxes (bvh.cpp): the illumination pre-cull
};

namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
constexpr uint32_t kMaxLenses = 8;
#ifndef BZR_MAX_CAND
#define BZR_MAX_CAND 40
#endif
constexpr uint32_t kMaxCand = BZR_MAX_CAND;  // candidate list length per ray and segment
constexpr uint32_t kOverflow = 0x8000u;  // count flag: resolve with the full scan (the low bits keep the listed count)
// Traversal stack entries per wave (LDS).  BZR_STACK (A/B and test knob): a tiny stack makes waves run out
// mid-walk, which sends the affected lanes to the in-order full scan (tests/test_gpu_variants.py).
#ifndef BZR_STACK
#define BZR_STACK 64
#endif
constexpr int kStack = BZR_STACK;
// Device work counters (bzr_ctx_counters) are kept in this many copies, summed by the report: a wave adds
// to copy (wave index mod kCounterReplicas), so a frame's ~10^5 waves do not queue on a few addresses.
constexpr uint32_t kCounterReplicas = 64;

// 64-byte wave-uniform records read through the constant address space: one s_load_dwordx16 each
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(4))) const u32x16 cu32x16;

// Blocks are dealt round-robin to the 8 XCDs (each with its own L2 and scalar caches).  This maps
// block b to a bijective index under which each XCD owns one contiguous range of the grid, so the
// blocks an XCD runs together work on neighbouring rays (same BVH nodes, same patches).
constexpr uint32_t kXcds = 8;
__device__ __forceinline__ uint32_t xcd_contiguous(uint32_t b, uint32_t nblocks) {
  const uint32_t q = nblocks / kXcds, r = nblocks % kXcds, x = b % kXcds;
  return x * q + (x < r ? x : r) + b / kXcds;
}
// Block b's index under a dealing policy: 0 = dispatch order (XCD x gets every 8th block), 1 =
// xcd_contiguous, G > 1 = runs of G blocks dealt round-robin to the XCDs (whole rounds of 8 runs; the
// ragged rest keeps its index).  A bijection on [0, nblocks) in every case.
template <uint32_t kPolicy>
__device__ __forceinline__ uint32_t deal_blocks(uint32_t b, uint32_t nblocks) {
  if constexpr (kPolicy == 0) {
    return b;
  } else if constexpr (kPolicy == 1) {
    return xcd_contiguous(b, nblocks);
  } else {
    const uint32_t full = nblocks / (kXcds * kPolicy) * (kXcds * kPolicy);
    if (b >= full) return b;
    const uint32_t x = b % kXcds, k = b / kXcds;
    return (k / kPolicy * kXcds + x) * kPolicy + k % kPolicy;
  }
}
// Threads per k_traverse block (BZR_TRAV_BLOCK, default 64): one-wave blocks let a finished wave be replaced
// at once, as in k_trace; 256 (4 waves sharing a CU's scalar cache on neighbouring rays, rounds 1-3) measured
// 0.5-1 % slower on cfg5 and 0.1-0.2 % on cfg3 at bench level, 128 4 % slower on cfg3
// (profiles/r04_bench_ab_trav_block.jsonl).
// BZR_TRAV_ABLOCK: the always list's bundle pre-test once per 256-thread block instead of once per wave, for
// meshes whose always list takes more than one 64-patch round (kAblockMin < n_always <= kAblockMax; others keep
// the one-wave kernel).  Before the walk every wave's bundle is in LDS; the block's union bundle tests the
// always-listed patches, one per thread, and keeps a mask in LDS.  1 (default): each wave gate-tests the
// block-kept patches per lane; 2: each wave first re-tests the block-kept patches against its own bundle in
// one (compacted) round; 0: off.  A dropped patch is one no ray of the block (so of the wave) can pass: the
// candidates are unchanged.  cfg5 (131 always-listed patches): k_traverse 4.01 -> 3.84 ms per frame with 1,
// 4.05 with 2 (profiles/r05_ab_traverse_ablock.jsonl).
// 3 (A/B): the pre-test in a kernel of its own before k_traverse (k_always_mask: the same union bundle per 256 rays
// and the same ballots, to a global mask), and k_traverse in one-wave blocks reading its 256-ray block's mask -- no
// barriers in the walk kernel.
#ifndef BZR_TRAV_ABLOCK
#define BZR_TRAV_ABLOCK 1
#endif
#ifndef BZR_TRAV_BLOCK
#define BZR_TRAV_BLOCK 64
#endif
#ifndef BZR_ABLOCK_BLOCK
#define BZR_ABLOCK_BLOCK 256
#endif
constexpr uint32_t kAblockMin = 64, kAblockMax = 1024, kAblockBlock = BZR_ABLOCK_BLOCK;  // threads per pre-testing block
constexpr uint32_t kAmaskWords = kAblockMax / 64u;  // mask words per pre-testing block (BZR_TRAV_ABLOCK 3)
// BZR_TRAV_ALDS (A/B knob, default 0): with the block pre-test (BZR_TRAV_ABLOCK 1), the block copies its kept
// always-listed records (the 96 bytes the per-lane gate reads) into LDS once, so the waves' per-lane gates read
// them there instead of waiting on one scalar load each (when at most kAldsMax are kept; else as before).
// Same 64 VGPRs and 8 waves, 18 KB of LDS per block; cfg5 k_traverse 3.85 -> 3.93 ms per lone frame, bench lines
// -0.8 % (profiles/r05_ab_traverse_alds.jsonl): the scalar loads hit the scalar cache; the copy and the records as
// VGPR operands cost more.  Not kept.
#ifndef BZR_TRAV_ALDS
#define BZR_TRAV_ALDS 0
#endif
constexpr uint32_t kAldsMax = 128, kAldsQuads = 6;
constexpr int kTravBlock = BZR_TRAV_BLOCK;
// BZR_SLAB_FMA (default 1): the traversal slab test as fma(lo, inv, -s*inv) (mirrored by bvh.cpp slab_h).
#ifndef BZR_SLAB_FMA
#define BZR_SLAB_FMA 1
#endif
// BZR_NEWTON_XCD (default 0): k_newton waves take chunks in XCD-contiguous order (measured +6 %, off).
// BZR_GATE_FLAT (default 1): planar_gate without early-out branches (see there).
// BZR_NODE_ASM (default 0): fetch a BVH node's two halves with one inline-asm pair of scalar loads and
// a single wait (node_children).
#ifndef BZR_NODE_ASM
#define BZR_NODE_ASM 0
#endif
// BZR_BUNDLE_SPREAD (default 0.5): waves whose ray directions spread wider (bundle_setup_dpp) take the
// per-lane walk instead of the bundle walk.
#ifndef BZR_BUNDLE_SPREAD
#define BZR_BUNDLE_SPREAD 0.5f
#endif
// BZR_TRAV_PRETEST (default 1): k_traverse's bundle walk pre-tests its queued leaves against the bundle
// (bundle_gate_keep, 64 leaves per pass) before the per-lane gates: the host replay keeps 64 % of cfg5's
// bundle leaves, 48 % of cfg3's, 36 % of cfg4's; k_traverse cfg5 -1.2 %, cfg3 -4 %, cfg2 within noise
// (profiles/r03s2_ab_leaf_pretest.jsonl; 68 VGPRs: 7 waves per SIMD instead of 8).
#ifndef BZR_TRAV_PRETEST
#define BZR_TRAV_PRETEST 1
#endif
// BZR_TRAV_LEAF_PAIRS (default 1): k_traverse's bundle walk fetches its queued leaves two at a time (cfg5 /
// cfg3 / cfg2 staged k_traverse -2 to -2.5 %, frames -1 %; profiles/r03s2_ab_leaf_pairs.jsonl).
#ifndef BZR_TRAV_LEAF_PAIRS
#define BZR_TRAV_LEAF_PAIRS 1
#endif
// BZR_TRAV_WIDE (default 1): k_traverse's bundle walk takes two tree levels per batch over 16-slot records
// (bzr_mesh wide / wide_near: each node's grandchildren), 4 nodes per batch instead of 16 nodes' children;
// 2: three levels over 64-slot records (one node per batch, a 4x deeper LDS stack); 0: one level.
#ifndef BZR_TRAV_WIDE
#define BZR_TRAV_WIDE 1
#endif
constexpr uint32_t kWideSlots = BZR_TRAV_WIDE == 2 ? 64u : 16u;  // slots per node of the wide records
// k_traverse's stack: a three-level batch (BZR_TRAV_WIDE 2) can push 64 entries at once
constexpr int kTravStack = BZR_TRAV_WIDE == 2 ? 4 * kStack : kStack;
// BZR_TRACE_BLEAF_PAIRS (A/B knob, default 0): k_trace's bundle walk gate-tests its queued leaves two at a time.
// Measured at bench level: cfg4 -4.1 %, cfg2 -2.7 %, cfg5 fused -3.4 % (80 VGPRs with 5 spilled to scratch,
// 49 SGPR spills; profiles/r04_bench_ab_trace_leaf_pairs.jsonl) -- unlike k_traverse, where pairs pay.
#ifndef BZR_TRACE_BLEAF_PAIRS
#define BZR_TRACE_BLEAF_PAIRS 0
#endif
// BZR_TRACE_WIDE (default 1, with BZR_TRACE_BUNDLE): k_trace's bundle walk over the same two-level records.
#ifndef BZR_TRACE_WIDE
#define BZR_TRACE_WIDE 1
#endif
// BZR_TRAV_BUNDLE (default 1): k_traverse walks with the wave-bundle test in batches (traverse_rays):
// cfg5 8192^2 staged k_traverse 6.61 -> 5.07 ms per frame, cfg3 0.283 -> 0.235, cfg2 0.134 -> 0.143
// (profiles/r03s2_ab_bundle_walk.jsonl).
#ifndef BZR_TRAV_BUNDLE
#define BZR_TRAV_BUNDLE 1
#endif
#ifndef BZR_GATE_FLAT
#define BZR_GATE_FLAT 1
#endif
#ifndef BZR_NEWTON_XCD
#define BZR_NEWTON_XCD 0
#endif
// Blocks of k_resolve at most (its overflow part is grid-stride over (overflow ray, patch slice) items).
#ifndef BZR_OVERFLOW_BLOCKS
#define BZR_OVERFLOW_BLOCKS 2048u
#endif
// BZR_NEWTON_QUEUE (A/B knob, default 0): k_newton's waves take their dense chunks from a work counter (w.ctr[5],
// one atomic per chunk and wave) instead of the static stride q, q + W, ...: a wave that drew cheap chunks takes
// more, so the kernel ends when the work does, not when its most loaded wave does.
#ifndef BZR_NEWTON_QUEUE
#define BZR_NEWTON_QUEUE 0
#endif
// BZR_NEWTON_GATED (default 1): k_newton skips the planar gate its pairs already passed in k_traverse.
#ifndef BZR_NEWTON_GATED
#define BZR_NEWTON_GATED 1
#endif
// BZR_STAGED_AOS (default 0): k_traverse also writes each ray of the chunk as a 32-byte AoS record (ox oy oz dx
// | dy dz), and the Newton / resolve kernels read a pair's ray from it -- one 32-byte sector instead of six
// SoA rows whose 128-byte lines serve few of a bucket's rays.
#ifndef BZR_STAGED_AOS
#define BZR_STAGED_AOS 0
#endif
// BZR_DENSE_MIN (default 16): the staged pair layout.  A patch bucket's pairs fill whole 64-pair chunks of
// that one patch (dense chunks: patch-uniform Newton passes, every lane busy); its last, partial chunk is
// padded to a whole chunk when it holds at least this many pairs, else its pairs go to the sparse region
// behind the dense chunks, where k_newton_lane runs one pair per lane with the lane's own patch record.
// 64 = no padding.  (A sparse chunk costs ~4 dense ones -- 4 waves per SIMD, per-lane record loads -- so a
// remainder of r pairs is cheaper padded from r ~ 16 on; cfg5: DESIGN.md.)  Padding is below 64 slots per
// patch, which sizes the pair array at cap + 64 (nb + 1).
#ifndef BZR_DENSE_MIN
#define BZR_DENSE_MIN 16
#endif
constexpr uint32_t kDenseMin = BZR_DENSE_MIN;
static_assert(kDenseMin >= 1 && kDenseMin <= 64, "BZR_DENSE_MIN: 1..64");
// Staged winner keys (t order << 32 | patch << 6 | list slot j) and pair records (ray | j << 26,
// patch | follow side << 30): chunk rays below 2^26, list slots below 64, patch indices below 2^25 (keys
// take 26 bits; the pair array's 32-bit indices, 64 padding slots per patch).
constexpr uint32_t kStagedPatchLimit = 1u << 25, kRayMask = (1u << 26) - 1u, kNoPair = 0xFFFFFFFFu;
struct MeshView {
  const float4 *__restrict__ planar;
  const float *__restrict__ full;
  const bzr_host::Bvh4Node *__restrict__ nodes;
  const float4 *__restrict__ leaf;
  const bzr_host::Bvh4Node *__restrict__ nodes_near;
  const float4 *__restrict__ leaf_near;
  const bzr_host::Bvh4ObbNode *__restrict__ obb;
  const bzr_host::Bvh4ObbNode *__restrict__ obb_near;
  const float4 *__restrict__ always;  // patches without a proven gate region: gate-tested by every wave-segment
  const float4 *__restrict__ kids;       // AoS child records of nodes / nodes_near (bzr_mesh)
  const float4 *__restrict__ kids_near;
  const float4 *__restrict__ wide;       // 16 grandchild records per node (BZR_TRAV_WIDE)
  const float4 *__restrict__ wide_near;
  uint32_t n_always;
  uint32_t n;
  float s_max;
  float s_near;
  float ri;
};
struct LensSet {
  MeshView lens[kMaxLenses];
  uint32_t count;
};

__device__ __forceinline__ void store_hit(float *__restrict__ hits, uint32_t n, uint32_t i, const Hit &h,
                                          uint32_t patch) {
  hits[i] = h.t;
  hits[(size_t)1 * n + i] = h.point.x;
  hits[(size_t)2 * n + i] = h.point.y;
  hits[(size_t)3 * n + i] = h.point.z;
  hits[(size_t)4 * n + i] = h.cs;
  hits[(size_t)5 * n + i] = h.bary.x;
  hits[(size_t)6 * n + i] = h.bary.y;
  hits[(size_t)7 * n + i] = h.bary.z;
  hits[(size_t)8 * n + i] = h.normal.x;
  hits[(size_t)9 * n + i] = h.normal.y;
  hits[(size_t)10 * n + i] = h.normal.z;
  reinterpret_cast<uint32_t *>(hits)[(size_t)11 * n + i] = h.what;
  reinterpret_cast<uint32_t *>(hits)[(size_t)12 * n + i] = patch;
}

__device__ __forceinline__ Hit no_hit() {
  Hit h;
  h.t = FLT_MAX;
  h.what = kNone;
  h.point = h.bary = h.normal = mk(0.0f, 0.0f, 0.0f);
  h.cs = 0.0f;
  return h;
}

// Planar gate of BezierTriangle::intersect with cThis (reference/bezierTriangle.cpp:124-131),
// evaluated from the 64-byte scan record; same arithmetic as patch_intersect's first lines.
__device__ __forceinline__ bool planar_gate(float4 q0, float4 q1, float4 q2, float4 q3, f3 s, f3 d) {
#if BZR_GATE_FLAT
  // Branch-free: every term is evaluated and the conditions are combined with '&' (the same decision as
  // plane_ray's early outs below -- a lane with |cos| < 1e-5 fails whatever its t), so the walk runs no
  // exec-mask bookkeeping (s_and_saveexec / s_or exec per condition) on the scalar unit.
  const f3 n = mk(q0.x, q0.y, q0.z);
  const float cs = dot(d, n);
  const float t = div_rn(q0.w - dot(n, s), cs);
  const f3 ip = add(s, scale(d, t));
  const bool valid = (fabsf(cs) >= 0.00001f) & (t > 0.0f) & (fabsf(t) > -q1.x) & (fabsf(t) > q1.y);
  const float b0 = q1.z * ip.x + (q1.w * ip.y + q2.x * ip.z);
  const float b1 = q2.y * ip.x + (q2.z * ip.y + q2.w * ip.z);
  const float b2 = q3.x * ip.x + (q3.y * ip.y + q3.z * ip.z);
  return valid & (b0 >= 0.0f) & (b0 <= 1.0f) & (b1 >= 0.0f) & (b1 <= 1.0f) & (b2 >= 0.0f) & (b2 <= 1.0f);
#else
  f3 n = mk(q0.x, q0.y, q0.z);
  f3 ip;
  float ic, it;
  bool valid = plane_ray(n, q0.w, s, d, ip, ic, it);
  if (!(valid && fabsf(it) > -q1.x && fabsf(it) > q1.y)) return false;
  // row-major copy of M: rows (q1.z q1.w q2.x) (q2.y q2.z q2.w) (q3.x q3.y q3.z)
  float b0 = q1.z * ip.x + (q1.w * ip.y + q2.x * ip.z);
  float b1 = q2.y * ip.x + (q2.z * ip.y + q2.w * ip.z);
  float b2 = q3.x * ip.x + (q3.y * ip.y + q3.z * ip.z);
  return b0 >= 0.0f && b0 <= 1.0f && b1 >= 0.0f && b1 <= 1.0f && b2 >= 0.0f && b2 <= 1.0f;
#endif
}

// One iteration of the reference loop body: patch b with cThis, and on a follow-side result its
// named neighbour with cNone (reference/bezierMesh.cpp:212-216).  `src` gets the patch that hit.
template <bool kFast = false>
__device__ __forceinline__ Hit evaluate_patch(const MeshView &m, uint32_t b, f3 s, f3 d, uint32_t &src) {
  uint32_t idx = b;
  bool limitNone = false;
  Hit h;
  for (int pass = 0; pass < 2; ++pass) {
    Patch p = load_patch(m.full + (size_t)rec::kWords * idx);
    h = patch_intersect<false, kFast>(p, s, d, limitNone);
    if (pass == 0 && h.what <= kFollow2) {
      idx = __float_as_uint(m.full[(size_t)rec::kWords * idx + rec::kNeigh + h.what]);
      limitNone = true;
      continue;
    }
    break;
  }
  src = idx;
  return h;
}

// BezierMesh::intersect by the reference's brute-force scan: index order, strict-< minimum.
__device__ __forceinline__ Hit mesh_intersect_scan(const MeshView &m, f3 s, f3 d, uint32_t &patch) {
  Hit best = no_hit();
  patch = 0xFFFFFFFFu;
  for (uint32_t b = 0; b < m.n; ++b) {
    const float4 *q = m.planar + 4u * b;  // wave-uniform address -> scalar loads
    if (!planar_gate(q[0], q[1], q[2], q[3], s, d)) continue;
    uint32_t src;
    Hit h = evaluate_patch(m, b, s, d, src);
    if (h.what == kIntersect && h.t < best.t) {
      best = h;
      patch = src;
    }
  }
  return best;
}

// The refraction of BezierLens::refract after the mesh intersection.  Returns the status;
// o_s/o_d = refracted ray when status != NONE.
__device__ __forceinline__ uint32_t refract_hit(const Hit &h, float ri, f3 s, f3 d, uint32_t expected, f3 &o_s,
                                                f3 &o_d) {
  o_s = s;
  o_d = d;
  uint32_t st = BZR_RR_NONE;
  if (h.what == kIntersect) {
    st = h.cs < 0.0f ? BZR_RR_INSIDE : BZR_RR_OUTSIDE;
    o_s = h.point;
    float eta = st == BZR_RR_INSIDE ? div_rn(1.0f, ri) : ri;
    float s2 = eta * eta * (1.0f - h.cs * h.cs);
    if (s2 < 0.99f) {
      if (s2 > 1e-12f) {
        float sgn = st == BZR_RR_INSIDE ? 1.0f : -1.0f;
        f3 nn = scale(h.normal, sgn);
        float c1 = fabsf(h.cs);
        float c2 = sqrt_rn(1.0f - s2);
        o_d = normalized(add(scale(d, eta), scale(nn, eta * c1 - c2)));
      }
    } else {
      st = BZR_RR_NONE;
    }
  }
  return st == expected ? st : BZR_RR_NONE;
}

__device__ __forceinline__ void load_ray(const float *__restrict__ r, uint32_t n, uint32_t i, f3 &s, f3 &d) {
  s = mk(r[i], r[(size_t)n + i], r[(size_t)2 * n + i]);
  d = mk(r[(size_t)3 * n + i], r[(size_t)4 * n + i], r[(size_t)5 * n + i]);
}
// A pair's ray in the staged path: the chunk's 32-byte AoS copy (BZR_STAGED_AOS) or the SoA rows.
__device__ __forceinline__ void load_pair_ray(const float4 *__restrict__ aos, const float *__restrict__ r, uint32_t ld,
                                              uint32_t off, uint32_t i, f3 &s, f3 &d) {
#if BZR_STAGED_AOS
  (void)r;
  (void)ld;
  (void)off;
  const float4 a = aos[2u * i], b = aos[2u * i + 1u];
  s = mk(a.x, a.y, a.z);
  d = mk(a.w, b.x, b.y);
#else
  (void)aos;
  load_ray(r, ld, off + i, s, d);
#endif
}
__device__ __forceinline__ void store_ray(float *__restrict__ r, uint32_t n, uint32_t i, f3 s, f3 d) {
  r[i] = s.x;
  r[(size_t)n + i] = s.y;
  r[(size_t)2 * n + i] = s.z;
  r[(size_t)3 * n + i] = d.x;
  r[(size_t)4 * n + i] = d.y;
  r[(size_t)5 * n + i] = d.z;
}

// Diagnostic builds (BZR_DIAG_WALK2 / BZR_DIAG_NEWTON2): a copy of a value the compiler cannot see through,
// so a phase evaluated twice is not folded -- the marginal cost of its arithmetic, with identical results.
__device__ __forceinline__ f3 opaque(f3 v) {
  asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z));
  return v;
}

// ------------------------------------------------------------ culled path
__device__ __forceinline__ float safe_inv(float x) {
  // slab test only (no parity requirement): keep 1/d finite so (b - o) * inv never makes 0 * inf
  return 1.0f / (fabsf(x) < 1e-20f ? copysignf(1e-20f, x) : x);
}

// Slab test of the ray (origin s, per-axis reciprocal direction inv, sinv = s * inv) against a box.
// Conservative only (the gate-region boxes are padded for its rounding, bvh.cpp): with FMA each
// plane distance is one fma(lo, inv, -s*inv), error <= (|s| + |t|) * 2^-23 < the pad.
__device__ __forceinline__ bool slab(float4 lo, float4 hi, f3 s, f3 sinv, f3 inv) {
#if BZR_SLAB_FMA
  (void)s;
  float ax = __builtin_fmaf(lo.x, inv.x, -sinv.x), bx = __builtin_fmaf(hi.x, inv.x, -sinv.x);
  float ay = __builtin_fmaf(lo.y, inv.y, -sinv.y), by = __builtin_fmaf(hi.y, inv.y, -sinv.y);
  float az = __builtin_fmaf(lo.z, inv.z, -sinv.z), bz = __builtin_fmaf(hi.z, inv.z, -sinv.z);
#else
  (void)sinv;
  float ax = (lo.x - s.x) * inv.x, bx = (hi.x - s.x) * inv.x;
  float ay = (lo.y - s.y) * inv.y, by = (hi.y - s.y) * inv.y;
  float az = (lo.z - s.z) * inv.z, bz = (hi.z - s.z) * inv.z;
#endif
  float tnear = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
  float tfar = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
  return tnear <= tfar && tfar >= 0.0f;
}

// Ray vs oriented box (bvh.hpp Bvh4ObbNode): the slab test in the box's frame.  Culling only (no parity
// requirement): FMA and v_rcp_f32 are fine, their error is inside the box's doubled padding (bvh.cpp).
__device__ __forceinline__ float clamped_rcp(float x) {
  return __builtin_amdgcn_rcpf(fabsf(x) < 1e-20f ? copysignf(1e-20f, x) : x);
}
// q: one child's 64-byte record (bvh.hpp Bvh4ObbChild)
__device__ __forceinline__ bool obb_hit(const u32x16 &q, f3 s, f3 d) {
  const float rx = s.x - __uint_as_float(q[0]), ry = s.y - __uint_as_float(q[1]), rz = s.z - __uint_as_float(q[2]);
  float tnear = -FLT_MAX, tfar = FLT_MAX;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const float ux = __uint_as_float(q[3 + 3 * a]), uy = __uint_as_float(q[4 + 3 * a]), uz = __uint_as_float(q[5 + 3 * a]);
    const float o = __builtin_fmaf(rx, ux, __builtin_fmaf(ry, uy, rz * uz));
    const float dd = __builtin_fmaf(d.x, ux, __builtin_fmaf(d.y, uy, d.z * uz));
    const float h = __uint_as_float(q[12 + a]), inv = clamped_rcp(dd);
    const float t1 = (-h - o) * inv, t2 = (h - o) * inv;
    tnear = fmaxf(tnear, fminf(t1, t2));
    tfar = fminf(tfar, fmaxf(t1, t2));
  }
  return tnear <= tfar && tfar >= 0.0f;
}

// The children of BVH node `ref` (an AABB node, or an oriented-box node when ref has kObbFlag): their
// refs and which lanes' rays hit their boxes (wave-uniform fetch: two or four 64-byte scalar loads).
__device__ __forceinline__ void node_children(const bzr_host::Bvh4Node *nodes, const bzr_host::Bvh4ObbNode *obb,
                                              uint32_t ref, bool act, f3 s, f3 d, f3 sinv, f3 inv, bool (&hit)[4],
                                              uint32_t (&ch)[4]) {
  if (ref & bzr_host::kObbFlag) {  // one 64-byte scalar load per child (16 SGPRs live at a time)
    const cu32x16 *np = (const cu32x16 *)(uintptr_t)(obb + (ref & ~bzr_host::kObbFlag));
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const u32x16 q = np[c];
      ch[c] = q[15];
      hit[c] = act & (ch[c] != bzr_host::kEmptyChild) & obb_hit(q, s, d);
    }
    return;
  }
  // the whole 128-byte node in two 64-byte scalar loads and one wait (all words used unconditionally)
  const cu32x16 *np = (const cu32x16 *)(uintptr_t)(nodes + ref);
#if BZR_NODE_ASM
  // Both loads issued back to back, then one wait.  Left to the compiler, k_trace's walk got a wait
  // between the two (a scalar load's destination may still have a write pending from the previous
  // iteration's leaf load on some path, and scalar loads return out of order, so the second load waited
  // for everything): two L2 round trips per node.  Early-clobber outputs: the first load must not
  // overwrite the address pair the second one reads.
  u32x16 na, nb;
  asm volatile("s_load_dwordx16 %0, %2, 0x0\n\ts_load_dwordx16 %1, %2, 0x40\n\ts_waitcnt lgkmcnt(0)"
               : "=&s"(na), "=&s"(nb)
               : "s"(np));
#else
  const u32x16 na = np[0], nb = np[1];
#endif
  // words: lo.x[0..3] lo.y lo.z hi.x | hi.y hi.z child[0..3] pad
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float4 lo = make_float4(__uint_as_float(na[c]), __uint_as_float(na[4 + c]), __uint_as_float(na[8 + c]), 0.0f);
    const float4 hi = make_float4(__uint_as_float(na[12 + c]), __uint_as_float(nb[c]), __uint_as_float(nb[4 + c]), 0.0f);
    ch[c] = nb[8 + c];
    hit[c] = act & (ch[c] != bzr_host::kEmptyChild) & slab(lo, hi, s, sinv, inv);
#if BZR_DIAG_WALK2
    hit[c] &= slab(lo, hi, s, opaque(sinv), opaque(inv));
#endif
  }
}

// Per-segment pipeline of the culled path (one BezierMesh::intersect per ray of a chunk of n rays;
// external arrays -- rays, alive, outputs -- are indexed off + i with row stride ld):
//   k_traverse  BVH walk, exact planar gate -> up to kMaxCand candidates per ray, a per-patch
//               histogram (rank of each (ray, patch) pair within its patch bucket) and the list
//               of rays that need the full scan (list/stack overflow, origin beyond s_max)
//   scan        exclusive sum over the buckets of (dense chunks << 32 | sparse pairs) (bucket_split;
//               hipCUB or k_scan_small) -> each bucket's dense chunk and sparse offsets, the totals
//   k_place     (ray, patch) pair records into their bucket's dense chunks or the sparse region (8-byte
//               records: the Newton stage reads the ray itself from the ray array -- neighbouring rays,
//               mostly cached -- instead of a 32-byte copy travelling with the pair); marks the padded
//               lanes of each bucket's last dense chunk; clears the histogram for the next segment
//   k_newton    the Newton stage over the dense chunks: one patch per chunk, its record in scalar
//               registers (uniform loads); hits go to the ray's list slot and a per-ray 64-bit atomicMin
//               on (t order, patch, slot)
//   k_newton_lane  the sparse region: one pair per lane, the lane's own patch record
//   k_resolve   follow-side results: the named neighbour with cNone, per lane; then the reference's
//               in-order scan for the overflow list, sliced over patches -> key
//   k_finish    winner -> BezierIntersection / refraction (overflow rays: their winner re-evaluated)
// For one ray (t order, patch, slot) orders like (t, scanned patch index): the atomicMin winner is the
// reference's strict-< in-order winner (record()).
// BZR_ROWS_DIRECT: where the Newton stage writes an intersect segment's hits (RowOut::rows non-null: the caller's
// hit rows, see record_row) instead of the list slots.
struct RowOut {
  float *rows = nullptr;        // [13][ld] hit rows, ray i at off + i
  uint32_t ld = 0, off = 0;
  uint32_t *count = nullptr;    // Work::count (kDirty)
  uint32_t *dirty = nullptr;    // [chunk] rays whose row two improving pairs may have written in either order
  uint32_t *ndirty = nullptr;   // Work::ctr + 4
};
struct Work {
  uint32_t *ctr;     // [0] follow count, [1] overflow count, [2] rays traced, [3] pairs listed, [4] dirty rows
  uint32_t *hist;    // [nb + 1] pair counts per patch (hist[nb] = 0); 256 bytes after ctr
  unsigned long long *offs;  // [nb + 1] exclusive prefix of bucket_split(hist); offs[nb] = the totals
  uint32_t *cand;    // [kMaxCand][n]
  uint32_t *rank;    // [kMaxCand][n]
  uint32_t *count;   // [n] list length, | kOverflow: the full scan
  unsigned long long *key;  // [n]
  float *slot;       // [kMaxCand][n] x kSlotWords: the hit of ray i's list slot j at j * n + i (AoS, 48 bytes)
  uint2 *pairs;      // [cap + 64 (nb + 1)] pair records (ray | j << 26, patch): dense chunks, then the sparse
                     // region; a follow request adds its side << 30 to the patch word
  uint32_t *fol;     // [cap] follow requests: pair indices
  uint32_t *ovf;     // [n]
  uint32_t *dirty;   // [n] BZR_ROWS_DIRECT: rays whose hit row k_finish_ovf evaluates again
  unsigned long long *amask;  // BZR_TRAV_ABLOCK 3: [n / 256][kAmaskWords] always-listed patches kept per 256 rays
  RowOut ro;         // BZR_ROWS_DIRECT (intersect segments): the Newton stage's direct row writes
  float4 *aos;       // [2 * chunk] the chunk's rays as 32-byte records (BZR_STAGED_AOS)
  void *cub;
  size_t cub_bytes;
  uint32_t cap;      // kMaxCand * chunk
  uint32_t hbase;    // BZR_TRAV_HYBRID: pair index of the in-wave follow requests' records (j * n + ray past it)
  uint32_t hyb_t;    // BZR_TRAV_HYBRID: lanes a leaf's gate must pass for its Newton pass to run in the walking wave
};
constexpr uint32_t kSlotWords = 12;  // t, point, cos, bary, normal, source patch

enum OutMode { kModeHits = 0, kModeRefract = 1, kModeStage = 2 };
struct Out {
  float *hits;               // kModeHits: SoA [13][ld]
  float *rays;               // kModeRefract: output rays; kModeStage: rays in flight (in place)
  const uint32_t *expected;  // per ray, or null -> expected_all
  uint32_t expected_all;
  uint32_t *status;
  uint32_t *segments;        // kModeStage, optional
  float ri;
  uint32_t first;            // kModeStage: the chain's first stage -- every ray is alive, its input comes
                             // from the caller's rays and its ray / status / segments are all written here
};

template <int kMode>
__device__ __forceinline__ void emit(const Out &o, uint32_t ld, uint32_t gi, f3 s, f3 d, const Hit &h, uint32_t patch) {
  if (kMode == kModeHits) {
    store_hit(o.hits, ld, gi, h, patch);
  } else {
    f3 os, od;
    uint32_t st = refract_hit(h, o.ri, s, d, o.expected ? o.expected[gi] : o.expected_all, os, od);
    if (kMode == kModeRefract || st != BZR_RR_NONE || (kMode == kModeStage && o.first)) {
      if (st == BZR_RR_NONE) {
        os = s;
        od = d;
      }
      store_ray(o.rays, ld, gi, os, od);
    }
    o.status[gi] = st;
    if (kMode == kModeStage && o.segments) o.segments[gi] = o.first ? 1u : o.segments[gi] + 1u;
  }
}

// Monotone map of t to uint32 (IEEE total order; -0 canonicalised to +0 so they tie like `<`).
__device__ __forceinline__ uint32_t t_order(float t) {
  uint32_t u = __float_as_uint(t == 0.0f ? 0.0f : t);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Number of lanes below this one in `mask`.
__device__ __forceinline__ uint32_t popc64_(unsigned long long m) { return (uint32_t)__popcll(m); }
__device__ __forceinline__ bool lane_bit64(unsigned long long m, uint32_t lane) { return ((m >> lane) & 1ull) != 0ull; }
__device__ __forceinline__ uint32_t lanes_below(unsigned long long mask) {
  return __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(mask), 0u));
}

// One intersecting pair result: its slot, then the ray's running (t, pair) minimum.  t that cannot
// beat the reference's initial FLT_MAX (NaN, FLT_MAX, +inf) is dropped; -0 ties with +0.
// A staged hit of ray `ray`'s list slot j (candidate patch b; the hit itself may be b's neighbour src after a
// follow): its 48-byte record goes to slot j * n + ray, and the ray's key takes the lexicographic minimum of
// (t order, b, j).  A ray's candidates are distinct patches, so for one ray that orders like the reference's
// (t, scanned patch index) with strict < -- the follow side's hit ranks at its candidate's position, as in
// reference/bezierMesh.cpp:206-227 (oracle orc_mesh_intersect).
// BZR_RECORD_RET (default 1; 0 = the round-4 record): take the key's old value back and write the slot only when
// this pair is the ray's best so far -- the final key's pair always wrote its slot (the minimum is unique), later
// losers skip their 48 bytes; the wave then waits for the atomic before its stores.  cfg5 per 8 M-ray chunk:
// k_newton writes 542 -> 450 MB, k_resolve 41 -> 33 MB (profiles/r05_cfg5_staged_recret.txt); time within noise
// (lone cfg5 +0.4 %, cfg3 -0.1 %; frames in flight cfg5 +0.3 %, cfg3 +1.1 %; profiles/r05_ab_record_ret.jsonl).
#ifndef BZR_RECORD_RET
#define BZR_RECORD_RET 1
#endif
__device__ __forceinline__ void write_slot(float *__restrict__ slot, uint32_t n, uint32_t ray, uint32_t j, const Hit &h,
                                           uint32_t src) {
  float4 *r = reinterpret_cast<float4 *>(slot) + (size_t)3 * ((size_t)j * n + ray);  // AoS: 48 bytes per slot
  r[0] = make_float4(h.t, h.point.x, h.point.y, h.point.z);
  r[1] = make_float4(h.cs, h.bary.x, h.bary.y, h.bary.z);
  r[2] = make_float4(h.normal.x, h.normal.y, h.normal.z, __uint_as_float(src));
}
__device__ __forceinline__ void record(float *__restrict__ slot, uint32_t n, uint32_t ray, uint32_t j, uint32_t b,
                                       const Hit &h, uint32_t src, unsigned long long *key) {
  if (!(h.t < FLT_MAX)) return;
  const unsigned long long k = ((unsigned long long)t_order(h.t) << 32) | (b << 6) | j;
#if BZR_RECORD_RET
  if (!(k < atomicMin(key, k))) return;
#endif
  write_slot(slot, n, ray, j, h, src);
#if !BZR_RECORD_RET
  atomicMin(key, k);
#endif
}

// BZR_ROWS_DIRECT (A/B knob, default 0): an intersect segment's Newton stage writes a pair's hit straight into the caller's
// hit rows instead of its 48-byte list slot, and k_finish only writes the misses' rows -- it no longer reads a slot
// and rewrites every hit row (cfg5: k_finish 822 -> ~260 MB per 8 M-ray chunk).  Ordering: a pair whose key improves
// the ray's (the returning atomicMin) writes its 13 words write-through (sc1: the line leaves the XCD's L2 for the
// memory side, MI355X_MICROARCH.md visibility table), waits for them (vmcnt(0)) and reads the key again at the
// coherence point (a second atomicMin).  Still its own key: any later improvement's atomic comes after that read, so
// its stores land after these and its row is the final one.  Changed: another pair improved meanwhile and the two
// writes may have landed in either order, so the ray is marked dirty (kDirty in its count, once, and listed) and
// k_finish_ovf evaluates its final winner again from the key (patch b, cThis, then the follow side's neighbour with
// cNone: the sequence that produced the key, same bits).  Misses are written by k_finish, overflow rays by
// k_finish_ovf, as before.  Measured (profiles/r06_ab_rows_direct.jsonl; all GPU tests bit-identical with it on):
// 0.43 % of cfg5's rays dirty; lone frames cfg5 -0.3 % (k_finish 1.17 -> 0.64 ms per frame, but k_newton +0.25 and
// k_resolve +0.13: the drain stalls the VALU-bound waves), cfg3 +3 %; at bench level, frames in flight, cfg5 6 758 ->
// 6 517 Mrays/s and cfg3 9 695 -> 9 433 -- the write-through stores cost more than k_finish's HBM bytes save.  Checking
// a row at the lane's next step instead (its stores long done): 3.4x the dirty rows and slower.  Not kept.
#ifndef BZR_ROWS_DIRECT
#define BZR_ROWS_DIRECT 0
#endif
constexpr uint32_t kDirty = 0x10000u;  // count flag (above kOverflow): the hit row is evaluated again
__device__ __forceinline__ void store_wt(float *p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
// Record a lane's hit (wr) -- ray `ray`'s list slot j, candidate patch b, from patch src -- into its row.
__device__ __forceinline__ void row_step(const RowOut &ro, unsigned long long *key, bool wr, uint32_t ray, uint32_t j,
                                         uint32_t b, const Hit &h, uint32_t src) {
  wr = wr && h.t < FLT_MAX;
  const unsigned long long kn = ((unsigned long long)t_order(h.t) << 32) | (b << 6) | j;
  if (wr) wr = kn < atomicMin(&key[ray], kn);
  if (!__any(wr)) return;
  if (wr) {
    const size_t ld = ro.ld, i = (size_t)ro.off + ray;
    float *r = ro.rows;
    store_wt(r + i, h.t);
    store_wt(r + ld + i, h.point.x);
    store_wt(r + 2 * ld + i, h.point.y);
    store_wt(r + 3 * ld + i, h.point.z);
    store_wt(r + 4 * ld + i, h.cs);
    store_wt(r + 5 * ld + i, h.bary.x);
    store_wt(r + 6 * ld + i, h.bary.y);
    store_wt(r + 7 * ld + i, h.bary.z);
    store_wt(r + 8 * ld + i, h.normal.x);
    store_wt(r + 9 * ld + i, h.normal.y);
    store_wt(r + 10 * ld + i, h.normal.z);
    store_wt(r + 11 * ld + i, __uint_as_float(kIntersect));
    store_wt(r + 12 * ld + i, __uint_as_float(src));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the rows have reached the memory side
  if (wr && atomicMin(&key[ray], kn) != kn && !(atomicOr(&ro.count[ray], kDirty) & kDirty))
    ro.dirty[atomicAdd(ro.ndirty, 1u)] = ray;
}

// Word group g of a 64-byte leaf record (planar record, patch index in the last word): q0..q3 of the gate.
__device__ __forceinline__ float4 leaf_q(const u32x16 &r, int g) {
  return make_float4(__uint_as_float(r[4 * g]), __uint_as_float(r[4 * g + 1]), __uint_as_float(r[4 * g + 2]),
                     g == 3 ? 0.0f : __uint_as_float(r[4 * g + 3]));
}

// The always list (bvh.hpp Bvh::always): patches without a proven gate region, gate-tested by every
// wave-segment.  Record k = kAlwaysQuads float4: the 64-byte leaf record, then the wedge pre-test words.
constexpr uint32_t kAlwaysQuads = 8;
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(4))) const u32x8 cu32x8;

// The planar gate of always-listed patch k for the active lanes, behind two exact pre-tests that only
// reject lanes whose gate surely fails (the rejections are strict comparisons, so NaN rejects nothing):
//   1. t = num / cs must be > 0 with |cs| >= 1e-5: decided from the signs of num and cs (no division);
//   2. the float plane point must lie in the patch's wedge (bvh.cpp always_wedge): w.p~ within
//      [L - B|p~| - C(|s|+|p~|), H + ...] at p~ = s + d (num x rcp(cs)) -- ~3 % of cfg5's pairs pass.
// Only then the exact gate (the division and fl(M p)), so the always list costs ~25 VALU per pair
// instead of ~50.  Same candidates as the gate alone.
__device__ __forceinline__ bool always_gate_rec(const u32x16 &r, const u32x8 &wq, bool act, f3 s, f3 d, uint32_t &patch) {
  patch = r[15];
  const float4 q0 = leaf_q(r, 0);
  const f3 n = mk(q0.x, q0.y, q0.z);
  const float cs = dot(d, n), num = q0.w - dot(n, s);
  bool keep = act & (fabsf(cs) >= 0.00001f) & (((num > 0.0f) & (cs > 0.0f)) | ((num < 0.0f) & (cs < 0.0f)));
  // NaN num / cs: keep (the gate itself decides)
  keep |= act & ((num != num) | (cs != cs));
  if (!__any(keep)) return false;
  const float tt = num * __builtin_amdgcn_rcpf(cs);
  const f3 p = mk(__builtin_fmaf(d.x, tt, s.x), __builtin_fmaf(d.y, tt, s.y), __builtin_fmaf(d.z, tt, s.z));
  const float pm = fmaxf(fmaxf(fabsf(p.x), fabsf(p.y)), fabsf(p.z)), sm = fmaxf(fmaxf(fabsf(s.x), fabsf(s.y)), fabsf(s.z));
  const float w = __builtin_fmaf(__uint_as_float(wq[0]), p.x, __builtin_fmaf(__uint_as_float(wq[1]), p.y, __uint_as_float(wq[2]) * p.z));
  const float slack = __builtin_fmaf(__uint_as_float(wq[5]), pm, __uint_as_float(wq[6]) * (sm + pm));
  keep &= !(w > __uint_as_float(wq[4]) + slack) & !(w < __uint_as_float(wq[3]) - slack);
  if (!__any(keep)) return false;
  return keep & planar_gate(q0, leaf_q(r, 1), leaf_q(r, 2), leaf_q(r, 3), s, d);
}
__device__ __forceinline__ bool always_gate(const float4 *always, uint32_t k, bool act, f3 s, f3 d, uint32_t &patch) {
  const u32x16 r = *((const cu32x16 *)(uintptr_t)(always + (size_t)kAlwaysQuads * k));
  const u32x8 wq = *((const cu32x8 *)(uintptr_t)(always + (size_t)kAlwaysQuads * k + 4));
  return always_gate_rec(r, wq, act, s, d, patch);
}
// The same gate from a record staged in LDS (BZR_TRAV_ALDS): quads 0-3 the leaf record, 4-5 the wedge words.
__device__ __forceinline__ bool always_gate_lds(const float4 *q, bool act, f3 s, f3 d, uint32_t &patch) {
  u32x16 r;
  u32x8 wq;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float4 v = q[k];
    r[4 * k] = __float_as_uint(v.x);
    r[4 * k + 1] = __float_as_uint(v.y);
    r[4 * k + 2] = __float_as_uint(v.z);
    r[4 * k + 3] = __float_as_uint(v.w);
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float4 v = q[4 + k];
    wq[4 * k] = __float_as_uint(v.x);
    wq[4 * k + 1] = __float_as_uint(v.y);
    wq[4 * k + 2] = __float_as_uint(v.z);
    wq[4 * k + 3] = __float_as_uint(v.w);
  }
  return always_gate_rec(r, wq, act, s, d, patch);
}

// Wave-level pre-test of the always list.  The active rays of a wave form a bundle: origins in the box
// [slo, shi], directions in [dlo, dhi] (wave min / max, once per segment).  Lane j tests always-listed
// patch 64 b + j against the whole bundle in interval arithmetic: the ranges of cs = n.d and num = c - n.s
// over the bundle (widened for the lanes' own float dot products), the plane distance t = num / cs over
// the corners (t > 0 and |cs| >= 1e-5 needed), the plane points P = S + D T, and the wedge of
// always_gate: w.P against [L - B|P| - ..., H + ...].  A patch whose interval misses is gate-failed by every
// ray of the wave; only the survivors (a ballot mask, one bit per patch) take the per-lane tests -- 64
// patches per VALU instruction instead of one.  Every margin rounds outward (u = 2^-24): the lanes' dot
// products 8u, the corner quotients 6u, the points 8u, the wedge product and the bound 64u of (|S| + |P|).
// Non-finite bundles (or t ranges beyond 1e30) keep everything.
// The bundle lives in LDS (13 words per wave: slo, shi, dlo, dhi, finite flag) and is read at its points of
// use (volatile: not hoisted): in registers it stayed live across the fused kernel's walk and cost two
// waves per SIMD of occupancy (69 -> 98 VGPRs).
// Wave min / max by ds_swizzle (xor within 32 lanes; the pattern is an immediate, so no lane-index
// registers -- __shfl_xor's bpermute addresses were hoisted and kept 5 VGPRs live across the whole kernel)
// and the two halves combined through readlane: the result is uniform.
template <int kXor>
__device__ __forceinline__ float swz(float v) {
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x1F | (kXor << 10)));
}
__device__ __forceinline__ float halves(float v, bool mx) {
  const float a = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  return mx ? fmaxf(a, b) : fminf(a, b);
}
__device__ __forceinline__ float wave_minf(float v) {
  v = fminf(v, swz<1>(v));
  v = fminf(v, swz<2>(v));
  v = fminf(v, swz<4>(v));
  v = fminf(v, swz<8>(v));
  v = fminf(v, swz<16>(v));
  return halves(v, false);
}
__device__ __forceinline__ float wave_maxf(float v) {
  v = fmaxf(v, swz<1>(v));
  v = fmaxf(v, swz<2>(v));
  v = fmaxf(v, swz<4>(v));
  v = fmaxf(v, swz<8>(v));
  v = fmaxf(v, swz<16>(v));
  return halves(v, true);
}
// The 12 reductions one after another (a loop that is not unrolled), each stored to the wave's LDS words as
// soon as it is done, so only one is in registers at a time; word 12 = 1 when every box bound is finite
// (false also for an empty bundle, whose boxes are +-inf).  Words 13..21: bundle_setup_dpp.
constexpr uint32_t kBundleWords = 22;
__device__ __forceinline__ void bundle_to_lds(bool act, f3 s, f3 d, float *out, uint32_t lane) {
  const float inf = __builtin_inff();
  float m = 0.0f;
#pragma unroll 1
  for (uint32_t k = 0; k < 12u; ++k) {
    const uint32_t a = k % 3u;
    const f3 v = k < 6u ? s : d;
    const float x = a == 0u ? v.x : (a == 1u ? v.y : v.z);
    const bool lo = (k / 3u) % 2u == 0u;
    const float r = lo ? wave_minf(act ? x : inf) : wave_maxf(act ? x : -inf);
    m = fmaxf(m, fabsf(r));
    if (lane == 0u) out[k] = r;
  }
  if (lane == 0u) out[12] = m <= 1e30f ? 1.0f : 0.0f;
  __builtin_amdgcn_wave_barrier();  // the words are read back by every lane of this wave
}
// Wave min / max with DPP row shifts and row broadcasts (no LDS round trips): lane 63 ends with the result,
// read back as a uniform value.  Lanes shifted in from outside a row contribute the identity.  The floats are
// reduced as order-preserving integers (sign-magnitude flipped to two's complement): a float fminf / fmaxf
// step costs a DPP move, two canonicalising v_max and the min (IEEE mode), an integer step is one
// v_min_i32 / v_max_i32 with the DPP operand folded in.  NaN lanes contribute the identity (as fminf / fmaxf
// ignore them); -0 orders below +0 (either is a valid bound).
__device__ __forceinline__ int float_order(float x) {
  const int b = __float_as_int(x);
  return b ^ ((b >> 31) & 0x7FFFFFFF);
}
// The 12 bundle reductions in lockstep (step k of all twelve, then step k + 1): each DPP read is then 12
// instructions behind the write it reads, so no s_nop hazard padding between the steps.  kMaxMask bit i:
// value i is reduced by max (else min).
template <uint32_t kMaxMask>
__device__ __forceinline__ void wave_reduce12_dpp(const float (&x)[12], float (&out)[12]) {
  int v[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const int id = ((kMaxMask >> i) & 1u) ? INT_MIN : INT_MAX;
    v[i] = x[i] == x[i] ? float_order(x[i]) : id;
  }
#define BZR_DPP_STEP(ctrl, rows)                                                        \
  _Pragma("unroll") for (int i = 0; i < 12; ++i) {                                     \
    const bool mx = (kMaxMask >> i) & 1u;                                              \
    const int o = __builtin_amdgcn_update_dpp(mx ? INT_MIN : INT_MAX, v[i], ctrl, rows, 0xF, false); \
    v[i] = mx ? max(v[i], o) : min(v[i], o);                                           \
  }
  BZR_DPP_STEP(0x111, 0xF)  // row_shr:1
  BZR_DPP_STEP(0x112, 0xF)  // row_shr:2
  BZR_DPP_STEP(0x114, 0xF)  // row_shr:4
  BZR_DPP_STEP(0x118, 0xF)  // row_shr:8: lane 15 of each row holds its row's result
  BZR_DPP_STEP(0x142, 0xA)  // row_bcast:15 into rows 1 and 3
  BZR_DPP_STEP(0x143, 0xC)  // row_bcast:31 into rows 2 and 3: lane 63 holds the wave's result
#undef BZR_DPP_STEP
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const int r = __builtin_amdgcn_readlane(v[i], 63);
    out[i] = __int_as_float(r ^ ((r >> 31) & 0x7FFFFFFF));  // (the map is its own inverse)
  }
}
// The whole bundle with the 12 reductions side by side in DPP form, written by lane 0: words 0..12 as
// bundle_to_lds, and for the bundle walk 13..21 -- per axis rl = 1 / Dl', rh = 1 / Dh' and mixed = 1 when
// Dl' < 0 < Dh', where Dl' <= Dl and Dh' >= Dh are the direction bounds moved away from zero (|D'| >= 1e-20:
// a wider direction box, so a superset of the rays).
__device__ __forceinline__ float bundle_setup_dpp(bool act, f3 s, f3 d, float *out, uint32_t lane) {
  const float inf = __builtin_inff();
  const float x[12] = {act ? s.x : inf,  act ? s.y : inf,  act ? s.z : inf,  act ? s.x : -inf,
                       act ? s.y : -inf, act ? s.z : -inf, act ? d.x : inf,  act ? d.y : inf,
                       act ? d.z : inf,  act ? d.x : -inf, act ? d.y : -inf, act ? d.z : -inf};
  float r[12];
  wave_reduce12_dpp<0xE38u>(x, r);  // max: values 3, 4, 5, 9, 10, 11
  if (lane == 0u) {
    float m = 0.0f;
#pragma unroll
    for (int k = 0; k < 12; ++k) {
      out[k] = r[k];
      m = fmaxf(m, fabsf(r[k]));
    }
    out[12] = m <= 1e30f ? 1.0f : 0.0f;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const float dl = r[6 + a], dh = r[9 + a];
      const float lo = dl > 1e-20f ? dl : fminf(dl, -1e-20f), hi = dh < -1e-20f ? dh : fmaxf(dh, 1e-20f);
      out[13 + a] = 1.0f / lo;
      out[16 + a] = 1.0f / hi;
      out[19 + a] = (lo < 0.0f && hi > 0.0f) ? 1.0f : 0.0f;
    }
  }
  __builtin_amdgcn_wave_barrier();
  // the walk choice's width measure (uniform): the widest direction interval (bvh.cpp bundle_spread_h)
  return fmaxf(fmaxf(r[9] - r[6], r[10] - r[7]), r[11] - r[8]);
}
// Wave-bundle box test (the bundle walk): false only when no ray s + t d, t >= 0, with s in [Sl, Sh] and d in
// [Dl', Dh'] (per axis, so a superset of the wave's active rays) meets the box.  On axis a the reachable
// coordinates at time t are [Sl + t Dl', Sh + t Dh'], which meet [lo, hi] iff Sl + t Dl' <= hi and
// Sh + t Dh' >= lo: with A = (hi - Sl) / Dl' and B = (lo - Sh) / Dh', t in [B, A] when 0 < Dl' (and B <= A
// whenever A >= 0, so [min, max] decides alike), t in [A, B] when Dh' < 0 (same), and t >= max(A, B) when
// the axis is mixed.  A and B carry at most ~3u relative rounding (one subtraction, the rounded reciprocal,
// one product); the bounds are widened by 8u relative + 2^-126 before tnear <= tfar and tfar >= 0, and a
// NaN keeps the box.  The per-lane walk's boxes are padded for the lanes' own float slab test; this test
// is conservative against the exact rays, so it keeps every box an exact ray of the wave meets (host
// mirror: bvh.cpp bundle_box_h, checked by tests/test_culling_conservative.py).
__device__ __forceinline__ bool bundle_box(const float *B, float4 lo, float4 hi) {
  float tn = -__builtin_inff(), tf = __builtin_inff();
  const float l3[3] = {lo.x, lo.y, lo.z}, h3[3] = {hi.x, hi.y, hi.z};
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const float A = (h3[a] - B[a]) * B[13 + a], Bq = (l3[a] - B[3 + a]) * B[16 + a];
    const float mn = fminf(A, Bq), mx = fmaxf(A, Bq);
    const bool mix = B[19 + a] > 0.0f;
    tn = fmaxf(tn, mix ? mx : mn);
    tf = fminf(tf, mix ? __builtin_inff() : mx);
  }
  tn -= fabsf(tn) * 0x1p-21f + 0x1p-126f;
  tf += fabsf(tf) * 0x1p-21f + 0x1p-126f;
  return !(B[12] > 0.0f) | (!(tn > tf) & !(tf < 0.0f));
}
// One batch of the bundle walk (k_trace and k_traverse): the k <= 16 axis-aligned nodes on top of the wave's
// LDS stack `stk` (the top one is axis-aligned; an oriented-box node below it ends the batch), lane 4 q + c
// taking node q's child c from the AoS child records `kids`.  Hit inner children are pushed, hit leaf slots
// written to `pend` (returns how many).  Returns with `full` set when the stack could not take every hit
// child (those subtrees are dropped: the caller sends its active lanes to the full scan).
// kSlots = 16: the same over the two-level records `wide` (4 nodes per batch, lane 16 q + s taking slot s of
// node q), so a batch descends two levels of the tree.
template <int kCap, uint32_t kSlots = 4>
__device__ __forceinline__ uint32_t bundle_batch(const float4 *kids, uint32_t *stk, int &sp, uint32_t *pend,
                                                 const float *B, uint32_t lane, bool &full, uint32_t &knodes,
                                                 uint32_t base = 0u) {
  // (the lane index laundered: lane-derived addresses hoisted out of the walk stayed live across the Newton
  // passes of k_trace and cost it a wave of occupancy)
  asm volatile("" : "+v"(lane));
  constexpr uint32_t kShift = kSlots == 64u ? 6u : (kSlots == 16u ? 4u : 2u);
  constexpr int kNodes = 64 / (int)kSlots;
  const uint32_t q = lane >> kShift, c = lane & (kSlots - 1u);
  // at most (kCap - sp) / (kSlots - 1) nodes (at least one), so their <= kSlots children each fit: the stack
  // overflows only from a nearly full stack (a wide bundle; the walk choice sends those to the per-lane walk)
  const int room = (kCap - sp) / (int)(kSlots - 1u), avail = sp < kNodes ? sp : kNodes;
  const uint32_t kmax = (uint32_t)(avail < room ? avail : (room > 1 ? room : 1));
  const uint32_t nd = q < kmax ? stk[sp - 1 - (int)q] : 0u;
  const unsigned long long ob = __ballot(c == 0u && q < kmax && (nd & bzr_host::kObbFlag));
  const uint32_t k = ob ? (uint32_t)__builtin_ctzll(ob) >> kShift : kmax;
  const bool slot = q < k;
  const float4 *kp = kids + ((size_t)(slot ? nd : 0u) * kSlots + c) * 2u;
  const float4 lo = kp[0], hi = kp[1];
  const uint32_t ref = __float_as_uint(lo.w);
  const bool hit = slot && ref != bzr_host::kEmptyChild && bundle_box(B, lo, hi);
  const bool isleaf = (ref & bzr_host::kLeafFlag) != 0u;
  const unsigned long long lm = __ballot(hit && isleaf), im = __ballot(hit && !isleaf);
  knodes = k;
  sp -= (int)k;
  const int below = (int)lanes_below(im);
  if (hit && !isleaf && sp + below < kCap) stk[sp + below] = ref;
  const int ni = (int)popc64_(im);
  full = sp + ni > kCap;
  sp = full ? kCap : sp + ni;
  if (hit && isleaf) pend[base + lanes_below(lm)] = ref & ~bzr_host::kLeafFlag;
  return popc64_(lm);
}
// Interval of n.x over x in [lo, hi] (n fixed).
__device__ __forceinline__ void ivdot(f3 n, f3 lo, f3 hi, float &a, float &b) {
  a = (n.x >= 0.0f ? n.x * lo.x : n.x * hi.x) + (n.y >= 0.0f ? n.y * lo.y : n.y * hi.y) + (n.z >= 0.0f ? n.z * lo.z : n.z * hi.z);
  b = (n.x >= 0.0f ? n.x * hi.x : n.x * lo.x) + (n.y >= 0.0f ? n.y * hi.y : n.y * lo.y) + (n.z >= 0.0f ? n.z * hi.z : n.z * lo.z);
}
__device__ __forceinline__ float absmax(float lo, float hi) { return fmaxf(fabsf(lo), fabsf(hi)); }
// false: no ray of the bundle (LDS words bl) can pass always-listed patch k's gate.
__device__ __forceinline__ bool always_bundle_keep_rec(float4 q0, float4 w0, float4 w1, const float *bl) {
  const float *B = bl;
  if (!(B[12] > 0.0f)) return true;
  constexpr float u = 0x1p-24f;
  const f3 n = mk(q0.x, q0.y, q0.z);
  float csl, csh, nsl, nsh;
  ivdot(n, mk(B[6], B[7], B[8]), mk(B[9], B[10], B[11]), csl, csh);
  ivdot(n, mk(B[0], B[1], B[2]), mk(B[3], B[4], B[5]), nsl, nsh);
  const float mc = 8.0f * u * (fabsf(n.x) * absmax(B[6], B[9]) + fabsf(n.y) * absmax(B[7], B[10]) + fabsf(n.z) * absmax(B[8], B[11]));
  const float ms = 8.0f * u * (fabsf(n.x) * absmax(B[0], B[3]) + fabsf(n.y) * absmax(B[1], B[4]) + fabsf(n.z) * absmax(B[2], B[5]) + fabsf(q0.w));
  csl -= mc;
  csh += mc;
  const float numl = (q0.w - nsh) - ms, numh = (q0.w - nsl) + ms;
  if (csl > -0.00001f && csh < 0.00001f) return false;  // |cs| < 1e-5 for every ray
  if (!(csl > 0.0f || csh < 0.0f)) return true;          // cs of either sign: t unbounded
  const float r1 = __builtin_amdgcn_rcpf(csl), r2 = __builtin_amdgcn_rcpf(csh);
  const float a1 = numl * r1, a2 = numl * r2, a3 = numh * r1, a4 = numh * r2;
  float tlo = fminf(fminf(a1, a2), fminf(a3, a4)), thi = fmaxf(fmaxf(a1, a2), fmaxf(a3, a4));
  tlo -= 6.0f * u * fabsf(tlo);
  thi += 6.0f * u * fabsf(thi);
  if (!(thi <= 1e30f)) return true;  // huge or NaN: no bound
  if (thi <= 0.0f) return false;     // t > 0 for no ray
  tlo = fmaxf(tlo, 0.0f);
  // plane points P = S + D T and the wedge w.P, one axis at a time
  float wlo = 0.0f, whi = 0.0f, pm0 = 0.0f, smax = 0.0f, wabs = 0.0f;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const float dl = B[6 + a], dh = B[9 + a], sl = B[a], sh = B[3 + a];
    const float x1 = dl * tlo, x2 = dl * thi, x3 = dh * tlo, x4 = dh * thi;
    const float pl = sl + fminf(fminf(x1, x2), fminf(x3, x4)), ph = sh + fmaxf(fmaxf(x1, x2), fmaxf(x3, x4));
    const float wa = a == 0 ? w0.x : (a == 1 ? w0.y : w0.z);
    wlo += wa >= 0.0f ? wa * pl : wa * ph;
    whi += wa >= 0.0f ? wa * ph : wa * pl;
    wabs += fabsf(wa);
    pm0 = fmaxf(pm0, absmax(pl, ph));
    smax = fmaxf(smax, absmax(sl, sh));
  }
  // the points' own rounding e on every axis moves w.P by at most |w|_1 e; the wedge product's and the
  // bound's rounding are inside 64 u (|S| + |P|)
  const float e = 8.0f * u * (smax + pm0);
  const float pmax = pm0 + e;
  wlo -= wabs * e;
  whi += wabs * e;
  const float slack = w1.y * pmax + (w1.z + 64.0f * u) * (smax + pmax);
  return !(wlo > w1.x + slack) & !(whi < w0.w - slack);
}
__device__ __forceinline__ bool always_bundle_keep(const float4 *always, uint32_t k, uint32_t n_always, const float *bl) {
  if (k >= n_always) return false;
  const float4 *a = always + (size_t)kAlwaysQuads * k;
  return always_bundle_keep_rec(a[0], a[4], a[5], bl);
}

// Wave-level pre-test of a tree leaf's planar gate (the bundle walk's queued leaves, one per lane): false
// only when no ray of the bundle (LDS words bl: origins [Sl, Sh], directions [Dl, Dh]) can pass the gate of
// planar record q0..q3 (planar_gate).  The interval steps and margins of always_bundle_keep (cs and num with
// the lanes' dot-product rounding, the corner quotients of t widened 6u -- v_rcp_f32 --, the plane points P =
// S + D T widened by e = 8u (|S| + |P|)), then the gate's own tests over the intervals: t > max(0, -hin,
// hout) for some ray, and each barycentric row b_k = M_k P (M_k . [Pl, Ph]) within [0, 1] widened by
// |M_k|_1 (e + 8u |P|) (the lanes' fl(M p) rounding is <= 3u |M_k|_1 |p|, the interval sums' own <= 3u).
// Host mirror: bvh.cpp bundle_gate_keep_h (tests/test_culling_conservative.py).
__device__ __forceinline__ bool bundle_gate_keep(const float *B, float4 q0, float4 q1, float4 q2, float4 q3) {
  if (!(B[12] > 0.0f)) return true;
  constexpr float u = 0x1p-24f;
  const f3 n = mk(q0.x, q0.y, q0.z);
  float csl, csh, nsl, nsh;
  ivdot(n, mk(B[6], B[7], B[8]), mk(B[9], B[10], B[11]), csl, csh);
  ivdot(n, mk(B[0], B[1], B[2]), mk(B[3], B[4], B[5]), nsl, nsh);
  const float mc = 8.0f * u * (fabsf(n.x) * absmax(B[6], B[9]) + fabsf(n.y) * absmax(B[7], B[10]) + fabsf(n.z) * absmax(B[8], B[11]));
  const float ms = 8.0f * u * (fabsf(n.x) * absmax(B[0], B[3]) + fabsf(n.y) * absmax(B[1], B[4]) + fabsf(n.z) * absmax(B[2], B[5]) + fabsf(q0.w));
  csl -= mc;
  csh += mc;
  const float numl = (q0.w - nsh) - ms, numh = (q0.w - nsl) + ms;
  if (csl > -0.00001f && csh < 0.00001f) return false;  // |cs| < 1e-5 for every ray
  if (!(csl > 0.0f || csh < 0.0f)) return true;          // cs of either sign: t unbounded
  const float r1 = __builtin_amdgcn_rcpf(csl), r2 = __builtin_amdgcn_rcpf(csh);
  const float a1 = numl * r1, a2 = numl * r2, a3 = numh * r1, a4 = numh * r2;
  float tlo = fminf(fminf(a1, a2), fminf(a3, a4)), thi = fmaxf(fmaxf(a1, a2), fmaxf(a3, a4));
  tlo -= 6.0f * u * fabsf(tlo);
  thi += 6.0f * u * fabsf(thi);
  if (!(thi <= 1e30f)) return true;                                   // huge or NaN: no bound
  if (thi <= fmaxf(fmaxf(-q1.x, q1.y), 0.0f)) return false;          // t > max(0, -hin, hout) for no ray
  tlo = fmaxf(tlo, 0.0f);
  float pl[3], ph[3], pm0 = 0.0f, smax = 0.0f;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const float dl = B[6 + a], dh = B[9 + a], sl = B[a], sh = B[3 + a];
    const float x1 = dl * tlo, x2 = dl * thi, x3 = dh * tlo, x4 = dh * thi;
    pl[a] = sl + fminf(fminf(x1, x2), fminf(x3, x4));
    ph[a] = sh + fmaxf(fmaxf(x1, x2), fmaxf(x3, x4));
    pm0 = fmaxf(pm0, absmax(pl[a], ph[a]));
    smax = fmaxf(smax, absmax(sl, sh));
  }
  const float e = 8.0f * u * (smax + pm0), ep = e + 8.0f * u * pm0;
  const f3 P0 = mk(pl[0], pl[1], pl[2]), P1 = mk(ph[0], ph[1], ph[2]);
  const f3 row[3] = {mk(q1.z, q1.w, q2.x), mk(q2.y, q2.z, q2.w), mk(q3.x, q3.y, q3.z)};
  bool keep = true;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    float lo, hi;
    ivdot(row[k], P0, P1, lo, hi);
    const float eb = (fabsf(row[k].x) + fabsf(row[k].y) + fabsf(row[k].z)) * ep + 1e-30f;
    keep &= !(hi + eb < 0.0f) & !(lo - eb > 1.0f);
  }
  return keep;
}

// BZR_TRAV_PHASES (diagnostic build, default 0): k_traverse stamps s_memtime at its phase boundaries and, with
// device counters on, adds each wave's cycles per phase to counter slots (their own counts are small beside
// them): node_visits <- setup (ray loads, bundle reductions), leaf_fetches <- the queued leaves' per-lane
// gates, gate_tests <- the walk's batches and leaf pre-tests, overflow_rays <- the per-lane walk, follows <-
// the always list, segments <- the ranking (variant travph: scripts/ab.py prints them as its counters; the
// stamps cost ~4 %).
#ifndef BZR_TRAV_PHASES
#define BZR_TRAV_PHASES 0
#endif
#if BZR_TRAV_PHASES
#define BZR_PHASE(k)                                          \
  {                                                           \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    ph_acc[ph_cur] += now_ - ph_t;                            \
    ph_t = now_;                                              \
    ph_cur = (k);                                             \
  }
#else
#define BZR_PHASE(k)
#endif
// The lanes whose gate of patch b passed list it as their next candidate (while the list has room; a lane
// past kMaxCand overflows to the full scan).  (Counting the listing lanes into b's histogram word right here --
// b is wave-uniform, so one atomic without return per wave -- and ranking the pairs in k_place instead of
// after the walk: k_traverse -1.6 % on cfg5 and -9 % on cfg3, but k_place's grouped ranking atomics cost more
// than that, cfg3 frames +7.6 %; profiles/r04_ab_rank_late.jsonl.)
// BZR_RANK_EARLY (A/B knob, default 0): each listed group (the lanes whose gate of the wave-uniform patch b
// passed) takes its ranks in b's bucket right away -- one returning atomic by its first lane -- instead of the
// ranking pass after the walk (the candidates' reload, a ballot loop per list slot grouping the lanes by patch,
// the atomics' round trip at the end of the wave: 13 % of a cfg5 wave, 22 % of a cfg3 one).  1: the ranks are
// stored at the next listing (one group pending, its base in a VGPR across the walk); 2: stored at once (the
// wave waits for each atomic).  A ray that later overflows its list keeps its ranked places; k_place fills them
// with idle (kNoPair) records.  Both lose: cfg5 k_traverse 3.88 -> 4.45 (1) / 4.20 (2) ms per frame, cfg3 0.173
// -> 0.201 / 0.187 (profiles/r05_ab_rank_early.jsonl): one atomic round trip per listing instead of one per four
// list slots, and with 1 the pending base spills VGPRs at the 8-wave budget.
#ifndef BZR_RANK_EARLY
#define BZR_RANK_EARLY 0
#endif
constexpr uint32_t kRankEntries = 64;  // BZR_RANK_EARLY 3: listings recorded per wave
struct RankPend {  // the last listed group of the wave (BZR_RANK_EARLY 1); the wave's listings (3)
  uint32_t base = 0u;           // its first place in the bucket (valid in its first lane)
  unsigned long long g = 0ull;  // its lanes
  uint32_t *ent = nullptr;      // 3: LDS [kRankEntries] patch, then [kRankEntries] lane masks (two words each)
  uint32_t ne = 0u;             // 3: listings so far (uniform; past kRankEntries the wave ranks the old way)
};
// Store the pending group's ranks: a lane's slot is its list count - 1 (its count changes only at a listing,
// after this; the overflow flag keeps the low bits).
__device__ __forceinline__ void rank_flush(RankPend &pr, const Work &w, uint32_t n, uint32_t i, uint32_t cnt) {
  if (pr.g) {
    const uint32_t bs = __builtin_amdgcn_readlane(pr.base, (uint32_t)__builtin_ctzll(pr.g));
    if (lane_bit64(pr.g, threadIdx.x & 63u))
      w.rank[(size_t)((cnt & (kOverflow - 1u)) - 1u) * n + i] = bs + lanes_below(pr.g);
    pr.g = 0ull;
  }
}
// BZR_TRAV_HYBRID (A/B knob, default 0 = round 5's k_traverse): in-wave Newton passes for dense leaves (VERDICT r05
// item 1).  A leaf whose exact planar gate passes for at least Work::hyb_t of the wave's lanes (runtime threshold,
// BZR_HYBRID_T; 0 = never) is not listed: its patch and lane mask go to the wave's LDS entries (up to kHybEntries;
// more are listed as before), and once the walk and the always list are done the wave runs one patch-uniform pass
// per entry with the record in SGPRs (k_trace's site, k_newton's arithmetic: kGated, the lanes passed this gate).
// A lane keeps its best in-wave (t order, patch) key; it becomes the ray's initial key, with list slot kHybSlot
// holding its record, so the staged pairs' atomicMin and k_finish treat it like any listed pair's hit.  A follow-side
// result becomes a follow request for k_resolve on a list slot of its own (cand word kCandFollow: no pair for the
// ranking or k_place; its pair record at hbase + j n + ray), or, when the list is full, is retried in the wave.
// Sparse leaves go to the buckets as before.  Same candidates, same keys: the schedule never changes a bit.
// Measured (cfg5 8192^2 staged, lone frames, scripts/ab.py; profiles/r06_ab_hybrid.jsonl): the in-wave passes
// cost what the same pairs cost in k_newton (T = 48 with the walk at priority 3: k_traverse +2.02 ms, k_newton
// -2.0 ms per frame) -- they do not hide behind the walk, which is issue-bound, not latency-bound -- and the
// compiled-in code alone costs the walk 7.6 % (3.90 -> 4.19 ms at T = 0: 90 SGPR spills, 3 VGPRs to scratch at the
// 8-wave budget); T = 32 / 16: 13.5 / 17.1 ms per frame against 11.2.  Not kept; same bits in every variant.
#ifndef BZR_TRAV_HYBRID
#define BZR_TRAV_HYBRID 0
#endif
// BZR_TRAV_PRIO (A/B knob, default 0): the walk at s_setprio(N) -- with BZR_TRAV_HYBRID the in-wave passes back at 0
// (as k_trace's BZR_TRACE_PRIO); without it the whole k_traverse wave, ahead of the other frame's k_newton waves
// that share its CUs when frames are in flight.
#ifndef BZR_TRAV_PRIO
#define BZR_TRAV_PRIO 0
#endif
#ifndef BZR_HYBRID_T_DEFAULT
#define BZR_HYBRID_T_DEFAULT 32
#endif
static_assert(!BZR_TRAV_HYBRID || BZR_RANK_EARLY == 0, "BZR_TRAV_HYBRID ranks after the walk");
constexpr uint32_t kHybEntries = 16;
constexpr uint32_t kListCap = BZR_TRAV_HYBRID ? kMaxCand - 1u : kMaxCand;  // listed slots per ray
constexpr uint32_t kHybSlot = kMaxCand - 1u;                               // the in-wave winner's list slot
constexpr uint32_t kCandFollow = 0x80000000u;                             // cand word of an in-wave follow request
struct HybEntries {  // the wave's dense leaves (LDS)
  uint32_t *b = nullptr;             // [kHybEntries] patch
  unsigned long long *g = nullptr;   // [kHybEntries] lanes whose gate passed
  uint32_t ne = 0u;                  // entries so far (uniform)
  uint32_t t = 0u;                   // the threshold (Work::hyb_t)
};

__device__ __forceinline__ void list_candidate(bool pass, uint32_t b, const Work &w, uint32_t n, uint32_t i,
                                               uint32_t &cnt, RankPend &pr) {
  const bool lst = pass && cnt < kListCap;
#if BZR_RANK_EARLY == 1
  rank_flush(pr, w, n, i, cnt);
#endif
#if BZR_RANK_EARLY == 3
  const unsigned long long g = __ballot(lst);
  if (g) {  // record the listing (patch, lanes) in the wave's LDS; ranked after the walk
    if (pr.ne < kRankEntries && (threadIdx.x & 63u) == 0u) {
      pr.ent[pr.ne] = b;
      reinterpret_cast<unsigned long long *>(pr.ent + kRankEntries)[pr.ne] = g;
    }
    ++pr.ne;
  }
#elif BZR_RANK_EARLY
  const unsigned long long g = __ballot(lst);
  if (g) {
    const uint32_t leader = (uint32_t)__builtin_ctzll(g);
    uint32_t base = 0u;
    if ((threadIdx.x & 63u) == leader) base = atomicAdd(&w.hist[b], (uint32_t)__popcll(g));
#if BZR_RANK_EARLY == 1
    pr.base = base;
    pr.g = g;
#elif BZR_RANK_EARLY == 3
    (void)base;
#else  // 2: wait for the atomic right here (no state across the walk)
    const uint32_t bs = __builtin_amdgcn_readlane(base, leader);
    if (lst) w.rank[(size_t)cnt * n + i] = bs + lanes_below(g);
#endif
  }
#endif
  if (lst) w.cand[(size_t)cnt * n + i] = b;
  if (pass) cnt = cnt < kListCap ? cnt + 1 : (cnt | kOverflow);
}
// A leaf's gate result: a dense leaf (BZR_TRAV_HYBRID) becomes one of the wave's entries, any other is listed.
__device__ __forceinline__ void take_leaf(bool pass, uint32_t b, const Work &w, uint32_t n, uint32_t i, uint32_t &cnt,
                                          RankPend &pr, HybEntries &hy) {
#if BZR_TRAV_HYBRID
  const unsigned long long g = __ballot(pass);
  if (g == 0ull) return;
  if (hy.ne < kHybEntries && (uint32_t)__popcll(g) >= hy.t && hy.t != 0u) {
    if ((threadIdx.x & 63u) == 0u) {
      hy.b[hy.ne] = b;
      hy.g[hy.ne] = g;
    }
    ++hy.ne;
    return;
  }
#else
  (void)hy;
#endif
  list_candidate(pass, b, w, n, i, cnt, pr);
}
// Candidate search.  `alive` (optional): a ray is traced iff alive[off + i] != BZR_RR_NONE.
// One wave's 64 rays i (lane l of the wave holds ray i); `stk` is the wave's LDS stack.
template <int kBlk, int kAblock, bool kFast>
__device__ __forceinline__ void traverse_rays(const MeshView &m, const float *__restrict__ rays, uint32_t ld,
                                              uint32_t off, const uint32_t *__restrict__ alive, uint32_t n,
                                              const Work &w, unsigned long long *counters, uint32_t i, uint32_t *stk,
                                              float *bl, uint32_t *pend, uint32_t *raw, HybEntries hy,
                                              float *ubl = nullptr, unsigned long long *akeep = nullptr,
                                              uint32_t *rk = nullptr, float4 *arec = nullptr) {
#if BZR_TRAV_PHASES
  unsigned long long ph_acc[6] = {0ull, 0ull, 0ull, 0ull, 0ull, 0ull}, ph_t = __builtin_amdgcn_s_memtime();
  uint32_t ph_cur = 0;
#endif
  uint32_t c_nodes = 0, c_leaves = 0, c_gates = 0;  // work counters (with counters on; wave-uniform)
#if BZR_TRAV_PRIO
  __builtin_amdgcn_s_setprio(BZR_TRAV_PRIO);  // the walk's chain of loads ahead of other waves' Newton passes
#endif
  bool active = i < n && (alive == nullptr || alive[off + i] != BZR_RR_NONE);
  f3 s = mk(0.0f, 0.0f, 0.0f), d = s;
  if (i < n) load_ray(rays, ld, off + i, s, d);
#if BZR_STAGED_AOS
  if (i < n) {
    w.aos[2u * i] = make_float4(s.x, s.y, s.z, d.x);
    w.aos[2u * i + 1u] = make_float4(d.y, d.z, 0.0f, 0.0f);
  }
#endif
  uint32_t cnt = 0;
  RankPend rpend;  // BZR_RANK_EARLY: the last listed group's ranks, stored at the next listing (1); listings (3)
  rpend.ent = rk;
  // gate-region boxes hold for ray origins within s_max (bvh.cpp); farther rays take the full scan
  if (active && !(fmaxf(fmaxf(fabsf(s.x), fabsf(s.y)), fabsf(s.z)) <= m.s_max)) {
    cnt |= kOverflow;
    active = false;
  }
  // tree tier, wave-uniform: the near tree's tighter boxes hold when every active ray starts within s_near
  const bool far_ray = active && !(fmaxf(fmaxf(fabsf(s.x), fabsf(s.y)), fabsf(s.z)) <= m.s_near);
  const bool near_tier = !__any(far_ray);
  const bzr_host::Bvh4Node *nodes = near_tier ? m.nodes_near : m.nodes;
  const bzr_host::Bvh4ObbNode *obb = near_tier ? m.obb_near : m.obb;
  const float4 *leaf = near_tier ? m.leaf_near : m.leaf;
  // (the per-lane walk's reciprocals: that walk never runs after the bundle walk, which ends with an empty
  // stack, but dropping them here put k_traverse<256, 1> at 3 VGPR spills (scratch) instead of 0 -- the
  // register allocator is sensitive to it; kept)
  const f3 inv = mk(safe_inv(d.x), safe_inv(d.y), safe_inv(d.z));
  const f3 sinv = mk(s.x * inv.x, s.y * inv.y, s.z * inv.z);
  int sp = 0;  // the node to visit next stays in a scalar register; the other hit children go to stk
  uint32_t next = (m.n > 0 && __any(active)) ? 0u : 0xFFFFFFFFu;
  unsigned long long next_hm = 0ull;
#if BZR_TRAV_BUNDLE
  // the bundle walk (trace_segment's): batches of up to 16 nodes against the wave's ray bundle, hit leaves
  // queued in pend and gate-tested by every active lane
  const bool walk = next != 0xFFFFFFFFu;  // (the bundle words are then in bl, for the always list too)
  bool bwalk = false;                    // the walk choice (trace_segment's)
  bool narrow = false;                   // else every node is tested per lane (as oriented-box nodes are)
  if (walk) {
    narrow = bundle_setup_dpp(active, s, d, bl, threadIdx.x & 63u) <= BZR_BUNDLE_SPREAD;
    if ((threadIdx.x & 63u) == 0u) stk[0] = 0u;
    sp = 1;
    next = 0xFFFFFFFFu;
    bwalk = true;
  }
  const float4 *kids = near_tier ? m.kids_near : m.kids;
#if BZR_TRAV_WIDE
  const float4 *wide = near_tier ? m.wide_near : m.wide;
  (void)kids;
#endif
  uint32_t npend = 0, pi = 0;  // leaves queued in pend, next to gate-test (uniform)
#if BZR_TRAV_PRETEST
  uint32_t nraw = 0;  // leaves queued in raw, not yet pre-tested
#endif
  // the always list's block pre-test (every thread of the block gets here: no early exit above); with
  // BZR_TRAV_ABLOCK 3 k_always_mask did it and akeep points at this ray block's mask
  if constexpr (kAblock == 1 || kAblock == 2) {
    if (!walk) bundle_setup_dpp(active, s, d, bl, threadIdx.x & 63u);  // (an empty wave's bundle is the identity)
    __syncthreads();
    if (threadIdx.x < 13u) {  // the union over the block's waves with rays (bl - wave * kBundleWords: wave 0's)
      const float *b0 = bl - (threadIdx.x >> 6) * kBundleWords;
      const uint32_t k = threadIdx.x;
      float v = k < 12u ? ((k % 6u) < 3u ? __builtin_inff() : -__builtin_inff()) : 1.0f;
      bool any = false;
      for (uint32_t q = 0; q < (uint32_t)kBlk / 64u; ++q) {
        const float *bq = b0 + q * kBundleWords;
        if (!(bq[0] <= bq[3])) continue;  // no active ray in wave q
        any = true;
        const float x = bq[k];
        v = k == 12u ? fminf(v, x) : ((k % 6u) < 3u ? fminf(v, x) : fmaxf(v, x));
      }
      ubl[k] = (k == 12u && !any) ? 0.0f : v;
    }
    __syncthreads();
    for (uint32_t base = 0; base < m.n_always; base += kBlk) {
      const unsigned long long km = __ballot(always_bundle_keep(m.always, base + threadIdx.x, m.n_always, ubl));
      if ((threadIdx.x & 63u) == 0u) akeep[(base + threadIdx.x) >> 6] = km;
    }
    __syncthreads();
#if BZR_TRAV_ALDS
    if constexpr (kAblock == 1) {  // the kept records into LDS, in list order (word, then bit)
      const uint32_t words = (m.n_always + 63u) / 64u;
      uint32_t total = 0;
      for (uint32_t q = 0; q < words; ++q) total += (uint32_t)__popcll(akeep[q]);
      if (total <= kAldsMax) {
        for (uint32_t e = threadIdx.x; e < total * kAldsQuads; e += kBlk) {
          const uint32_t j = e / kAldsQuads, qd = e - j * kAldsQuads;
          uint32_t q = 0, before = 0;
          while (before + (uint32_t)__popcll(akeep[q]) <= j) before += (uint32_t)__popcll(akeep[q++]);
          unsigned long long bits = akeep[q];
          for (uint32_t k = before; k < j; ++k) bits &= bits - 1ull;  // drop the kept patches before j
          arec[e] = m.always[(size_t)kAlwaysQuads * (q * 64u + (uint32_t)__builtin_ctzll(bits)) + qd];
        }
      }
      __syncthreads();
    }
#endif
  }
  while (bwalk) {
    if (pi < npend) {
      BZR_PHASE(1)
#if BZR_TRAV_LEAF_PAIRS
      // two queued leaves per step: both 64-byte records in flight together (one wait for two round trips)
      const bool two = pi + 1u < npend;
      const uint32_t slot0 = __builtin_amdgcn_readfirstlane(pend[pi]);
      const uint32_t slot1 = __builtin_amdgcn_readfirstlane(pend[two ? pi + 1u : pi]);
      pi += two ? 2u : 1u;
      u32x16 r0, r1;
      asm volatile("s_load_dwordx16 %0, %2, 0x0\n\ts_load_dwordx16 %1, %3, 0x0\n\ts_waitcnt lgkmcnt(0)"
                   : "=&s"(r0), "=&s"(r1)
                   : "s"(leaf + 4u * slot0), "s"(leaf + 4u * slot1));
      if (counters) {
        c_leaves += two ? 2u : 1u;
        c_gates += (two ? 2u : 1u) * (uint32_t)__popcll(__ballot(active));
      }
      take_leaf(active & planar_gate(leaf_q(r0, 0), leaf_q(r0, 1), leaf_q(r0, 2), leaf_q(r0, 3), s, d), r0[15], w,
                     n, i, cnt, rpend, hy);
      if (two)
        take_leaf(active & planar_gate(leaf_q(r1, 0), leaf_q(r1, 1), leaf_q(r1, 2), leaf_q(r1, 3), s, d), r1[15],
                       w, n, i, cnt, rpend, hy);
#else
      const uint32_t slot = __builtin_amdgcn_readfirstlane(pend[pi]);
      ++pi;
      const u32x16 r = *((const cu32x16 *)(uintptr_t)leaf + slot);
      if (counters) {
        ++c_leaves;
        c_gates += (uint32_t)__popcll(__ballot(active));
      }
      take_leaf(active & planar_gate(leaf_q(r, 0), leaf_q(r, 1), leaf_q(r, 2), leaf_q(r, 3), s, d), r[15], w, n,
                     i, cnt, rpend, hy);
#endif
      continue;
    }
    BZR_PHASE(2)
#if BZR_TRAV_PRETEST
    if (sp == 0 || nraw > 64u) {  // the queued leaves' wave-level gate pre-test: the survivors go to pend
      if (nraw == 0u) break;
      pi = npend = 0;
      for (uint32_t j0 = 0; j0 < nraw; j0 += 64u) {
        const uint32_t j = j0 + (threadIdx.x & 63u);
        uint32_t slot = 0u;
        bool keep = false;
        if (j < nraw) {
          slot = raw[j];
          const float4 *lq = leaf + 4u * slot;
          keep = bundle_gate_keep(bl, lq[0], lq[1], lq[2], lq[3]);
        }
        const unsigned long long km = __ballot(keep);
        if (keep) pend[npend + lanes_below(km)] = slot;
        npend += (uint32_t)__popcll(km);
      }
      nraw = 0u;
      continue;
    }
    uint32_t *qbuf = raw;  // where this step queues its leaves
    uint32_t &qn = nraw;
#else
    if (sp == 0) break;
    pi = npend = 0;
    uint32_t *qbuf = pend;
    uint32_t &qn = npend;
#endif
    const uint32_t top = __builtin_amdgcn_readfirstlane(stk[sp - 1]);
    if (!narrow || (top & bzr_host::kObbFlag)) {  // one node, its children tested by each lane's own ray
      --sp;
      if (counters) ++c_nodes;
      bool hit[4];
      uint32_t ch[4];
      // (the reciprocals computed here, not kept from the segment's start: wide waves are rare, and 6
        // registers live across the Newton passes would cost occupancy)
        const f3 linv = mk(safe_inv(d.x), safe_inv(d.y), safe_inv(d.z));
        node_children(nodes, obb, top, active, s, d, mk(s.x * linv.x, s.y * linv.y, s.z * linv.z), linv, hit, ch);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const unsigned long long hm = __ballot(hit[c]);
        if (hm == 0ull) continue;
        if (ch[c] & bzr_host::kLeafFlag) {
          if ((threadIdx.x & 63u) == 0u) qbuf[qn] = ch[c] & ~bzr_host::kLeafFlag;
          ++qn;
        } else if (sp < kTravStack) {
          if ((threadIdx.x & 63u) == 0u) stk[sp] = ch[c];
          ++sp;
        } else if ((hm >> (threadIdx.x & 63u)) & 1ull) {
          cnt |= kOverflow;  // stack exhausted: full scan
        }
      }
      continue;
    }
    bool full;
    uint32_t k;
#if BZR_TRAV_WIDE
    qn += bundle_batch<kTravStack, kWideSlots>(wide, stk, sp, qbuf, bl, threadIdx.x & 63u, full, k, qn);
#else
    qn += bundle_batch<kTravStack>(kids, stk, sp, qbuf, bl, threadIdx.x & 63u, full, k, qn);
#endif
    if (full && active) cnt |= kOverflow;  // stack exhausted: every active lane takes the full scan
    if (counters) c_nodes += k;
  }
#endif
  BZR_PHASE(3)
  while (next != 0xFFFFFFFFu || sp > 0) {  // the per-lane walk
    const uint32_t node = next != 0xFFFFFFFFu ? next : __builtin_amdgcn_readfirstlane(stk[--sp]);
    next = 0xFFFFFFFFu;
    if (counters) ++c_nodes;
    bool hit[4];
    uint32_t ch[4];
    node_children(nodes, obb, node, active, s, d, sinv, inv, hit, ch);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const unsigned long long hm = __ballot(hit[c]);
      if (hm == 0ull) continue;
      if (ch[c] & bzr_host::kLeafFlag) {
        const u32x16 r = *((const cu32x16 *)(uintptr_t)leaf + (ch[c] & ~bzr_host::kLeafFlag));
        const float4 q0 = make_float4(__uint_as_float(r[0]), __uint_as_float(r[1]), __uint_as_float(r[2]), __uint_as_float(r[3]));
        const float4 q1 = make_float4(__uint_as_float(r[4]), __uint_as_float(r[5]), __uint_as_float(r[6]), __uint_as_float(r[7]));
        const float4 q2 = make_float4(__uint_as_float(r[8]), __uint_as_float(r[9]), __uint_as_float(r[10]), __uint_as_float(r[11]));
        const float4 q3 = make_float4(__uint_as_float(r[12]), __uint_as_float(r[13]), __uint_as_float(r[14]), 0.0f);
        if (counters) {
          ++c_leaves;
          c_gates += (uint32_t)__popcll(hm);
        }
        take_leaf(hit[c] & planar_gate(q0, q1, q2, q3, s, d), r[15], w, n, i, cnt, rpend, hy);
      } else {
        if (next != 0xFFFFFFFFu) {
          if (sp < kTravStack) stk[sp++] = next;
          else if ((next_hm >> (threadIdx.x & 63u)) & 1ull) cnt |= kOverflow;  // stack exhausted: full scan
        }
        next = ch[c];
        next_hm = hm;
      }
    }
  }
  // the always list (patches without a proven gate region, bvh.cpp): gate-tested for every active ray
  BZR_PHASE(4)
  if (m.n_always && __any(active)) {
#if BZR_TRAV_BUNDLE
    if (!walk)  // (the bundle walk built it already)
#endif
      bundle_to_lds(active, s, d, bl, threadIdx.x & 63u);
    if constexpr (kAblock != 0) {
      const uint32_t lane = threadIdx.x & 63u, words = (m.n_always + 63u) / 64u;
      if constexpr (kAblock == 2) {
      // the block-kept patches compacted into the wave's (now idle) pend buffer, re-tested with its own bundle
      uint32_t total = 0;
      for (uint32_t q = 0; q < words; ++q) {
        const unsigned long long kq = akeep[q];
        if (lane_bit64(kq, lane)) pend[total + lanes_below(kq)] = q * 64u + lane;
        total += (uint32_t)__popcll(kq);
      }
      __builtin_amdgcn_wave_barrier();
      for (uint32_t r0 = 0; r0 < total; r0 += 64u) {
        const uint32_t k = r0 + lane;
        const uint32_t id = k < total ? pend[k] : 0u;
        unsigned long long am = __ballot(k < total && always_bundle_keep(m.always, id, m.n_always, bl));
        for (; am; am &= am - 1ull) {
          uint32_t b;
          if (counters) {
            ++c_leaves;
            c_gates += (uint32_t)__popcll(__ballot(active));
          }
          const uint32_t patch = __builtin_amdgcn_readfirstlane(pend[r0 + __builtin_ctzll(am)]);
          const bool pass = always_gate(m.always, patch, active, s, d, b);
          take_leaf(pass, b, w, n, i, cnt, rpend, hy);
        }
      }
      } else {
#if BZR_TRAV_ALDS
      uint32_t total = 0;
      for (uint32_t q = 0; q < words; ++q) total += (uint32_t)__popcll(akeep[q]);
      if (total <= kAldsMax) {
        for (uint32_t j = 0; j < total; ++j) {
          uint32_t b;
          if (counters) {
            ++c_leaves;
            c_gates += (uint32_t)__popcll(__ballot(active));
          }
          const bool pass = always_gate_lds(arec + (size_t)kAldsQuads * j, active, s, d, b);
          take_leaf(pass, b, w, n, i, cnt, rpend, hy);
        }
      } else
#endif
      for (uint32_t q = 0; q < words; ++q) {
        for (unsigned long long am = akeep[q]; am; am &= am - 1ull) {
          uint32_t b;
          if (counters) {
            ++c_leaves;
            c_gates += (uint32_t)__popcll(__ballot(active));
          }
          const bool pass = always_gate(m.always, q * 64u + __builtin_ctzll(am), active, s, d, b);
          take_leaf(pass, b, w, n, i, cnt, rpend, hy);
        }
      }
      }
    } else
    for (uint32_t ab = 0; ab * 64u < m.n_always; ++ab) {
      unsigned long long am = __ballot(always_bundle_keep(m.always, ab * 64u + (threadIdx.x & 63u), m.n_always, bl));
      for (; am; am &= am - 1ull) {
        uint32_t b;
        if (counters) {
          ++c_leaves;
          c_gates += (uint32_t)__popcll(__ballot(active));
        }
        const bool pass = always_gate(m.always, ab * 64u + __builtin_ctzll(am), active, s, d, b);
        take_leaf(pass, b, w, n, i, cnt, rpend, hy);
      }
    }

  }
  // BZR_TRAV_HYBRID: the wave's dense leaves, one patch-uniform Newton pass each (k_trace's site).  A lane's best
  // (t order, patch) key becomes the ray's initial key (list slot kHybSlot holds its record); a follow-side result
  // becomes a follow request on a list slot of its own, or is retried here when the list is full.
  unsigned long long hbest = ~0ull;
  uint32_t h_pairs = 0u, h_rounds = 0u;  // work counters (uniform)
#if BZR_TRAV_HYBRID
  if (hy.ne) {
    BZR_PHASE(3)
#if BZR_TRAV_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t e = 0; e < hy.ne; ++e) {
      const uint32_t b = __builtin_amdgcn_readfirstlane(hy.b[e]);
      const unsigned long long g0 = hy.g[e];
      const unsigned long long g = ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(g0 >> 32)) << 32) |
                                   (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)g0);
      const bool run = lane_bit64(g, lane) && !(cnt & kOverflow);  // (an overflowed lane takes the full scan)
      if (counters) {
        h_pairs += (uint32_t)__popcll(__ballot(run));
        ++h_rounds;
      }
      const auto pa = uniform_patch(m.full, b);
      uint32_t what = kNone;
      if (run) {
        const Hit h = patch_intersect<BZR_NEWTON_GATED != 0, kFast>(pa, s, d, false);
        what = h.what;
        if (h.what == kIntersect && h.t < FLT_MAX) {
          const unsigned long long k = ((unsigned long long)t_order(h.t) << 32) | (b << 6) | kHybSlot;
          if (k < hbest) {
            hbest = k;
            write_slot(w.slot, n, i, kHybSlot, h, b);
          }
        }
      }
      const bool fol = run && what <= kFollow2;
      if (!__any(fol)) continue;
      const bool room = fol && cnt < kListCap;
      const unsigned long long rm = __ballot(room);
      if (rm) {  // follow requests for k_resolve: pair record (ray | j << 26, b | side << 30) at hbase + j n + ray
        uint32_t base = 0u;
        if (lane == 0u) base = atomicAdd(&w.ctr[0], (uint32_t)__popcll(rm));
        base = __builtin_amdgcn_readfirstlane(base);
        if (room) {
          const uint32_t p = w.hbase + cnt * n + i;
          w.pairs[p] = make_uint2(i | (cnt << 26), b | (what << 30));
          w.cand[(size_t)cnt * n + i] = kCandFollow;
          w.fol[base + lanes_below(rm)] = p;
          ++cnt;
        }
      }
      for (uint32_t side = 0; side < 3u; ++side) {  // list full: the retry runs here (cNone, ranked at b)
        const bool fl = fol && !room && what == side;
        if (!__any(fl)) continue;
        const uint32_t nb = __float_as_uint(pa.r[rec::kNeigh + side]);
        const auto pn = uniform_patch(m.full, nb);
        if (counters) {
          h_pairs += (uint32_t)__popcll(__ballot(fl));
          ++h_rounds;
        }
        if (fl) {
          const Hit h = patch_intersect<false, kFast>(pn, s, d, true);
          if (h.what == kIntersect && h.t < FLT_MAX) {
            const unsigned long long k = ((unsigned long long)t_order(h.t) << 32) | (b << 6) | kHybSlot;
            if (k < hbest) {
              hbest = k;
              write_slot(w.slot, n, i, kHybSlot, h, nb);
            }
          }
        }
      }
    }
  }
#endif
  if (counters) {  // rays traced (one atomic per wave: on one address, so only with counters on)
    const unsigned long long traced = __ballot(i < n && (alive == nullptr || alive[off + i] != BZR_RR_NONE));
    if ((threadIdx.x & 63u) == 0 && traced) atomicAdd(&w.ctr[2], (uint32_t)__popcll(traced));
    // walk work (bzr_ctx_counters node_visits / leaf_fetches / gate_tests), spread over the replicas
    const uint32_t lane = threadIdx.x & 63u, rep = (i >> 6) % kCounterReplicas;
#if BZR_TRAV_HYBRID  // and the in-wave Newton passes' pairs and passes
    const uint32_t v = lane == 0u ? c_nodes : lane == 1u ? c_leaves : lane == 2u ? c_gates : lane == 3u ? h_pairs : h_rounds;
    const uint32_t which = lane == 0u ? BZR_COUNTER_NODE_VISITS : lane == 1u ? BZR_COUNTER_LEAF_FETCHES
                           : lane == 2u ? BZR_COUNTER_GATE_TESTS : lane == 3u ? BZR_COUNTER_PAIRS : BZR_COUNTER_NEWTON_ROUNDS;
    if (!BZR_TRAV_PHASES && lane < 5u && v) atomicAdd(&counters[(size_t)rep * BZR_COUNTER_COUNT + which], (unsigned long long)v);
#else
    (void)h_pairs;
    (void)h_rounds;
    const uint32_t v = lane == 0u ? c_nodes : (lane == 1u ? c_leaves : c_gates);
    const uint32_t which = lane == 0u ? BZR_COUNTER_NODE_VISITS : (lane == 1u ? BZR_COUNTER_LEAF_FETCHES : BZR_COUNTER_GATE_TESTS);
    if (!BZR_TRAV_PHASES && lane < 3u && v) atomicAdd(&counters[(size_t)rep * BZR_COUNTER_COUNT + which], (unsigned long long)v);
#endif
  }
#if BZR_RANK_EARLY == 1
  rank_flush(rpend, w, n, i, cnt);
#endif
  if (i >= n) return;
  w.count[i] = cnt;
#if BZR_TRAV_HYBRID
  w.key[i] = cnt > kMaxCand ? ~0ull : hbest;
#else
  (void)hbest;
  w.key[i] = ~0ull;
#endif
  if (cnt > kMaxCand) w.ovf[atomicAdd(&w.ctr[1], 1u)] = i;
#if BZR_RANK_EARLY == 3
  const uint32_t lane = threadIdx.x & 63u;
  BZR_PHASE(5)
  if (rpend.ne <= kRankEntries) {
    // every recorded listing's atomic at once (lane e: listing e, its lanes minus the overflow rays, which rank
    // nothing: the full scan takes them), one wait, then each listing's lanes store base + their rank in it --
    // a lane's j-th listing is its list slot j
    const unsigned long long ovf = __ballot(cnt > kMaxCand);
    const uint32_t ne = rpend.ne;
    const unsigned long long *eg = reinterpret_cast<const unsigned long long *>(rk + kRankEntries);
    uint32_t base = 0u;
    if (lane < ne) {
      const unsigned long long g = eg[lane] & ~ovf;
      if (g) base = atomicAdd(&w.hist[rk[lane]], (uint32_t)__popcll(g));
    }
    uint32_t slot = 0u;
    for (uint32_t e = 0; e < ne; ++e) {
      const unsigned long long g0 = eg[e];
      const unsigned long long g = ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(g0 >> 32)) << 32) |
                                   (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)g0);
      const uint32_t bs = __builtin_amdgcn_readlane(base, e);
      if (lane_bit64(g & ~ovf, lane)) w.rank[(size_t)slot * n + i] = bs + lanes_below(g & ~ovf);
      slot += lane_bit64(g, lane) ? 1u : 0u;
    }
  } else {
#endif
#if !BZR_RANK_EARLY || BZR_RANK_EARLY == 3
  // Rank of each (ray, patch) pair within its patch bucket.  Neighbouring rays mostly share
  // patches: the lanes naming the same patch form a group (found with ballots, no memory traffic),
  // each group's first lane adds the group size -- all groups in one atomic instruction -- and the
  // lanes take their rank from the returned base.
  const uint32_t lane = threadIdx.x & 63u;
  BZR_PHASE(5)
  const uint32_t listed = cnt <= kMaxCand ? cnt : 0u;
  // Four list slots per round: their candidate loads first, then the grouping, then all four rounds'
  // returning atomics in flight together (one wait instead of four: vmcnt retires in issue order).
#ifndef BZR_RANK_BATCH
#define BZR_RANK_BATCH 4
#endif
  constexpr int kRankBatch = BZR_RANK_BATCH;
  for (uint32_t j0 = 0; __any(j0 < listed); j0 += kRankBatch) {
    uint32_t b[kRankBatch], leader[kRankBatch], below[kRankBatch], base[kRankBatch];
#pragma unroll
    for (int k = 0; k < kRankBatch; ++k)
      b[k] = j0 + k < listed ? w.cand[(size_t)(j0 + k) * n + i] : (BZR_TRAV_HYBRID ? kCandFollow : 0u);
#pragma unroll
    for (int k = 0; k < kRankBatch; ++k) {
      // (an in-wave follow request is no pair: BZR_TRAV_HYBRID)
      const bool pend = BZR_TRAV_HYBRID ? !(b[k] & kCandFollow) : j0 + k < listed;
      unsigned long long group = 0ull;
      bool todo = pend;
      for (;;) {
        const unsigned long long mask = __ballot(todo);
        if (mask == 0ull) break;
        const uint32_t b0 = __builtin_amdgcn_readlane(b[k], __builtin_ctzll(mask));
        const bool same = todo && b[k] == b0;
        const unsigned long long g = __ballot(same);
        if (same) {
          group = g;
          todo = false;
        }
      }
      leader[k] = pend ? (uint32_t)__builtin_ctzll(group) : lane;
      below[k] = lanes_below(group);
      base[k] = 0u;
      if (pend && lane == leader[k]) base[k] = atomicAdd(&w.hist[b[k]], (uint32_t)__popcll(group));
    }
#pragma unroll
    for (int k = 0; k < kRankBatch; ++k) {
      const uint32_t bs = __shfl(base[k], (int)leader[k], 64);
      if (BZR_TRAV_HYBRID ? !(b[k] & kCandFollow) : j0 + k < listed) w.rank[(size_t)(j0 + k) * n + i] = bs + below[k];
    }
  }
#else
  const uint32_t lane = threadIdx.x & 63u;
  (void)lane;
#endif
#if BZR_RANK_EARLY == 3
  }
#endif
#if BZR_TRAV_PHASES
  BZR_PHASE(0)
  if (counters && lane < 6u) {
    const uint32_t id[6] = {BZR_COUNTER_NODE_VISITS, BZR_COUNTER_LEAF_FETCHES, BZR_COUNTER_GATE_TESTS,
                            BZR_COUNTER_OVERFLOW_RAYS, BZR_COUNTER_FOLLOWS, BZR_COUNTER_SEGMENTS};
    unsigned long long v = 0ull;
    uint32_t which = 0;
#pragma unroll
    for (uint32_t k = 0; k < 6u; ++k)
      if (lane == k) {
        v = ph_acc[k];
        which = id[k];
      }
    atomicAdd(&counters[(size_t)((i >> 6) % kCounterReplicas) * BZR_COUNTER_COUNT + which], v);
  }
#endif
}

// Candidate search, one 64-ray wave per 64 consecutive rays.
// BZR_TRAV_XCD (A/B knob, deal_blocks policy): 1 = XCD-contiguous ray ranges (round 1), 0 = dispatch
// order, G > 1 = runs of G blocks per XCD.
#ifndef BZR_TRAV_XCD
#define BZR_TRAV_XCD 1
#endif
// BZR_TRAV_WPE (default 8; 0 = the compiler's choice, 7 waves): amdgpu_waves_per_eu lower bound for k_traverse.
// At 8 waves per SIMD it keeps 64 VGPRs (35 SGPRs spill into VGPR lanes, no scratch): its walk waits on memory
// 45 % of its cycles, and the eighth wave hides more of it -- k_traverse -8 % on cfg5 (4.91 -> 4.52 ms per
// frame) and -10 % on cfg3 (0.221 -> 0.200 ms), frames -4.2 / -4.8 %, same bits (two box runs agree;
// profiles/r04_ab_traverse_wpe8.jsonl).
#ifndef BZR_TRAV_WPE
#define BZR_TRAV_WPE 8
#endif
#if BZR_TRAV_WPE
#define BZR_TRAV_ATTR __attribute__((amdgpu_waves_per_eu(BZR_TRAV_WPE)))
#else
#define BZR_TRAV_ATTR
#endif
template <int kBlk, int kAblock, bool kFast>
__global__ __launch_bounds__(kBlk) BZR_TRAV_ATTR void k_traverse(MeshView m, const float *__restrict__ rays, uint32_t ld,
                                                         uint32_t off, const uint32_t *__restrict__ alive, uint32_t n,
                                                         Work w, unsigned long long *counters) {
  __shared__ uint32_t stack[kBlk / 64][kTravStack];
  __shared__ float bundle[kBlk / 64][kBundleWords];  // the wave's ray bundle (bundle walk, always list)
#if BZR_TRAV_BUNDLE
  __shared__ uint32_t pend[kBlk / 64][BZR_TRAV_PRETEST ? 128 : 64];  // the bundle walk's queued leaf slots
  uint32_t *wpend = pend[threadIdx.x >> 6];
#else
  uint32_t *wpend = nullptr;
#endif
#if BZR_TRAV_BUNDLE && BZR_TRAV_PRETEST
  __shared__ uint32_t raw[kBlk / 64][128];  // leaves before the pre-test (up to two batches' worth)
  uint32_t *wraw = raw[threadIdx.x >> 6];
#else
  uint32_t *wraw = nullptr;
#endif
  const uint32_t b = deal_blocks<BZR_TRAV_XCD>(blockIdx.x, gridDim.x);
#if BZR_RANK_EARLY == 3
  __shared__ __attribute__((aligned(8))) uint32_t rk[kBlk / 64][3 * kRankEntries];  // the wave's listings (patch, lane mask)
  uint32_t *wrk = rk[threadIdx.x >> 6];
#else
  uint32_t *wrk = nullptr;
#endif
  HybEntries hy;  // the wave's dense leaves (BZR_TRAV_HYBRID)
#if BZR_TRAV_HYBRID
  __shared__ uint32_t hyb_b[kBlk / 64][kHybEntries];
  __shared__ unsigned long long hyb_g[kBlk / 64][kHybEntries];
  hy.b = hyb_b[threadIdx.x >> 6];
  hy.g = hyb_g[threadIdx.x >> 6];
  hy.t = w.hyb_t;
#endif
  if constexpr (kAblock == 3) {  // the mask of this wave's 256-ray block (k_always_mask)
    traverse_rays<kBlk, 3, kFast>(m, rays, ld, off, alive, n, w, counters, b * kBlk + threadIdx.x, stack[threadIdx.x >> 6],
                                  bundle[threadIdx.x >> 6], wpend, wraw, hy, nullptr,
                                  w.amask + (size_t)((b * kBlk) / kAblockBlock) * kAmaskWords, wrk);
  } else if constexpr (kAblock != 0) {
    static_assert(!kAblock || BZR_TRAV_BUNDLE, "BZR_TRAV_ABLOCK needs the bundle walk");
    __shared__ float ubl[16];                                  // the block's union bundle (words 0..12)
    __shared__ unsigned long long akeep[kAblockMax / 64u];     // block-kept always-listed patches
#if BZR_TRAV_ALDS
    __shared__ float4 arec[kAldsMax * kAldsQuads];             // their records (BZR_TRAV_ALDS)
#else
    float4 *arec = nullptr;
#endif
    traverse_rays<kBlk, kAblock, kFast>(m, rays, ld, off, alive, n, w, counters, b * kBlk + threadIdx.x,
                                        stack[threadIdx.x >> 6], bundle[threadIdx.x >> 6], wpend, wraw, hy, ubl, akeep,
                                        wrk, arec);
  } else {
    traverse_rays<kBlk, 0, kFast>(m, rays, ld, off, alive, n, w, counters, b * kBlk + threadIdx.x, stack[threadIdx.x >> 6],
                                  bundle[threadIdx.x >> 6], wpend, wraw, hy, nullptr, nullptr, wrk);
  }
}


// BZR_TRAV_ABLOCK 3: the always list's block pre-test as a kernel of its own.  Block b (kAblockBlock rays) forms
// its waves' ray bundles (bundle_setup_dpp) and their union, ballots always_bundle_keep for every always-listed
// patch and writes the kept mask to amask[b].  The union is over every ray of the block that is traced (a superset
// of the walk's active rays: rays beyond s_max take the full scan there), so a dropped patch is one no traced ray of
// the block can pass -- the candidates are unchanged.
__global__ __launch_bounds__(kAblockBlock) void k_always_mask(MeshView m, const float *__restrict__ rays, uint32_t ld,
                                                              uint32_t off, const uint32_t *__restrict__ alive, uint32_t n,
                                                              unsigned long long *__restrict__ amask) {
  __shared__ float bundle[kAblockBlock / 64][kBundleWords];
  __shared__ float ubl[16];
  const uint32_t i = blockIdx.x * kAblockBlock + threadIdx.x, lane = threadIdx.x & 63u;
  const bool active = i < n && (alive == nullptr || alive[off + i] != BZR_RR_NONE);
  f3 s = mk(0.0f, 0.0f, 0.0f), d = s;
  if (i < n) load_ray(rays, ld, off + i, s, d);
  bundle_setup_dpp(active, s, d, bundle[threadIdx.x >> 6], lane);
  __syncthreads();
  if (threadIdx.x < 13u) {  // the union over the block's waves with rays (as traverse_rays' block pre-test)
    const uint32_t k = threadIdx.x;
    float v = k < 12u ? ((k % 6u) < 3u ? __builtin_inff() : -__builtin_inff()) : 1.0f;
    bool any = false;
    for (uint32_t q = 0; q < kAblockBlock / 64u; ++q) {
      const float *bq = bundle[q];
      if (!(bq[0] <= bq[3])) continue;  // no traced ray in wave q
      any = true;
      const float x = bq[k];
      v = k == 12u ? fminf(v, x) : ((k % 6u) < 3u ? fminf(v, x) : fmaxf(v, x));
    }
    ubl[k] = (k == 12u && !any) ? 0.0f : v;
  }
  __syncthreads();
  for (uint32_t base = 0; base < m.n_always; base += kAblockBlock) {
    const unsigned long long km = __ballot(always_bundle_keep(m.always, base + threadIdx.x, m.n_always, ubl));
    if (lane == 0u) amask[(size_t)blockIdx.x * kAmaskWords + ((base + threadIdx.x) >> 6)] = km;
  }
}

// A bucket of c pairs in the staged layout (BZR_DENSE_MIN): (dense chunks << 32) | pairs in the sparse region.
struct BucketSplit {
  __host__ __device__ __forceinline__ unsigned long long operator()(uint32_t c) const {
    const uint32_t rem = c & 63u;
    const bool pad = rem >= kDenseMin;
    return ((unsigned long long)((c >> 6) + (pad ? 1u : 0u)) << 32) | (pad ? 0u : rem);
  }
};

// Threads t < nb: bucket t's padded lanes (the last dense chunk's lanes past its pairs) get the kNoPair
// record, its histogram word is cleared for the next segment, and (pair_count: with device counters on) the
// wave adds its buckets' pair counts to ctr[3].  Threads t < n: ray t's listed pairs go to their places -- rank r of bucket b is dense pair
// 64 dense_base(b) + r while r < 64 dense_chunks(b), else sparse pair r - 64 dense_chunks(b) of the bucket.
__global__ __launch_bounds__(kBlock) void k_place(uint32_t n, uint32_t nb, Work w, uint32_t *__restrict__ pair_count) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  uint32_t c = 0;
  if (t < nb) {
    c = w.hist[t];
    if (c) {
      w.hist[t] = 0u;
      if ((c & 63u) >= kDenseMin) {
        const uint32_t p0 = static_cast<uint32_t>(w.offs[t] >> 32) * 64u + c, p1 = (p0 + 63u) & ~63u;
        for (uint32_t p = p0; p < p1; ++p) w.pairs[p] = make_uint2(kNoPair, t);
      }
    }
  }
  // the wave's buckets' pairs (bzr_ctx_counters "pairs": the pairs the Newton stage runs): one atomic per
  // bucket wave -- per ray wave, the atomics on one address cost k_place 30 %
  if (pair_count && blockIdx.x * kBlock < nb) {
    uint32_t sum = c;
#pragma unroll
    for (int k = 32; k >= 1; k >>= 1) sum += __shfl_xor(sum, k, 64);
    if ((threadIdx.x & 63u) == 0u && sum) atomicAdd(pair_count, sum);
  }
  if (t >= n) return;
  const uint32_t c0 = w.count[t];
#if BZR_RANK_EARLY == 1 || BZR_RANK_EARLY == 2
  // an overflow ray (the full scan takes it) had its listed pairs ranked in k_traverse: their places get idle
  // kNoPair records (its patch in .y, as the dense chunks' padding), and the pair counter drops them
  const bool idle = c0 > kMaxCand;
  const uint32_t cnt = c0 & (kOverflow - 1u);
  if (idle && cnt && pair_count) atomicSub(pair_count, cnt);
#else
  if (c0 > kMaxCand) return;  // (an overflow ray's list is not ranked: the full scan takes it)
  const bool idle = false;
  const uint32_t cnt = c0;
#endif
  if (cnt == 0) return;
  const unsigned long long tot = w.offs[nb];
  const uint32_t sparse0 = static_cast<uint32_t>(tot >> 32) * 64u;  // the sparse region's first pair
  // four list slots per round: their loads first, then the offsets, then the stores
  for (uint32_t j0 = 0; j0 < cnt; j0 += 4u) {
    uint32_t b[4], r[4];
    unsigned long long o0[4], o1[4];
#pragma unroll
    for (uint32_t k = 0; k < 4u; ++k) {
      const uint32_t j = j0 + k < cnt ? j0 + k : j0;
      b[k] = w.cand[(size_t)j * n + t];
      r[k] = w.rank[(size_t)j * n + t];
    }
#pragma unroll
    for (uint32_t k = 0; k < 4u; ++k) {
      const uint32_t bb = BZR_TRAV_HYBRID ? b[k] & ~kCandFollow : b[k];  // (BZR_TRAV_HYBRID: follow requests place no pair)
      o0[k] = w.offs[bb];
      o1[k] = w.offs[bb + 1u];
    }
#pragma unroll
    for (uint32_t k = 0; k < 4u; ++k) {
      if (j0 + k >= cnt) break;
#if BZR_TRAV_HYBRID
      if (b[k] & kCandFollow) continue;
#endif
      const uint32_t dbase = static_cast<uint32_t>(o0[k] >> 32), dlen = 64u * (static_cast<uint32_t>(o1[k] >> 32) - dbase);
      const uint32_t p = r[k] < dlen ? dbase * 64u + r[k] : sparse0 + static_cast<uint32_t>(o0[k]) + (r[k] - dlen);
      w.pairs[p] = make_uint2(idle ? kNoPair : t | ((j0 + k) << 26), b[k]);
    }
  }
}

constexpr uint32_t kFolBuf = 256;  // per-wave LDS staging of follow requests

// Copies a wave's staged follow requests to the global list (one atomicAdd for all of them).
__device__ __forceinline__ void flush_follow(uint32_t *buf, uint32_t &nf, uint32_t *__restrict__ fol,
                                             uint32_t *__restrict__ nfol, uint32_t lane) {
  uint32_t base = 0;
  if (lane == 0) base = atomicAdd(nfol, nf);
  base = __builtin_amdgcn_readfirstlane(base);
  for (uint32_t k = lane; k < nf; k += 64u) fol[base + k] = buf[k];
  nf = 0;
}

// Persistent waves over the dense chunks: wave g takes chunks g, g + W, ... and fetches the next chunk's
// pair records while it computes the current one.  A dense chunk holds one patch (its lane 0 always a real
// pair), processed with the record in scalar registers, `full` being a __restrict__ constant-address-space
// read; the padded lanes of a bucket's last chunk (kNoPair) idle.
// BZR_NEWTON_WPE (default 8): amdgpu_waves_per_eu lower bound for k_newton.  At 8 waves per SIMD the
// compiler spills ~33 SGPRs to VGPR lanes and keeps 64 VGPRs; measured 2.4 % faster per frame than
// the unconstrained 7 waves (66 VGPRs, 106 SGPRs), same output bits.
#ifndef BZR_NEWTON_WPE
#define BZR_NEWTON_WPE 8
#endif
#define BZR_NEWTON_ATTR __attribute__((amdgpu_waves_per_eu(BZR_NEWTON_WPE)))
// BZR_NEWTON_PREFETCH (A/B knob, default 0): k_newton loads a chunk's rays while the previous chunk computes
// (and the pair records two chunks ahead) instead of at the chunk's start.  61 instead of 54 VGPRs, still 8
// waves: cfg5 k_newton 4.32 -> 4.26 ms per frame, frames within noise; cfg3 frames -3 % (noisy)
// (profiles/r05_ab_newton_prefetch.jsonl): the eight waves per SIMD already hide the gathers.  Not kept.
#ifndef BZR_NEWTON_PREFETCH
#define BZR_NEWTON_PREFETCH 0
#endif
template <bool kFast>
__global__ __launch_bounds__(kBlock) BZR_NEWTON_ATTR void k_newton(const float *__restrict__ full,
                                                   const unsigned long long *__restrict__ total,
                                                   uint2 *__restrict__ pairs, const float *__restrict__ rays,
                                                   uint32_t ld, uint32_t off, uint32_t n, float *__restrict__ slot,
                                                   unsigned long long *__restrict__ key,
                                                   uint32_t *__restrict__ fol, uint32_t *__restrict__ nfol,
                                                   const float4 *__restrict__ aos, RowOut ro) {
  __shared__ uint32_t fbuf[kWaves][kFolBuf];
  const uint32_t wv = threadIdx.x >> 6;
  uint32_t nf = 0;  // staged follow requests of this wave (uniform)
  const uint32_t D = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(*total >> 32));  // dense chunks
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t W = gridDim.x * kWaves;
#if BZR_NEWTON_XCD
  uint32_t q = xcd_contiguous(blockIdx.x, gridDim.x) * kWaves + (threadIdx.x >> 6);
#else
  uint32_t q = blockIdx.x * kWaves + (threadIdx.x >> 6);
#endif
  q = __builtin_amdgcn_readfirstlane(q);
  uint2 pr = make_uint2(kNoPair, 0u);
  if (q < D) pr = pairs[q * 64u + lane];
#if BZR_NEWTON_PREFETCH
  // two-deep pipeline: this chunk's rays were loaded during the previous chunk, the next chunk's pair records
  // two chunks ahead
  f3 ns = mk(0.0f, 0.0f, 0.0f), nd = ns;
  if (q < D && pr.x != kNoPair) load_pair_ray(aos, rays, ld, off, pr.x & kRayMask, ns, nd);
  uint2 pr2 = make_uint2(kNoPair, 0u);
  if (q + W < D) pr2 = pairs[(q + W) * 64u + lane];
#endif
#if BZR_NEWTON_QUEUE && !BZR_NEWTON_PREFETCH
  for (uint32_t qnext = 0; q < D; q = qnext) {
#else
  for (; q < D; q += W) {
#endif
    const uint32_t p = q * 64u + lane;
    const bool todo = pr.x != kNoPair;
    const uint32_t ray = pr.x & kRayMask, j = pr.x >> 26;
    const uint32_t b = __builtin_amdgcn_readfirstlane(pr.y);  // the chunk's patch (lane 0 is a real pair)
#if BZR_NEWTON_PREFETCH
    const f3 s = ns, d = nd;
    const uint32_t qn = q + W;
    pr = pr2;  // the next chunk's pairs (loaded a chunk ago): its rays now, its successor's pairs too
    if (qn < D && pr.x != kNoPair) load_pair_ray(aos, rays, ld, off, pr.x & kRayMask, ns, nd);
    if (qn + W < D) pr2 = pairs[(qn + W) * 64u + lane];
#else
    f3 s = mk(0.0f, 0.0f, 0.0f), d = s;
    if (todo) load_pair_ray(aos, rays, ld, off, ray, s, d);  // pairs of one patch: mostly neighbouring rays
#if BZR_NEWTON_QUEUE
    uint32_t qn = 0;  // the wave's next chunk: the W first chunks went to the waves by id, the rest from the counter
    if (lane == 0u) qn = atomicAdd(nfol + 5, 1u);
    qn = __builtin_amdgcn_readfirstlane(qn) + W;
#else
    const uint32_t qn = q + W;
#endif
    if (qn < D) pr = pairs[qn * 64u + lane];  // prefetch the next chunk's pair records
#endif
#if BZR_NEWTON_QUEUE && !BZR_NEWTON_PREFETCH
    qnext = qn;
#endif
    bool is_fol = false;
    const auto pa = uniform_patch(full, b);
#if BZR_ROWS_DIRECT
    if (ro.rows) {
      Hit h = no_hit();
      // every pair passed this patch's planar gate in k_traverse (same arithmetic, same record values)
      if (todo) h = patch_intersect<BZR_NEWTON_GATED != 0, kFast>(pa, s, d, false);
      row_step(ro, key, todo && h.what == kIntersect, ray, j, b, h, b);
      is_fol = todo && h.what <= kFollow2;
      if (is_fol) reinterpret_cast<uint32_t *>(pairs)[2u * p + 1u] = b | (h.what << 30);  // the side, for k_resolve
    } else
#else
    (void)ro;
#endif
    if (todo) {
      const Hit h = patch_intersect<BZR_NEWTON_GATED != 0, kFast>(pa, s, d, false);
      if (h.what == kIntersect) record(slot, n, ray, j, b, h, b, &key[ray]);
      is_fol = h.what <= kFollow2;
      if (is_fol) reinterpret_cast<uint32_t *>(pairs)[2u * p + 1u] = b | (h.what << 30);  // the side, for k_resolve
    }
    // follow requests: staged in this wave's LDS buffer, published with one atomic per flush
    const unsigned long long fm = __ballot(is_fol);
    if (fm) {
      if (is_fol) fbuf[wv][nf + lanes_below(fm)] = p;
      nf += (uint32_t)__popcll(fm);
      if (nf > kFolBuf - 64u) flush_follow(fbuf[wv], nf, fol, nfol, lane);
    }
  }
  if (nf) flush_follow(fbuf[wv], nf, fol, nfol, lane);
}

// The sparse region (buckets' remainders below BZR_DENSE_MIN pairs): every lane runs its own pair with its
// own patch record, so a chunk of many small buckets costs one pass instead of one per patch.
template <bool kFast>
__global__ __launch_bounds__(kBlock) void k_newton_lane(const float *__restrict__ full,
                                                        const unsigned long long *__restrict__ total,
                                                        uint2 *__restrict__ pairs, const float *__restrict__ rays,
                                                        uint32_t ld, uint32_t off, uint32_t n, float *__restrict__ slot,
                                                        unsigned long long *__restrict__ key,
                                                        uint32_t *__restrict__ fol, uint32_t *__restrict__ nfol,
                                                        const float4 *__restrict__ aos, RowOut ro) {
  const unsigned long long tot = *total;
  const uint32_t base = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(tot >> 32)) * 64u;
  const uint32_t S = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(tot));
  const uint32_t lane = threadIdx.x & 63u;
  for (uint32_t c = blockIdx.x * kWaves + (threadIdx.x >> 6); c * 64u < S; c += gridDim.x * kWaves) {
    const uint32_t p = base + c * 64u + lane;
    bool is_fol = false;
    const uint2 pr = c * 64u + lane < S ? pairs[p] : make_uint2(kNoPair, 0u);
#if BZR_ROWS_DIRECT
    const bool todo = pr.x != kNoPair;
    const uint32_t ray = pr.x & kRayMask, j = pr.x >> 26, b = pr.y;
    Hit h = no_hit();
    if (todo) {
      f3 s, d;
      load_pair_ray(aos, rays, ld, off, ray, s, d);
      const Patch pa = load_patch(full + (size_t)rec::kWords * b);
      h = patch_intersect<BZR_NEWTON_GATED != 0, kFast>(pa, s, d, false);
    }
    if (ro.rows) row_step(ro, key, todo && h.what == kIntersect, ray, j, b, h, b);
    else if (todo && h.what == kIntersect) record(slot, n, ray, j, b, h, b, &key[ray]);
    if (todo) {
      is_fol = h.what <= kFollow2;
      if (is_fol) reinterpret_cast<uint32_t *>(pairs)[2u * p + 1u] = b | (h.what << 30);
    }
#else
    (void)ro;
    if (pr.x != kNoPair) {
      const uint32_t ray = pr.x & kRayMask, j = pr.x >> 26, b = pr.y;
      f3 s, d;
      load_pair_ray(aos, rays, ld, off, ray, s, d);
      const Patch pa = load_patch(full + (size_t)rec::kWords * b);
      const Hit h = patch_intersect<BZR_NEWTON_GATED != 0, kFast>(pa, s, d, false);
      if (h.what == kIntersect) record(slot, n, ray, j, b, h, b, &key[ray]);
      is_fol = h.what <= kFollow2;
      if (is_fol) reinterpret_cast<uint32_t *>(pairs)[2u * p + 1u] = b | (h.what << 30);
    }
#endif
    const unsigned long long fm = __ballot(is_fol);
    if (fm) {
      uint32_t fb = 0;
      if (lane == 0u) fb = atomicAdd(nfol, (uint32_t)__popcll(fm));
      fb = __builtin_amdgcn_readfirstlane(fb);
      if (is_fol) fol[fb + lanes_below(fm)] = p;
    }
  }
}

template <int kMode, bool kFast>
// BZR_FINISH_WPE / BZR_RESOLVE_WPE (A/B knobs, default 0 = the compiler's choice): amdgpu_waves_per_eu lower
// bounds for k_finish (112 VGPRs -- the overflow rays' Newton re-evaluation -- so 4 waves per SIMD) and
// k_resolve (120 VGPRs, 4 waves).  k_finish at 6 or 8 waves (27 / 72 VGPRs spilled) measured no faster -- it
// is HBM-bound at ~6 TB/s either way (profiles/r04_ab_finish_split.jsonl); k_resolve spills 143 / 378.
#ifndef BZR_FINISH_WPE
#define BZR_FINISH_WPE 0
#endif
#ifndef BZR_RESOLVE_WPE
#define BZR_RESOLVE_WPE 0
#endif
#if BZR_FINISH_WPE
#define BZR_FINISH_ATTR __attribute__((amdgpu_waves_per_eu(BZR_FINISH_WPE)))
#else
#define BZR_FINISH_ATTR
#endif
#if BZR_RESOLVE_WPE
#define BZR_RESOLVE_ATTR __attribute__((amdgpu_waves_per_eu(BZR_RESOLVE_WPE)))
#else
#define BZR_RESOLVE_ATTR
#endif
// BZR_FINISH_NORAY (default 1; 0 = the round-4 k_finish): the intersect segments' k_finish reads no ray -- a
// BezierIntersection needs none -- and the overflow rays (whose winner k_finish would evaluate again, with the ray)
// are emitted by k_finish_ovf just before it; 24 B per ray less, one small launch more per chunk.  First measured
// with the count tested before the key was loaded (the key and slot loads then waited on it): cfg5 +0.6 %, cfg3
// -0.6 to -1 % with frames in flight, lone frames slower (profiles/r05_ab_finish_noray.jsonl).  With count and
// key loaded together: lone frames cfg5 -0.5 %, cfg3 -1.2 %; frames in flight cfg5 +-0.3 %, cfg3 +1.9 %
// (profiles/r05_ab_finish_noray_v2.jsonl), same bits; the intersect k_finish drops from 112 to 12 VGPRs (the
// overflow rays' re-evaluation moved out).  Its HBM reads did not move (385.7 MB per 8 M-ray cfg5 chunk either
// way, profiles/r05_cfg5_staged_noray.txt): the compiler had already sunk the old kernel's ray loads into its
// overflow branch (its ISA loads count and key, then the slot).  Kept for the VGPRs and the lone frames.
#ifndef BZR_FINISH_NORAY
#define BZR_FINISH_NORAY 1
#endif
__global__ __launch_bounds__(kBlock) BZR_FINISH_ATTR void k_finish(MeshView m, const float *rays, uint32_t ld, uint32_t off, uint32_t n,
                                                   Work w, Out o) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x < 6) w.ctr[threadIdx.x] = 0u;  // last reader of the counters this segment
  if (i >= n) return;
  const uint32_t gi = off + i;
  if constexpr (kMode == kModeHits && BZR_FINISH_NORAY) {
    // count and key together (testing the count first would make the key and slot loads wait on it)
    const uint32_t c = w.count[i];
    const unsigned long long k = w.key[i];
    if (c > kMaxCand) return;  // an overflow ray or a dirty row (BZR_ROWS_DIRECT): k_finish_ovf emitted it
    if (BZR_ROWS_DIRECT && w.ro.rows) {  // BZR_ROWS_DIRECT: a hit's row is written already; a miss's here
      if (k == ~0ull) store_hit(o.hits, ld, gi, no_hit(), 0xFFFFFFFFu);
      return;
    }
    Hit h = no_hit();
    uint32_t patch = 0xFFFFFFFFu;
    if (k != ~0ull) {
      const size_t sl = (size_t)(static_cast<uint32_t>(k) & 63u) * n + i;
      const float4 *r = reinterpret_cast<const float4 *>(w.slot) + 3 * sl;
      const float4 r0 = r[0], r1 = r[1], r2 = r[2];
      h.t = r0.x;
      h.point = mk(r0.y, r0.z, r0.w);
      h.cs = r1.x;
      h.bary = mk(r1.y, r1.z, r1.w);
      h.normal = mk(r2.x, r2.y, r2.z);
      h.what = kIntersect;
      patch = __float_as_uint(r2.w);
    }
    store_hit(o.hits, ld, gi, h, patch);
    return;
  }
  if (kMode == kModeStage && !o.first && o.status[gi] == BZR_RR_NONE) return;
  // the ray is loaded unconditionally: making the load depend on w.count (an intersect chunk's hits need it
  // only for an overflow ray) serialises the two reads and measured slower (cfg3 k_finish 0.059 -> 0.069 ms,
  // profiles/r04_ab_traverse_wpe8.jsonl, variant "finish")
  f3 s, d;
  load_ray(rays, ld, gi, s, d);
  Hit h = no_hit();
  uint32_t patch = 0xFFFFFFFFu;
  const unsigned long long k = w.key[i];
  if (w.count[i] > kMaxCand) {  // overflow ray: k_resolve left (t order, scanned patch) -- evaluate it again
    // (in a separate launch over the overflow list instead, k_finish would drop from 112 VGPRs to far fewer:
    // measured no faster -- an HBM-bound kernel -- and +30 % on cfg2's short frames; r04_ab_finish_split.jsonl)
    if (k != ~0ull) h = evaluate_patch<kFast>(m, static_cast<uint32_t>(k), s, d, patch);
  } else if (k != ~0ull) {
    const size_t sl = (size_t)(static_cast<uint32_t>(k) & 63u) * n + i;  // the winner's list slot (record())
    const float4 *r = reinterpret_cast<const float4 *>(w.slot) + 3 * sl;  // AoS: 48 bytes per slot
    const float4 r0 = r[0], r1 = r[1], r2 = r[2];
    h.t = r0.x;
    h.point = mk(r0.y, r0.z, r0.w);
    h.cs = r1.x;
    h.bary = mk(r1.y, r1.z, r1.w);
    h.normal = mk(r2.x, r2.y, r2.z);
    h.what = kIntersect;
    patch = __float_as_uint(r2.w);
  }
  emit<kMode>(o, ld, gi, s, d, h, patch);
}

// BZR_FINISH_NORAY: the overflow rays of an intersect segment (the w.ovf list), emitted before k_finish (which
// clears the counters and skips these rays): their winner -- k_resolve's full-scan key -- evaluated again.
template <bool kFast>
__global__ __launch_bounds__(kBlock) void k_finish_ovf(MeshView m, const float *rays, uint32_t ld, uint32_t off, Work w,
                                                       Out o) {
  const uint32_t V = __builtin_amdgcn_readfirstlane(w.ctr[1]);
  for (uint32_t q = blockIdx.x * kBlock + threadIdx.x; q < V; q += gridDim.x * kBlock) {
    const uint32_t i = w.ovf[q], gi = off + i;
    f3 s, d;
    load_ray(rays, ld, gi, s, d);
    Hit h = no_hit();
    uint32_t patch = 0xFFFFFFFFu;
    const unsigned long long k = w.key[i];
    if (k != ~0ull) h = evaluate_patch<kFast>(m, static_cast<uint32_t>(k), s, d, patch);
    store_hit(o.hits, ld, gi, h, patch);
  }
#if BZR_ROWS_DIRECT
  // BZR_ROWS_DIRECT's dirty rows: the final key's pair (candidate b, list slot j) evaluated again -- b with cThis,
  // then its follow side's neighbour with cNone, as k_newton / k_resolve did
  const uint32_t D = __builtin_amdgcn_readfirstlane(w.ctr[4]);
  for (uint32_t q = blockIdx.x * kBlock + threadIdx.x; q < D; q += gridDim.x * kBlock) {
    const uint32_t i = w.dirty[q], gi = off + i;
    f3 s, d;
    load_ray(rays, ld, gi, s, d);
    uint32_t patch = 0xFFFFFFFFu;
    const Hit h = evaluate_patch<kFast>(m, static_cast<uint32_t>(w.key[i]) >> 6, s, d, patch);
    store_hit(o.hits, ld, gi, h, patch);
  }
#endif
}

// The rays k_traverse could not take: the reference's full in-order scan, split into
// (overflow ray, patch slice) items so a few rays over a large mesh still fill the chip.  Each thread
// scans patches t, t+256, ... of its slice (strict <: per thread the lowest index wins ties), and each
// wave folds its (t order, patch index) lexicographic minimum into the ray's key with one atomicMin:
// the winner of the reference's single in-order scan.  k_finish evaluates the winning patch again
// (same arithmetic, same bits) and emits it.  (Waves walking a slice with scalar-loaded records for
// 64 rays at once, as k_intersect_scan does, measured 4x slower: the serial walk waits on each load.)
constexpr uint32_t kOvfSlice = kBlock * 8;  // patches per item
__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
  for (int k = 32; k >= 1; k >>= 1) {
    unsigned long long o = __shfl_xor(v, k, 64);
    v = o < v ? o : v;
  }
  return v;
}

// Follow-side retries and the overflow rays' full scans in one launch (both feed the per-ray keys
// k_finish reads; they are independent of each other): threads first take follow requests, then
// blocks take (overflow ray, patch slice) items.  With no overflow rays the second loop is empty --
// one launch per segment saved over separate kernels.
template <bool kFast>
__global__ __launch_bounds__(kBlock) BZR_RESOLVE_ATTR void k_resolve(MeshView m, const float *__restrict__ rays, uint32_t ld,
                                                    uint32_t off, uint32_t n, Work w) {
  const uint32_t F = __builtin_amdgcn_readfirstlane(w.ctr[0]);
#if BZR_ROWS_DIRECT
  for (uint32_t q0 = blockIdx.x * kBlock; q0 < F; q0 += gridDim.x * kBlock) {  // (whole waves: row_step votes)
    const uint32_t q = q0 + threadIdx.x;
    const bool todo = q < F;
    uint32_t ray = 0u, j = 0u, b = 0u, nbr = 0u;
    Hit h = no_hit();
    if (todo) {
      const uint2 pr = w.pairs[w.fol[q]];
      ray = pr.x & kRayMask;
      j = pr.x >> 26;
      b = pr.y & ~(3u << 30);
      const uint32_t what = pr.y >> 30;
      f3 s, d;
      load_pair_ray(w.aos, rays, ld, off, ray, s, d);
      nbr = __float_as_uint(m.full[(size_t)rec::kWords * b + rec::kNeigh + what]);
      Patch pa = load_patch(m.full + (size_t)rec::kWords * nbr);
      h = patch_intersect<false, kFast>(pa, s, d, true);
    }
    // (a follow result ranks at its candidate b)
    if (w.ro.rows) row_step(w.ro, w.key, todo && h.what == kIntersect, ray, j, b, h, nbr);
    else if (todo && h.what == kIntersect) record(w.slot, n, ray, j, b, h, nbr, &w.key[ray]);
  }
#else
  for (uint32_t q = blockIdx.x * kBlock + threadIdx.x; q < F; q += gridDim.x * kBlock) {
    const uint2 pr = w.pairs[w.fol[q]];
    const uint32_t ray = pr.x & kRayMask, j = pr.x >> 26, b = pr.y & ~(3u << 30), what = pr.y >> 30;
    f3 s, d;
    load_pair_ray(w.aos, rays, ld, off, ray, s, d);
    const uint32_t nbr = __float_as_uint(m.full[(size_t)rec::kWords * b + rec::kNeigh + what]);
    Patch pa = load_patch(m.full + (size_t)rec::kWords * nbr);
    Hit h = patch_intersect<false, kFast>(pa, s, d, true);
    if (h.what == kIntersect) record(w.slot, n, ray, j, b, h, nbr, &w.key[ray]);  // ranks at its candidate
  }
#endif
  const uint32_t V = __builtin_amdgcn_readfirstlane(w.ctr[1]);
  const uint32_t S = (m.n + kOvfSlice - 1) / kOvfSlice;
  const uint64_t items = (uint64_t)V * S;  // 64-bit: 2^20-ray chunks x slices of meshes above ~8M patches
  for (uint64_t item = blockIdx.x; item < items; item += gridDim.x) {
    const uint32_t q = (uint32_t)(item / S), lo = (uint32_t)(item - (uint64_t)q * S) * kOvfSlice, hi = min(m.n, lo + kOvfSlice);
    const uint32_t i = w.ovf[q];
    f3 s, d;
    load_pair_ray(w.aos, rays, ld, off, i, s, d);
    float best_t = FLT_MAX;
    uint32_t best_b = 0xFFFFFFFFu;
    // (not unrolled: newton_tail's wave vote in div_heights is a convergent operation)
    for (uint32_t b = lo + threadIdx.x; b < hi; b += kBlock) {
      const float4 *qq = m.planar + 4u * b;
      if (!planar_gate(qq[0], qq[1], qq[2], qq[3], s, d)) continue;
      uint32_t src;
      Hit h = evaluate_patch<kFast>(m, b, s, d, src);
      if (h.what == kIntersect && h.t < best_t) {
        best_t = h.t;
        best_b = b;
      }
    }
    const unsigned long long win =
        wave_min_u64(best_b != 0xFFFFFFFFu ? ((unsigned long long)t_order(best_t) << 32) | best_b : ~0ull);
    if ((threadIdx.x & 63u) == 0 && win != ~0ull) atomicMin(&w.key[i], win);
  }
}

__global__ void k_count(Work w, uint32_t nb, unsigned long long *__restrict__ counters) {
  if (threadIdx.x != 0) return;
  counters[BZR_COUNTER_SEGMENTS] += w.ctr[2];
  counters[BZR_COUNTER_PAIRS] += w.ctr[3];
  counters[BZR_COUNTER_FOLLOWS] += w.ctr[0];
  counters[BZR_COUNTER_OVERFLOW_RAYS] += w.ctr[1];
  counters[BZR_COUNTER_DIRTY_ROWS] += w.ctr[4];
  // k_newton_lane's chunks; Newton passes = dense chunks + those
  const unsigned long long tot = w.offs[nb];
  const uint32_t sparse_chunks = (static_cast<uint32_t>(tot) + 63u) / 64u;
  counters[BZR_COUNTER_LANE_CHUNKS] += sparse_chunks;
  counters[BZR_COUNTER_NEWTON_ROUNDS] += static_cast<uint32_t>(tot >> 32) + sparse_chunks;
}

// Exclusive prefix sum of bucket_split(hist) in one block (meshes of up to kScanSmall - 1 patches; larger
// ones use hipCUB over the same values): offs[i] = sum of BucketSplit(hist[j]) over j < i.  (k_place clears
// the histogram.)
constexpr uint32_t kScanThreads = 1024, kScanPer = 8, kScanSmall = kScanThreads * kScanPer;
__global__ __launch_bounds__(kScanThreads) void k_scan_small(const uint32_t *__restrict__ hist,
                                                             unsigned long long *__restrict__ offs, uint32_t count) {
  __shared__ unsigned long long wave_total[kScanThreads / 64];
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6, base = t * kScanPer;
  unsigned long long v[kScanPer], sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanPer; ++k) {
    v[k] = base + k < count ? BucketSplit()(hist[base + k]) : 0ull;
    sum += v[k];
  }
  unsigned long long x = sum;  // inclusive scan over the wave
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const unsigned long long y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) wave_total[wv] = x;
  __syncthreads();
  unsigned long long before = 0;
  for (uint32_t k = 0; k < wv; ++k) before += wave_total[k];
  unsigned long long run = before + x - sum;
#pragma unroll
  for (uint32_t k = 0; k < kScanPer; ++k) {
    if (base + k < count) offs[base + k] = run;
    run += v[k];
  }
}

// ------------------------------------------------------------ fused path (default)
// One kernel per call: each wave takes 64 rays and runs every segment of them (one BezierMesh::intersect,
// or the whole refraction chain) without leaving the wave.  Per segment (trace_segment):
//  - the wave walks the lens BVH as k_traverse does and collects, in LDS, each leaf whose exact planar
//    gate passes for some lanes (wave-uniform patch index + lane mask, up to kEntries per batch);
//  - the collected leaves run through ONE Newton site, in order: the lanes that passed run
//    BezierTriangle::intersect with the patch record in SGPRs (uniform constant-address loads); lanes
//    whose result is follow-side K retry the named neighbour with cNone (reference/bezierMesh.cpp:212-216;
//    the neighbour of side K is uniform too).  A retry whose neighbour is a collected leaf still to come
//    joins that leaf's pass; one whose neighbour already ran takes the result that pass parked for it
//    (below); only the rest take a pass of their own;
//  - parking (BZR_TRACE_SPEC): a leaf's pass also runs, in its otherwise idle lanes, the cNone evaluation
//    for the lanes of later leaves that neighbour it -- the retry those lanes would ask for -- and parks
//    the result in LDS (one per lane and segment; not for kModeHits, whose 12-word winner leaves no room).
// Each lane keeps the lexicographic minimum of (t order key, scanned patch index) -- the reference's
// strict-< in-order winner, as in the staged path -- with the winning hit in LDS.  The schedule decides
// which pass evaluates a (lane, patch, limit), never the evaluation or its key.  Nothing per pair leaves
// the CU: HBM sees the rays in and the results out.  A patch sits in one leaf, so a wave runs a patch's
// pass at most once per segment (plus retries that could neither join nor use a parked result); lanes
// that need neither idle through it (lane utilisation).  Rays whose origin lies beyond the
// tree's validity radius, or whose stack overflows, take the reference's in-order scan in the same wave
// (same Newton site, patches in index order).
struct TraceCtr {  // wave-uniform work counters (kCount)
  uint32_t nodes = 0, leaves = 0, gate_tests = 0, rounds = 0, pairs = 0, follows = 0, segments = 0, ovf = 0;
  uint32_t rounds_odd = 0, runs_odd = 0;  // odd chain segments (a lens's back surface): passes, pairs + follows
};
// BZR_TRACE_PRIO (default 3; 0 = off): wave priority (s_setprio) of k_trace's BVH walk phase, back to 0
// for the Newton passes.  The walk is a chain of dependent scalar loads with little VALU work; issuing
// it ahead of the VALU-bound passes of the CU's other waves keeps its loads in flight (cfg4 -3 %).
#ifndef BZR_TRACE_PRIO
#define BZR_TRACE_PRIO 3
#endif
#ifndef BZR_TRACE_ENTRIES
#define BZR_TRACE_ENTRIES 16
#endif
#ifndef BZR_TRACE_SPEC
#define BZR_TRACE_SPEC 1
#endif
// BZR_TRACE_PARK_HITS (default 1): park cNone results in the intersect kernel (kModeHits) as well: cfg5
// fused -7.8 % Newton passes, +3.2 % Mrays/s; cfg3 +1 % (profiles/r03_ab_cfg{5,3}_fused_parkhits.jsonl).
// BZR_TRACE_BUNDLE (default 1): k_trace walks the tree with the wave-bundle test in batches (trace_segment)
// instead of one node at a time with each lane's slab test (0; rim waves whose bundle is wide take that walk
// anyway).  Round 3 measured the 4-wide bundle walk slower on the chains (cfg4 +5 to +6 %, cfg2 +3 %; cfg5
// fused -7 %, profiles/r03s2_ab_trace_bundle.jsonl): the bundle setup and the per-level batches cost what
// the fewer slab tests saved.  Round 4's integer DPP reductions and two-level batches (BZR_TRACE_WIDE) turn
// it around: bench.py with frames in flight, same bits, cfg4 11 074 -> 11 525 Mrays/s (+4.1 %), cfg2 +1.1 %,
// cfg5 fused +14 %, cfg3 fused +0.7 % (profiles/r04_bench_ab_trace_wide.jsonl; one serialized frame is
// within 1 %: the walk's VALU is what overlapping frames compete for).
#ifndef BZR_TRACE_BUNDLE
#define BZR_TRACE_BUNDLE 1
#endif
#ifndef BZR_TRACE_PARK_HITS
#define BZR_TRACE_PARK_HITS 1
#endif
constexpr uint32_t kEntries = BZR_TRACE_ENTRIES;  // collected leaves per batch: power of two, <= 64
static_assert(kEntries >= 4 && kEntries <= 64 && (kEntries & (kEntries - 1)) == 0, "kEntries");
// Words kept per lane: the winner (all of BezierIntersection for kModeHits; what refraction reads
// otherwise: point, cos, normal) and a parked retry result (t, point, cos, normal).
template <int kMode>
struct TraceWords {
  static constexpr int kHit = kMode == kModeHits ? 12 : 7;
  // kModeHits parks the barycentrics too (11 words): 6.4 KB of LDS per wave, which its 6 waves per SIMD
  // (80 VGPRs) leave room for (24 waves x 6.4 KB <= 160 KB)
  static constexpr int kPark = !BZR_TRACE_SPEC ? 0 : (kMode != kModeHits ? 8 : (BZR_TRACE_PARK_HITS ? 11 : 0));
  // traversal stack entries: the bundle walk's batches push up to 64 children at once, so the refraction
  // kernels (4.6 KB of LDS per wave at 7 waves per SIMD) take twice BZR_STACK; the intersect kernel's LDS
  // (6.5 KB per wave at 6 waves per SIMD) has no room left
  static constexpr int kStackCap = (BZR_TRACE_BUNDLE && kMode != kModeHits) ? 2 * kStack : kStack;
};
template <int kMode>
struct TraceLds {  // per wave
  uint32_t stack[TraceWords<kMode>::kStackCap];
  float hit[TraceWords<kMode>::kHit][64];    // the lane's current winner (written only when it improves)
  unsigned long long emask[kEntries];        // collected leaves: gate ballot
  float bundle[kBundleWords];                // the always list's ray bundle (always_bundle_keep)
  uint32_t eid[kEntries];                    // and patch index
#if BZR_TRACE_BUNDLE
  uint32_t pend[64];                         // the bundle walk's queued leaf slots
#endif
  float park[TraceWords<kMode>::kPark ? TraceWords<kMode>::kPark : 1][64];
};

__device__ __forceinline__ uint32_t popc64(unsigned long long m) { return (uint32_t)__popcll(m); }
__device__ __forceinline__ unsigned long long uniform_u64(unsigned long long v) {
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)), lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  return ((unsigned long long)hi << 32) | lo;  // (readfirstlane returns int: widen the unsigned halves)
}
__device__ __forceinline__ bool lane_bit(unsigned long long m, uint32_t lane) { return ((m >> lane) & 1ull) != 0ull; }

// The lane's candidate `h` from scanned patch `scan` (the hit itself from patch `src`).
template <int kMode>
__device__ __forceinline__ void consider(const Hit &h, uint32_t scan, uint32_t src, unsigned long long &best,
                                         TraceLds<kMode> &L, uint32_t lane) {
  if (h.what == kIntersect && h.t < FLT_MAX) {
    const unsigned long long k = ((unsigned long long)t_order(h.t) << 32) | scan;
    if (k < best) {
      best = k;
      if constexpr (kMode == kModeHits) {
        L.hit[0][lane] = h.t;
        L.hit[1][lane] = h.point.x;
        L.hit[2][lane] = h.point.y;
        L.hit[3][lane] = h.point.z;
        L.hit[4][lane] = h.cs;
        L.hit[5][lane] = h.bary.x;
        L.hit[6][lane] = h.bary.y;
        L.hit[7][lane] = h.bary.z;
        L.hit[8][lane] = h.normal.x;
        L.hit[9][lane] = h.normal.y;
        L.hit[10][lane] = h.normal.z;
        L.hit[11][lane] = __uint_as_float(src);
      } else {
        L.hit[0][lane] = h.point.x;
        L.hit[1][lane] = h.point.y;
        L.hit[2][lane] = h.point.z;
        L.hit[3][lane] = h.cs;
        L.hit[4][lane] = h.normal.x;
        L.hit[5][lane] = h.normal.y;
        L.hit[6][lane] = h.normal.z;
      }
    }
  }
}

// The lane's winner back from LDS (best != ~0).
template <int kMode>
__device__ __forceinline__ Hit winner(TraceLds<kMode> &L, uint32_t lane, uint32_t &patch) {
  Hit h = no_hit();
  h.what = kIntersect;
  if constexpr (kMode == kModeHits) {
    h.t = L.hit[0][lane];
    h.point = mk(L.hit[1][lane], L.hit[2][lane], L.hit[3][lane]);
    h.cs = L.hit[4][lane];
    h.bary = mk(L.hit[5][lane], L.hit[6][lane], L.hit[7][lane]);
    h.normal = mk(L.hit[8][lane], L.hit[9][lane], L.hit[10][lane]);
    patch = __float_as_uint(L.hit[11][lane]);
  } else {  // refract_hit reads point, cos and normal
    h.point = mk(L.hit[0][lane], L.hit[1][lane], L.hit[2][lane]);
    h.cs = L.hit[3][lane];
    h.normal = mk(L.hit[4][lane], L.hit[5][lane], L.hit[6][lane]);
    patch = 0xFFFFFFFFu;
  }
  return h;
}

// A parked cNone result: t (NaN when it is not an intersection, which consider() drops like a miss),
// point, cos, normal -- what consider() and the refraction read.
template <int kMode>
__device__ __forceinline__ void park(const Hit &h, TraceLds<kMode> &L, uint32_t lane) {
  if constexpr (TraceWords<kMode>::kPark > 0) {
    L.park[0][lane] = h.what == kIntersect ? h.t : __uint_as_float(0x7FC00000u);
    L.park[1][lane] = h.point.x;
    L.park[2][lane] = h.point.y;
    L.park[3][lane] = h.point.z;
    L.park[4][lane] = h.cs;
    L.park[5][lane] = h.normal.x;
    L.park[6][lane] = h.normal.y;
    L.park[7][lane] = h.normal.z;
    if constexpr (TraceWords<kMode>::kPark >= 11) {  // kModeHits: the whole BezierIntersection
      L.park[8][lane] = h.bary.x;
      L.park[9][lane] = h.bary.y;
      L.park[10][lane] = h.bary.z;
    }
  }
}
template <int kMode>
__device__ __forceinline__ Hit parked(TraceLds<kMode> &L, uint32_t lane) {
  Hit h = no_hit();
  if constexpr (TraceWords<kMode>::kPark > 0) {
    h.t = L.park[0][lane];
    h.point = mk(L.park[1][lane], L.park[2][lane], L.park[3][lane]);
    h.cs = L.park[4][lane];
    h.normal = mk(L.park[5][lane], L.park[6][lane], L.park[7][lane]);
    if constexpr (TraceWords<kMode>::kPark >= 11) h.bary = mk(L.park[8][lane], L.park[9][lane], L.park[10][lane]);
    h.what = kIntersect;
  }
  return h;
}

// One BezierMesh::intersect for the wave's active lanes; the winner is left in `best` / L.hit.
template <int kMode, bool kFast, bool kCount>
__device__ __forceinline__ void trace_segment(const MeshView &m, f3 s, f3 d, bool act, unsigned long long &best,
                                              TraceLds<kMode> &L, uint32_t lane, TraceCtr &ctr,
                                              uint32_t *pflag = nullptr) {
  constexpr bool kPark = TraceWords<kMode>::kPark > 0;
  constexpr uint32_t kNo = 0xFFFFFFFFu;
  constexpr int kCap = TraceWords<kMode>::kStackCap;
  best = ~0ull;
  const float amax = fmaxf(fmaxf(fabsf(s.x), fabsf(s.y)), fabsf(s.z));
  bool ovf = false;  // this lane takes the in-order full scan
  if (act && !(amax <= m.s_max)) {
    ovf = true;
    act = false;
  }
  const bool near_tier = !__any(act && !(amax <= m.s_near));
  const bzr_host::Bvh4Node *nodes = near_tier ? m.nodes_near : m.nodes;
  const bzr_host::Bvh4ObbNode *obb = near_tier ? m.obb_near : m.obb;
  const float4 *leaf = near_tier ? m.leaf_near : m.leaf;
  const f3 inv = mk(safe_inv(d.x), safe_inv(d.y), safe_inv(d.z));
  const f3 sinv = mk(s.x * inv.x, s.y * inv.y, s.z * inv.z);
  // The node to visit next is held in a scalar register (`next`); only the other hit children go to the
  // LDS stack, so a descent costs no LDS round trip (same visit order as pushing them all).
  int sp = 0;
  uint32_t next = (m.n > 0 && __any(act)) ? 0u : kNo;
  unsigned long long next_hm = 0ull;  // the lanes whose rays hit `next`'s box
  uint32_t scan = kNo;                // next patch of the full scan (kNo: not scanning)
  uint32_t join = kNo, join_src = 0;  // a retry waiting for a later leaf's pass: that leaf, scanned patch
  uint32_t parked_nb = kNo;           // the patch whose cNone result is parked for this lane
  // the always list: batches of 64 patches bundle-tested against the wave (uniform state; the bundle is
  // built once per segment into LDS, so no register holds it across the walk and the Newton passes)
  uint32_t ab = (m.n_always && __any(act)) ? 0u : (m.n_always + 63u) / 64u;  // next batch
  unsigned long long am = 0ull;  // the current batch's patches left to gate-test
  bool bwalk = false;  // this wave-segment takes the bundle walk
#if BZR_TRACE_BUNDLE
  // The bundle walk: the wave's active rays as one bundle (bundle_box), the tree taken in batches of up to
  // 16 nodes -- one child per lane -- from the top of the LDS stack; hit inner children are pushed, hit
  // leaves queued (L.pend) and gate-tested one by one with every active lane's own exact planar gate.
  uint32_t npend = 0, pi = 0;  // queued leaves, next to gate-test (uniform)
  const float4 *kids = near_tier ? m.kids_near : m.kids;
  // the walk choice, per wave-segment: a bundle whose directions spread wider than BZR_BUNDLE_SPREAD (rim
  // waves of refracted rays, incoherent batches) walks per lane instead -- its hull would reach far more
  // boxes than its rays do
  bool narrow = false;  // else every node is tested per lane (the oriented-box nodes always are)
  if (next != kNo) {
    narrow = bundle_setup_dpp(act, s, d, L.bundle, lane) <= BZR_BUNDLE_SPREAD;
#if BZR_BUNDLE_ALWAYS_NARROW
    narrow = true;  // (A/B knob: no per-lane walk for wide bundles)
#endif
    if (lane == 0u) L.stack[0] = 0u;
    sp = 1;
    next = kNo;
    bwalk = true;
  }
#endif
#if BZR_TRACE_PAIRSYNC
  bool seg_done = false;  // this wave has no batch left in the segment (its partner may)
#endif
  for (;;) {
    uint32_t ne = 0;  // collected leaves (uniform)
#if BZR_TRACE_PAIRSYNC
    // meeting point A: where two-wave lending would swap the waves' entry lists; the loop
    // ends once both waves are done, and a done wave keeps meeting its partner with empty batches
    if (lane == 0u) pflag[threadIdx.x >> 6] = seg_done ? 1u : 0u;
    __syncthreads();
    if (pflag[0] && pflag[1]) break;
    if (!seg_done) {
#endif
#if BZR_TRACE_PRIO
    __builtin_amdgcn_s_setprio(BZR_TRACE_PRIO);  // the walk is latency-bound: issue it ahead of Newton passes
#endif
#if BZR_TRACE_BUNDLE
    while (bwalk && ne < kEntries) {
      if (pi < npend) {  // a queued leaf: every active lane's planar gate
#if BZR_TRACE_BLEAF_PAIRS
        // two queued leaves per step when the entry list has room for both: both records in flight, one wait
        const bool two = pi + 1u < npend && ne + 1u < kEntries;
        const uint32_t slot0 = __builtin_amdgcn_readfirstlane(L.pend[pi]);
        const uint32_t slot1 = __builtin_amdgcn_readfirstlane(L.pend[two ? pi + 1u : pi]);
        pi += two ? 2u : 1u;
        u32x16 r0, r1;
        asm volatile("s_load_dwordx16 %0, %2, 0x0\n\ts_load_dwordx16 %1, %3, 0x0\n\ts_waitcnt lgkmcnt(0)"
                     : "=&s"(r0), "=&s"(r1)
                     : "s"(leaf + 4u * slot0), "s"(leaf + 4u * slot1));
        if (kCount) {
          ctr.leaves += two ? 2u : 1u;
          ctr.gate_tests += (two ? 2u : 1u) * popc64(__ballot(act));
        }
        const unsigned long long pm0 =
            __ballot(act & planar_gate(leaf_q(r0, 0), leaf_q(r0, 1), leaf_q(r0, 2), leaf_q(r0, 3), s, d));
        if (pm0) {
          if (lane == 0u) {
            L.eid[ne] = r0[15];
            L.emask[ne] = pm0;
          }
          ++ne;
        }
        if (two) {
          const unsigned long long pm1 =
              __ballot(act & planar_gate(leaf_q(r1, 0), leaf_q(r1, 1), leaf_q(r1, 2), leaf_q(r1, 3), s, d));
          if (pm1) {
            if (lane == 0u) {
              L.eid[ne] = r1[15];
              L.emask[ne] = pm1;
            }
            ++ne;
          }
        }
#else
        const uint32_t slot = __builtin_amdgcn_readfirstlane(L.pend[pi]);
        ++pi;
        const u32x16 r = *((const cu32x16 *)(uintptr_t)leaf + slot);
        const bool pass = act & planar_gate(leaf_q(r, 0), leaf_q(r, 1), leaf_q(r, 2), leaf_q(r, 3), s, d);
        if (kCount) {
          ++ctr.leaves;
          ctr.gate_tests += popc64(__ballot(act));
        }
        const unsigned long long pm = __ballot(pass);
        if (pm) {
          if (lane == 0u) {
            L.eid[ne] = r[15];
            L.emask[ne] = pm;
          }
          ++ne;
        }
#endif
        continue;
      }
      if (sp == 0) break;
      pi = npend = 0;
      const uint32_t top = __builtin_amdgcn_readfirstlane(L.stack[sp - 1]);
      if (!narrow || (top & bzr_host::kObbFlag)) {  // one node, its children tested by each lane's own ray
        --sp;
        if (kCount) ++ctr.nodes;
        bool hit[4];
        uint32_t ch[4];
        // (the reciprocals computed here, not kept from the segment's start: wide waves are rare, and 6
        // registers live across the Newton passes would cost occupancy)
        const f3 linv = mk(safe_inv(d.x), safe_inv(d.y), safe_inv(d.z));
        node_children(nodes, obb, top, act, s, d, mk(s.x * linv.x, s.y * linv.y, s.z * linv.z), linv, hit, ch);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const unsigned long long hm = __ballot(hit[c]);
          if (hm == 0ull) continue;
          if (ch[c] & bzr_host::kLeafFlag) {
            if (lane == 0u) L.pend[npend] = ch[c] & ~bzr_host::kLeafFlag;
            ++npend;
          } else if (sp < kCap) {
            if (lane == 0u) L.stack[sp] = ch[c];
            ++sp;
          } else if (lane_bit(hm, lane)) {
            ovf = true;  // traversal stack exhausted: these lanes take the full scan
          }
        }
        continue;
      }
      bool full;
      uint32_t k;
#if BZR_TRACE_WIDE
      npend = bundle_batch<kCap, 16>(near_tier ? m.wide_near : m.wide, L.stack, sp, L.pend, L.bundle, lane, full, k);
#else
      npend = bundle_batch<kCap>(kids, L.stack, sp, L.pend, L.bundle, lane, full, k);
#endif
      if (full) ovf |= act;  // traversal stack exhausted: every active lane takes the full scan
      if (kCount) ctr.nodes += k;
    }
#else
    while ((next != kNo || sp > 0) && ne + 4u <= kEntries) {
      const uint32_t node = next != kNo ? next : __builtin_amdgcn_readfirstlane(L.stack[--sp]);
      next = kNo;
      if (kCount) ++ctr.nodes;
      bool hit[4];
      uint32_t ch[4];
      node_children(nodes, obb, node, act, s, d, sinv, inv, hit, ch);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const unsigned long long hm = __ballot(hit[c]);
        if (hm == 0ull) continue;
        if (ch[c] & bzr_host::kLeafFlag) {
          const u32x16 r = *((const cu32x16 *)(uintptr_t)leaf + (ch[c] & ~bzr_host::kLeafFlag));
          const float4 g0 = make_float4(__uint_as_float(r[0]), __uint_as_float(r[1]), __uint_as_float(r[2]), __uint_as_float(r[3]));
          const float4 g1 = make_float4(__uint_as_float(r[4]), __uint_as_float(r[5]), __uint_as_float(r[6]), __uint_as_float(r[7]));
          const float4 g2 = make_float4(__uint_as_float(r[8]), __uint_as_float(r[9]), __uint_as_float(r[10]), __uint_as_float(r[11]));
          const float4 g3 = make_float4(__uint_as_float(r[12]), __uint_as_float(r[13]), __uint_as_float(r[14]), 0.0f);
          const bool pass = hit[c] & planar_gate(g0, g1, g2, g3, s, d)
#if BZR_DIAG_WALK2
                            & planar_gate(g0, g1, g2, g3, opaque(s), opaque(d))
#endif
              ;
          if (kCount) {
            ++ctr.leaves;
            ctr.gate_tests += popc64(hm);
          }
          const unsigned long long pm = __ballot(pass);
          if (pm) {
            if (lane == 0u) {
              L.eid[ne] = r[15];
              L.emask[ne] = pm;
            }
            ++ne;
          }
        } else {
          if (next != kNo) {
            if (sp < kCap) L.stack[sp++] = next;
            else if (lane_bit(next_hm, lane)) ovf = true;  // traversal stack exhausted: these lanes take the full scan
          }
          next = ch[c];
          next_hm = hm;
        }
      }
    }
#endif
    // tree done: the always list (patches without a proven gate region, bvh.cpp), gate-tested by every
    // wave-segment -- the candidates no box may cull
    while (next == kNo && sp == 0 && ne < kEntries) {  // (bundle walk: its leaf queue is empty here too)
      if (am == 0ull) {
        if (ab * 64u >= m.n_always) break;
        if (ab == 0u && !BZR_TRACE_BUNDLE) bundle_to_lds(act, s, d, L.bundle, lane);
        am = __ballot(always_bundle_keep(m.always, ab * 64u + lane, m.n_always, L.bundle));
        ++ab;
        continue;
      }
      const uint32_t k = (ab - 1u) * 64u + __builtin_ctzll(am);
      am &= am - 1ull;
      uint32_t b;
      const bool pass = always_gate(m.always, k, act, s, d, b);
      if (kCount) {
        ++ctr.leaves;
        ctr.gate_tests += popc64(__ballot(act));
      }
      const unsigned long long pm = __ballot(pass);
      if (pm) {
        if (lane == 0u) {
          L.eid[ne] = b;
          L.emask[ne] = pm;
        }
        ++ne;
      }
    }
    if (ne == 0u) {  // tree done: the reference's in-order scan for the lanes that could not use it
#if BZR_TRACE_PAIRSYNC
#define BZR_SEG_END       \
  {                       \
    seg_done = true;      \
    goto pair_b;          \
  }
#else
#define BZR_SEG_END break;
#endif
      if (scan == kNo) {
        if (!__any(ovf)) BZR_SEG_END
        scan = 0;
        if (kCount) ctr.ovf += popc64(__ballot(ovf));
      }
      bool pass = false;
      for (; scan < m.n; ++scan) {
        const float4 *g = m.planar + 4u * scan;  // wave-uniform address -> scalar loads
        pass = ovf && planar_gate(g[0], g[1], g[2], g[3], s, d);
        if (__any(pass)) break;
      }
      if (scan >= m.n) BZR_SEG_END
#undef BZR_SEG_END
      const unsigned long long pm = __ballot(pass);
      if (lane == 0u) {
        L.eid[0] = scan;
        L.emask[0] = pm;
      }
      ne = 1;
      ++scan;
    }
#if BZR_TRACE_PAIRSYNC
    }  // !seg_done
  pair_b:
    __syncthreads();  // meeting point B: where lending would hand the borrowed lanes' results back
    if (seg_done) ne = 0u;
#endif
    // the collected leaves' passes, in order
#if BZR_TRACE_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
    for (uint32_t e = 0; e < ne; ++e) {
      const uint32_t b = __builtin_amdgcn_readfirstlane(L.eid[e]);
      const auto hp = uniform_patch(m.full, b);
      const bool run0 = lane_bit(uniform_u64(L.emask[e]), lane);
      const bool joined = join == b;  // an earlier leaf's retry on this one
      const uint32_t sidx = joined ? join_src : b;
      if (joined) join = kNo;
      bool spec = false;  // park this leaf's cNone result for lanes of later leaves that neighbour it
      if (kPark && e + 1u < ne) {
        unsigned long long sm = 0ull;
#pragma unroll
        for (uint32_t side = 0; side < 3u; ++side) {
          const uint32_t nb = __float_as_uint(hp.r[rec::kNeigh + side]);
          const unsigned long long later = __ballot(lane > e && lane < ne && L.eid[lane & (kEntries - 1u)] == nb);
          if (later) sm |= uniform_u64(L.emask[__builtin_ctzll(later)]);
        }
        spec = lane_bit(sm, lane) && !run0 && !joined && parked_nb == kNo;
      }
      if (kCount) {
        ++ctr.rounds;
        ctr.pairs += popc64(__ballot(run0));
        ctr.follows += popc64(__ballot(joined));
      }
      uint32_t what = kNone;
      if (run0 || joined || spec) {
#if BZR_DIAG_NEWTON2
        // the extra evaluation first, folded to one word, so it adds ~1 live register to the real one
        const Hit h2 = patch_intersect<false, kFast>(hp, opaque(s), opaque(d), joined || spec);
        const uint32_t k2 = __float_as_uint(h2.t) ^ h2.what ^ __float_as_uint(h2.normal.x) ^ __float_as_uint(h2.point.y);
        Hit h = patch_intersect<false, kFast>(hp, s, d, joined || spec);
        if (k2 != (__float_as_uint(h.t) ^ h.what ^ __float_as_uint(h.normal.x) ^ __float_as_uint(h.point.y)))
          h.what = kNone;  // never (the same evaluation): keeps h2's whole evaluation
#else
        const Hit h = patch_intersect<false, kFast>(hp, s, d, joined || spec);
#endif
        if (spec) {
          park(h, L, lane);
          parked_nb = b;
        } else {
          consider(h, sidx, b, best, L, lane);
          if (!joined) what = h.what;
        }
      }
      for (uint32_t side = 0; side < 3u; ++side) {
        bool fl = run0 && what == side;
        if (!__any(fl)) continue;
        const uint32_t nb = __float_as_uint(hp.r[rec::kNeigh + side]);
        if (kPark) {  // computed by an earlier pass
          const bool use = fl && parked_nb == nb;
          if (use) {
            consider(parked(L, lane), b, nb, best, L, lane);
            fl = false;
          }
          if (kCount) ctr.follows += popc64(__ballot(use));
          if (!__any(fl)) continue;
        }
        // the neighbour among the leaves still to come: the retry joins its pass
        const unsigned long long later = __ballot(lane > e && lane < ne && L.eid[lane & (kEntries - 1u)] == nb);
        if (later) {
          const unsigned long long fm = uniform_u64(L.emask[__builtin_ctzll(later)]);
          if (fl && join == kNo && !lane_bit(fm, lane)) {
            join = nb;
            join_src = b;
            fl = false;
          }
        }
        if (!__any(fl)) continue;
        if (kCount) {
          ++ctr.rounds;
          ctr.follows += popc64(__ballot(fl));
        }
        const auto pa = uniform_patch(m.full, nb);
        if (fl) {
          const Hit h = patch_intersect<false, kFast>(pa, s, d, true);
          consider(h, b, nb, best, L, lane);
        }
      }
    }
  }
}

// Trace job of one launch.  Modes: kModeHits (one BezierMesh::intersect per ray -> hits), kModeRefract
// (one BezierLens::refract -> ray', status), kModeStage (the chain over lenses [0, count): refract(INSIDE)
// then refract(OUTSIDE) per lens, a NONE ends the ray -- reference/test.cpp:376-401).
struct TraceJob {
  const float *rays;         // input [6][n]
  float *hits;               // kModeHits [13][n]
  float *out_rays;           // kModeRefract / kModeStage [6][n] (may alias rays in kModeStage)
  uint32_t *status;          // kModeRefract / kModeStage [n]
  uint32_t *segments;        // kModeStage, optional [n]
  const uint32_t *expected;  // kModeRefract: per ray, or null -> expected_all
  const uint32_t *alive_in;  // kModeStage: rays with alive_in[i] == NONE are skipped and left untouched
  uint32_t expected_all;
  uint32_t n;
  uint32_t ld;               // row stride of rays / out_rays / hits (>= n)
  unsigned long long *wave_clock;  // optional test hook: [2 * waves] start, duration (s_memtime ticks)
  uint32_t wave_real;              // wave_clock holds [4 * waves]: + s_memrealtime start, duration (100 MHz)
  const uint32_t *order;           // optional: block b traces tile order[b] (cost-ordered dispatch, run_fused)
  uint32_t *cost;                  // optional: per tile, its cost bin (sched_bin of the block's duration)
};

// BZR_TRACE_WPE (default 6): amdgpu_waves_per_eu lower bound for k_trace.  The chain kernel needs 72 VGPRs
// (7 waves per SIMD) by itself; the intersect kernel (kModeHits: a 12-word winner) would take 82 (5 waves)
// since the always list's bundle code, and the bound holds it at 80 (6 waves, as before) without scratch.
#ifndef BZR_TRACE_WPE
#define BZR_TRACE_WPE 6
#endif
// BZR_TRACE_WPE_CHAIN (default BZR_TRACE_WPE): the same bound for the refraction kernels (kModeRefract,
// kModeStage), which hold 72 VGPRs = 7 waves per SIMD by themselves (7 here trades SGPRs for spills).
#ifndef BZR_TRACE_WPE_CHAIN
#define BZR_TRACE_WPE_CHAIN BZR_TRACE_WPE
#endif
#if BZR_TRACE_WPE
#define BZR_TRACE_ATTR __attribute__((amdgpu_waves_per_eu(kMode == kModeHits ? BZR_TRACE_WPE : BZR_TRACE_WPE_CHAIN)))
#else
#define BZR_TRACE_ATTR
#endif
// Threads per k_trace block (BZR_TRACE_BLOCK): its waves share nothing but the CU, so one-wave blocks let
// a finished wave be replaced at once (waves run 1-4 segments; 64 vs 256: cfg4 -3 %, cfg5 -7 %).
// BZR_TRACE_PAIRSYNC (diagnostic A/B, default 0): two-wave k_trace blocks whose waves meet twice per collected
// batch, as lane lending between them would need, with nothing lent: the measured cost of
// the pairing alone, against scripts/pair_sim.py's bound on what lending could save.  Same bits
// and passes; cfg4 -8.4 %, cfg2 -8.6 % (profiles/r05_ab_pairsync.jsonl) against <= ~2 % lending could recover.
#ifndef BZR_TRACE_PAIRSYNC
#define BZR_TRACE_PAIRSYNC 0
#endif
#ifndef BZR_TRACE_BLOCK
#define BZR_TRACE_BLOCK (BZR_TRACE_PAIRSYNC ? 128 : 64)
#endif
constexpr int kTraceBlock = BZR_TRACE_BLOCK, kTraceWaves = kTraceBlock / 64;
// Which 64-ray tile block b takes (BZR_TRACE_XCD): 0 = the dispatch order itself (XCD x gets every 8th
// tile), 1 = xcd_contiguous (each XCD one contiguous range of the image), G > 1 = runs of G tiles dealt
// round-robin to the XCDs.  0 is the default: a lens covers the middle of the image, so contiguous
// ranges give the middle XCDs ~2x the work of the outer ones, and a lens's records fit every XCD's L2
// anyway (cfg4: 6.26 ms with 1, 5.85 with 16, 5.67 with 0; cfg5 fused within 1 %).
#ifndef BZR_TRACE_XCD
#define BZR_TRACE_XCD 0
#endif
__device__ __forceinline__ uint32_t trace_tile(uint32_t b, uint32_t nblocks) {
  return deal_blocks<BZR_TRACE_XCD>(b, nblocks);
}
// Cost-ordered dispatch (BZR_TRACE_SCHED, default on).  A frame's waves differ up to ~6x
// in duration (rim waves meet many patches), and the hardware dispatches blocks in index order as slots free
// up -- greedy list scheduling.  One frame alone therefore ends on whichever long waves were dispatched late.
// Each k_trace block records its duration's cost bin; k_sched_* order the tiles longest-first (a counting
// sort over kSchedBins classes, 4 per octave of cycles), and the context's next fused call of the same size
// dispatches in that order: longest-processing-time-first list scheduling.  Every tile is traced exactly
// once either way and waves share nothing, so the output bits do not depend on the order.
#ifndef BZR_TRACE_SCHED
#define BZR_TRACE_SCHED 1
#endif
// BZR_TRACE_SCHED_REFRESH (default 16): the order is rebuilt from the latest costs on the first call of a size
// and then every this many calls (the three order kernels cost a short frame with others in flight ~8 % when
// run on every call; the costs of a frame loop's tiles barely change from frame to frame).
#ifndef BZR_TRACE_SCHED_REFRESH
#define BZR_TRACE_SCHED_REFRESH 16
#endif
// BZR_TRACE_SCHED_OCT (default 4): cost classes per octave of cycles (1, 2 or 4).  Within a class the tiles keep
// roughly their input order (each k_sched_place block reserves its tiles' places in dispatch order), so coarser
// classes keep more of the input order's locality.
#ifndef BZR_TRACE_SCHED_OCT
#define BZR_TRACE_SCHED_OCT 4
#endif
constexpr uint32_t kSchedBins = 128, kSchedMinTiles = 2048, kSchedThreads = 256;
__device__ __forceinline__ uint32_t sched_bin(unsigned long long cycles) {
  const uint32_t c = static_cast<uint32_t>(cycles > 0xFFFFFFFFull ? 0xFFFFFFFFull : cycles) | 4u;
  const uint32_t lg = 31u - __clz(c);                           // >= 2
  constexpr uint32_t kSub = BZR_TRACE_SCHED_OCT == 4 ? 2u : (BZR_TRACE_SCHED_OCT == 2 ? 1u : 0u);
  const uint32_t key = 4u * lg + (((c >> (lg - 2u)) & 3u) >> (2u - kSub) << (2u - kSub));  // <= 127
  return kSchedBins - 1u - key;                                  // bin 0 = the longest
}
// tiles per bin (hist zeroed by the previous k_sched_scan, or at allocation)
__global__ __launch_bounds__(kSchedThreads) void k_sched_count(const uint32_t *__restrict__ bin, uint32_t tiles,
                                                               uint32_t *__restrict__ hist) {
  __shared__ uint32_t h[kSchedBins];
  for (uint32_t k = threadIdx.x; k < kSchedBins; k += kSchedThreads) h[k] = 0u;
  __syncthreads();
  const uint32_t t = blockIdx.x * kSchedThreads + threadIdx.x;
  if (t < tiles) atomicAdd(&h[bin[t] & (kSchedBins - 1u)], 1u);
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < kSchedBins; k += kSchedThreads)
    if (h[k]) atomicAdd(&hist[k], h[k]);
}
// offs = exclusive scan of hist; hist back to zero for the next count
__global__ __launch_bounds__(kSchedBins) void k_sched_scan(uint32_t *__restrict__ hist, uint32_t *__restrict__ offs) {
  __shared__ uint32_t v[kSchedBins];
  const uint32_t k = threadIdx.x;
  const uint32_t mine = hist[k];
  v[k] = mine;
  __syncthreads();
  for (uint32_t s = 1; s < kSchedBins; s <<= 1) {
    const uint32_t a = k >= s ? v[k - s] : 0u;
    __syncthreads();
    v[k] += a;
    __syncthreads();
  }
  offs[k] = v[k] - mine;
  hist[k] = 0u;
}
// order[offs[bin] + rank within the bin] = tile (block-aggregated reservations)
__global__ __launch_bounds__(kSchedThreads) void k_sched_place(const uint32_t *__restrict__ bin, uint32_t tiles,
                                                               uint32_t *__restrict__ offs, uint32_t *__restrict__ order) {
  __shared__ uint32_t h[kSchedBins], base[kSchedBins];
  for (uint32_t k = threadIdx.x; k < kSchedBins; k += kSchedThreads) h[k] = 0u;
  __syncthreads();
  const uint32_t t = blockIdx.x * kSchedThreads + threadIdx.x;
  const uint32_t b = t < tiles ? (bin[t] & (kSchedBins - 1u)) : 0u;
  const uint32_t r = t < tiles ? atomicAdd(&h[b], 1u) : 0u;
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < kSchedBins; k += kSchedThreads)
    base[k] = h[k] ? atomicAdd(&offs[k], h[k]) : 0u;
  __syncthreads();
  if (t < tiles) order[base[b] + r] = t;
}
template <int kMode, bool kFast, bool kCount>
__global__ __launch_bounds__(kTraceBlock) BZR_TRACE_ATTR void k_trace(LensSet lenses, TraceJob job,
                                                                      unsigned long long *__restrict__ counters) {
  __shared__ TraceLds<kMode> lds[kTraceWaves];
#if BZR_TRACE_PAIRSYNC
  static_assert(kTraceWaves == 2, "BZR_TRACE_PAIRSYNC pairs the two waves of a 128-thread block");
  __shared__ uint32_t pflag[2];
#else
  uint32_t *const pflag = nullptr;
#endif
  const uint32_t lane = threadIdx.x & 63u;
  TraceLds<kMode> &L = lds[threadIdx.x >> 6];
  const uint32_t tile = job.order ? job.order[blockIdx.x] : trace_tile(blockIdx.x, gridDim.x);
  const uint32_t i = tile * kTraceBlock + threadIdx.x;
  const unsigned long long t_start = (job.wave_clock || job.cost) ? __builtin_amdgcn_s_memtime() : 0ull;
  const unsigned long long r_start = (job.wave_clock && job.wave_real) ? __builtin_amdgcn_s_memrealtime() : 0ull;
  const uint32_t n = job.n;
  TraceCtr ctr;
  bool alive = i < n;
  if (kMode == kModeStage && job.alive_in && alive) alive = job.alive_in[i] != BZR_RR_NONE;
  const bool traced = alive;
  f3 s = mk(0.0f, 0.0f, 0.0f), d = s;
  if (i < n) load_ray(job.rays, job.ld, i, s, d);
  const uint32_t nseg = kMode == kModeStage ? 2u * lenses.count : 1u;
  uint32_t st = BZR_RR_NONE, seg = 0;
  for (uint32_t k = 0; k < nseg; ++k) {
    if (!BZR_TRACE_PAIRSYNC && !__any(alive)) break;  // (paired waves both run every segment: same meetings)
    const MeshView &m = lenses.lens[k >> 1];
    unsigned long long best;
    const uint32_t r0 = ctr.rounds, w0 = ctr.pairs + ctr.follows;
    trace_segment<kMode, kFast, kCount>(m, s, d, alive, best, L, lane, ctr, pflag);
    if (kCount) {
      ctr.segments += popc64(__ballot(alive));
      if (k & 1u) {  // per-segment lane utilisation: front (even) vs back (odd) surfaces
        ctr.rounds_odd += ctr.rounds - r0;
        ctr.runs_odd += ctr.pairs + ctr.follows - w0;
      }
    }
    Hit h = no_hit();
    uint32_t patch = 0xFFFFFFFFu;
    if (best != ~0ull) h = winner(L, lane, patch);
    if (kMode == kModeHits) {
      if (alive) store_hit(job.hits, job.ld, i, h, patch);
    } else {
      const uint32_t expected = kMode == kModeRefract ? (job.expected ? (alive ? job.expected[i] : 0u) : job.expected_all)
                                                      : ((k & 1u) ? uint32_t(BZR_RR_OUTSIDE) : uint32_t(BZR_RR_INSIDE));
      f3 os, od;
      const uint32_t r = refract_hit(h, m.ri, s, d, expected, os, od);
      if (alive) {
        ++seg;
        st = r;
        if (r == BZR_RR_NONE) alive = false;
        else {
          s = os;
          d = od;
        }
      }
    }
  }
  if (kMode != kModeHits && traced) {
    store_ray(job.out_rays, job.ld, i, s, d);
    job.status[i] = st;
    if (kMode == kModeStage && job.segments) job.segments[i] = seg;
  }
  if (job.cost && threadIdx.x == 0u) job.cost[tile] = sched_bin(__builtin_amdgcn_s_memtime() - t_start);
  if (job.wave_clock && lane == 0u) {  // the wave's tile (ray index / 64): start tick and duration
    const unsigned long long t_end = __builtin_amdgcn_s_memtime();
    if (job.wave_real) {  // diagnostic: the wave's shader clock = d(s_memtime) / d(s_memrealtime) x 100 MHz
      const unsigned long long r_end = __builtin_amdgcn_s_memrealtime();
      job.wave_clock[4 * (i >> 6)] = t_start;
      job.wave_clock[4 * (i >> 6) + 1] = t_end - t_start;
      job.wave_clock[4 * (i >> 6) + 2] = r_start;
      job.wave_clock[4 * (i >> 6) + 3] = r_end - r_start;
    } else {
      job.wave_clock[2 * (i >> 6)] = t_start;
      job.wave_clock[2 * (i >> 6) + 1] = t_end - t_start;
    }
  }
  if (kCount && lane < 10u) {  // one atomic per counter per wave, spread over kCounterReplicas copies
    const uint32_t v[10] = {ctr.segments, ctr.pairs, ctr.follows, ctr.ovf, ctr.nodes, ctr.leaves, ctr.gate_tests,
                            ctr.rounds, ctr.rounds_odd, ctr.runs_odd};
    const uint32_t id[10] = {BZR_COUNTER_SEGMENTS, BZR_COUNTER_PAIRS, BZR_COUNTER_FOLLOWS, BZR_COUNTER_OVERFLOW_RAYS,
                             BZR_COUNTER_NODE_VISITS, BZR_COUNTER_LEAF_FETCHES, BZR_COUNTER_GATE_TESTS,
                             BZR_COUNTER_NEWTON_ROUNDS, BZR_COUNTER_ROUNDS_ODD, BZR_COUNTER_RUNS_ODD};
    uint32_t mine = 0, which = 0;
#pragma unroll
    for (uint32_t k = 0; k < 10u; ++k)
      if (lane == k) {
        mine = v[k];
        which = id[k];
      }
    const uint32_t rep = (blockIdx.x * kTraceWaves + (threadIdx.x >> 6)) % kCounterReplicas;
    if (mine) atomicAdd(&counters[(size_t)rep * BZR_COUNTER_COUNT + which], (unsigned long long)mine);
  }
}

// BZR_TRACE_RPL (default 1): rays per lane of the fused kernel.  2 or 4: k_trace_r (trace_pool.inc), one wave
// per 64 R rays with the Newton passes pooled over all of them.
#ifndef BZR_TRACE_RPL
#define BZR_TRACE_RPL 1
#endif
#if BZR_TRACE_RPL > 1
#include "trace_pool.inc"
#endif

// ------------------------------------------------------------ brute-force path
__global__ __launch_bounds__(kBlock) void k_intersect_scan(MeshView m, const float *__restrict__ rays, uint32_t n,
                                                           float *__restrict__ hits) {
  uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  f3 s, d;
  load_ray(rays, n, i, s, d);
  uint32_t patch;
  Hit h = mesh_intersect_scan(m, s, d, patch);
  store_hit(hits, n, i, h, patch);
}

__global__ __launch_bounds__(kBlock) void k_refract_scan(MeshView m, const float *__restrict__ rays,
                                                         const uint32_t *__restrict__ expected, uint32_t expected_all,
                                                         uint32_t n, float *__restrict__ out_rays,
                                                         uint32_t *__restrict__ out_status) {
  uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  f3 s, d, os, od;
  load_ray(rays, n, i, s, d);
  uint32_t patch;
  Hit h = mesh_intersect_scan(m, s, d, patch);
  uint32_t st = refract_hit(h, m.ri, s, d, expected ? expected[i] : expected_all, os, od);
  if (st == BZR_RR_NONE) {
    os = s;
    od = d;
  }
  store_ray(out_rays, n, i, os, od);
  out_status[i] = st;
}

__global__ __launch_bounds__(kBlock) void k_chain_scan(LensSet lenses, const float *__restrict__ rays, uint32_t n,
                                                       float *__restrict__ out_rays, uint32_t *__restrict__ out_status,
                                                       uint32_t *__restrict__ out_segments) {
  uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  f3 s, d;
  load_ray(rays, n, i, s, d);
  uint32_t st = BZR_RR_NONE, seg = 0;
  bool alive = true;
  for (uint32_t l = 0; l < lenses.count && alive; ++l) {
    for (uint32_t j = 0; j < 2u && alive; ++j) {
      f3 os, od;
      uint32_t patch;
      ++seg;
      Hit h = mesh_intersect_scan(lenses.lens[l], s, d, patch);
      st = refract_hit(h, lenses.lens[l].ri, s, d, j == 0 ? BZR_RR_INSIDE : BZR_RR_OUTSIDE, os, od);
      if (st == BZR_RR_NONE) {
        alive = false;
      } else {
        s = os;
        d = od;
      }
    }
  }
  store_ray(out_rays, n, i, s, d);
  out_status[i] = st;
  if (out_segments) out_segments[i] = seg;
}

template <bool kFast>
__global__ __launch_bounds__(kBlock) void k_patch(MeshView m, const uint32_t *__restrict__ idx,
                                                  const uint32_t *__restrict__ limit, const float *__restrict__ rays,
                                                  uint32_t n, float *__restrict__ hits) {
  uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  f3 s, d;
  load_ray(rays, n, i, s, d);
  uint32_t pi = idx[i];
  Hit h;
  if (pi < m.n) {
    Patch p = load_patch(m.full + (size_t)rec::kWords * pi);
    h = patch_intersect<false, kFast>(p, s, d, limit[i] != 0u);
  } else {
    h = no_hit();
    h.t = 0.0f;
  }
  store_hit(hits, n, i, h, pi);
}

// ------------------------------------------------------------ host helpers
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

MeshView view_of(const bzr_mesh *m, float ri = 1.0f) {
  return MeshView{m->planar, m->full, m->nodes, m->leaf, m->nodes_near, m->leaf_near, m->obb, m->obb_near,
                  m->always, m->kids, m->kids_near, m->wide, m->wide_near, m->n_always, m->n, m->s_max, m->s_near, ri};
}
unsigned grid_for(uint32_t n) { return (n + kBlock - 1) / kBlock; }
size_t round256(size_t b) { return (b + 255) & ~size_t(255); }

bzr_status ensure_buffer(void *&buf, size_t &have, size_t bytes) {
  if (have >= bytes) return BZR_OK;
  if (buf) BZR_HIP(hipFree(buf));
  buf = nullptr;
  have = 0;
  BZR_HIP(hipMalloc(&buf, bytes));
  have = bytes;
  return BZR_OK;
}

struct Staging {  // carves device buffers out of a context-owned allocation
  char *base;
  size_t off = 0;
  template <typename T>
  T *take(size_t count) {
    T *p = reinterpret_cast<T *>(base + off);
    off += round256(count * sizeof(T));
    return p;
  }
};

// The caller's rays into the kernels' rows `r` ([6][n] on the device): copied from host memory and/or
// transposed from [n][6] records (BZR_RAYS_AOS; a host source lands in `tmp` first).
bzr_status rays_in(bzr_ctx *ctx, const float *rays, float *r, uint32_t n, bool host, bool aos, float *tmp) {
  if (host) BZR_HIP(hipMemcpyAsync(aos ? tmp : r, rays, (size_t)n * 24, hipMemcpyHostToDevice, ctx->stream));
  if (aos) BZR_HIP(bzr_rays_relayout(ctx->stream, host ? tmp : rays, r, n, true));
  return BZR_OK;
}
// The kernels' output rows `d_out` to the caller's out_rays: transposed to [n][6] records (BZR_RAYS_AOS; for a
// host destination into `tmp` first) and/or copied to host memory (queued, not waited for).
bzr_status rays_out(bzr_ctx *ctx, const float *d_out, float *out_rays, uint32_t n, bool host, bool aos, float *tmp) {
  if (aos) BZR_HIP(bzr_rays_relayout(ctx->stream, d_out, host ? tmp : out_rays, n, false));
  if (host) BZR_HIP(hipMemcpyAsync(out_rays, aos ? tmp : d_out, (size_t)n * 24, hipMemcpyDeviceToHost, ctx->stream));
  return BZR_OK;
}

bzr_status check_ctx_mesh(bzr_ctx *ctx, const bzr_mesh *mesh) {
  if (!ctx) return set_error(BZR_ERR_INVALID_ARGUMENT, "null context");
  if (!mesh) return set_error(BZR_ERR_INVALID_ARGUMENT, "null mesh");
  if (mesh->device != ctx->device) return set_error(BZR_ERR_INVALID_ARGUMENT, "mesh lives on another device");
  return BZR_OK;
}

bool use_scan(uint32_t flags) { return (flags & BZR_ACCEL_NONE) != 0; }
bool use_fast(uint32_t flags) { return (flags & BZR_MODE_FAST) != 0; }
// Culled-path pipeline for a call of n rays over meshes of at most nb patches (include/bzr.h): forced by
// BZR_PIPELINE_STAGED / BZR_PIPELINE_FUSED, otherwise fused for dense batches (rays per patch >= 256;
// rays per patch stands in for how many patches a wave's 64 rays meet).  Chosen for callers that keep
// frames in flight (bench.py): cfg4 at 4096^2 (5461 rays per patch) and cfg2 at 1024^2
// (341) run fused -- cfg2 5593 vs 5205 Mrays/s at three / two frames in flight, though a lone cfg2 frame
// is faster staged; cfg3 (145) and cfg5 (223) run staged.  Meshes of kStagedPatchLimit patches or more
// (the staged key and pair encoding's limit) always run fused, which takes any mesh.
constexpr uint64_t kFusedRaysPerPatch = 256;
bool use_staged(uint32_t flags, uint64_t n, uint64_t nb) {
  if (flags & BZR_PIPELINE_STAGED) return true;
  if (flags & BZR_PIPELINE_FUSED) return false;
  return nb < kStagedPatchLimit && n < kFusedRaysPerPatch * nb;
}
// BZR_MODE_FAST runs on the culled pipeline's kernels only; the brute-force scan is the parity reference.
constexpr uint32_t kKnownFlags = BZR_DEVICE_PTRS | BZR_MODE_FAST | BZR_ACCEL_NONE | BZR_PIPELINE_STAGED | BZR_PIPELINE_FUSED;
// aos_ok: the call takes BZR_RAYS_AOS (the ray-batch entries: intersect, refract, trace_chain)
bzr_status check_flags(uint32_t flags, bool aos_ok = false) {
  if ((flags & BZR_RAYS_AOS) && !aos_ok) return set_error(BZR_ERR_INVALID_ARGUMENT, "BZR_RAYS_AOS is not accepted by this call");
  if (aos_ok) flags &= ~uint32_t(BZR_RAYS_AOS);
  if (flags & ~kKnownFlags) return set_error(BZR_ERR_INVALID_ARGUMENT, "unknown flag bits " + std::to_string(flags & ~kKnownFlags));
  if ((flags & BZR_PIPELINE_STAGED) && (flags & BZR_PIPELINE_FUSED))
    return set_error(BZR_ERR_INVALID_ARGUMENT, "BZR_PIPELINE_STAGED and BZR_PIPELINE_FUSED are exclusive");
  if (use_fast(flags) && use_scan(flags))
    return set_error(BZR_ERR_INVALID_ARGUMENT, "BZR_MODE_FAST needs the culled path (drop BZR_ACCEL_NONE)");
  return BZR_OK;
}

hipEvent_t take_event(bzr_ctx *ctx) {
  if (!ctx->spare.empty()) {
    hipEvent_t e = ctx->spare.back();
    ctx->spare.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

// Launch on `stream`; with timing enabled, bracket the launch with events on that stream.
template <typename... Args>
void launch_on(bzr_ctx *ctx, hipStream_t stream, dim3 block, int kernel_id, void (*kernel)(Args...), dim3 grid,
               typename std::decay<Args>::type... args) {
  const bool timed = ctx->timing && kernel_id >= 0;
  hipEvent_t a = nullptr, b = nullptr;
  if (timed) {
    a = take_event(ctx);
    b = take_event(ctx);
    (void)hipEventRecord(a, stream);
  }
  hipLaunchKernelGGL(kernel, grid, block, 0, stream, args...);
  if (timed) {
    (void)hipEventRecord(b, stream);
    ctx->marks.push_back({kernel_id, a, b});
  }
}
// Launch on the context's stream.
template <typename... Args>
void launch(bzr_ctx *ctx, int kernel_id, void (*kernel)(Args...), dim3 grid, typename std::decay<Args>::type... args) {
  launch_on(ctx, ctx->stream, dim3(kBlock), kernel_id, kernel, grid, args...);
}

// Event bracket around a group of launches (timing enabled only).
struct Span {
  bzr_ctx *ctx;
  int id;
  hipEvent_t a = nullptr;
  Span(bzr_ctx *c, int kernel_id) : ctx(c), id(kernel_id) {
    if (ctx->timing) {
      a = take_event(ctx);
      (void)hipEventRecord(a, ctx->stream);
    }
  }
  ~Span() {
    if (!a) return;
    hipEvent_t b = take_event(ctx);
    (void)hipEventRecord(b, ctx->stream);
    ctx->marks.push_back({id, a, b});
  }
};

// Blocks of `kernel` (kBlock threads) the device holds at once: the persistent-grid size.
template <typename K>
uint32_t resident_blocks(bzr_ctx *ctx, K kernel) {
  static thread_local std::vector<std::pair<const void *, uint32_t>> cache;  // (kernel, blocks) per device below
  const void *key = reinterpret_cast<const void *>(kernel);
  for (auto const &c : cache)
    if (c.first == key) return c.second;
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, 0) != hipSuccess || per_cu < 1) per_cu = 1;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess || cus < 1) cus = 256;
  uint32_t blocks = static_cast<uint32_t>(per_cu) * static_cast<uint32_t>(cus);
  cache.emplace_back(key, blocks);
  return blocks;
}

// BZR_TRAV_HYBRID's threshold: lanes a leaf's gate must pass for k_traverse to run its Newton pass in the wave
// (environment BZR_HYBRID_T, 1..64; 0 = list every leaf, round 5's pipeline; read once per process).
uint32_t hybrid_threshold() {
  static const uint32_t t = [] {
    const char *e = std::getenv("BZR_HYBRID_T");
    if (!e || !*e) return (uint32_t)BZR_HYBRID_T_DEFAULT;
    const long v = std::strtol(e, nullptr, 10);
    return (uint32_t)(v < 0 ? 0 : v > 64 ? 64 : v);
  }();
  return BZR_TRAV_HYBRID ? t : 0u;
}

// Grid of the persistent staged kernels (k_newton, k_resolve) in units of the device's resident capacity
// (A/B knobs, environment BZR_NEWTON_GRIDX / BZR_RESOLVE_GRIDX, 1..64, read once per process).  A grid
// of exactly the resident capacity holds every wave slot until the kernel ends, so another frame's kernels (frames
// in flight, their own streams) cannot start beside it; k x capacity ends in k generations of blocks, between
// which the dispatcher also takes the other streams' blocks.
uint32_t env_scale(const char *name, uint32_t dflt = 1u) {
  const char *e = std::getenv(name);
  if (!e || !*e) return dflt;
  const long v = std::strtol(e, nullptr, 10);
  return (uint32_t)(v < 1 ? 1 : v > 64 ? 64 : v);
}
// k_newton: 2 x the resident capacity on meshes of at least 2^17 patches, else 1 x (BZR_NEWTON_GRIDX overrides).
// Measured (profiles/r06_ab_gridx_cfg5.jsonl, same bits): cfg5 (301 056 patches, 8 M-ray chunks) k_newton 4.33 ->
// 4.15 ms per lone frame and +0.8 to +1.5 % at bench level on three boxes, 4 x / 8 x / 16 x lose (every wave's
// follow-list flush is an atomic on one counter); cfg3 (28 800 patches) k_newton 0.174 -> 0.205 ms lone, -1 to -2 %
// at bench level.
constexpr uint32_t kNewtonGrid2Patches = 1u << 17;
uint32_t newton_gridx(uint32_t nb) {
  static const uint32_t s = env_scale("BZR_NEWTON_GRIDX", 0u);
  return s ? s : nb >= kNewtonGrid2Patches ? 2u : 1u;
}
// k_resolve's block cap: BZR_RESOLVE_BLOCKS (absolute, 64..65536) if set, else 1024 x BZR_RESOLVE_GRIDX
uint32_t resolve_blocks() {
  static const uint32_t s = [] {
    const char *e = std::getenv("BZR_RESOLVE_BLOCKS");
    if (e && *e) {
      const long v = std::strtol(e, nullptr, 10);
      return (uint32_t)(v < 64 ? 64 : v > 65536 ? 65536 : v);
    }
    return 1024u * env_scale("BZR_RESOLVE_GRIDX");
  }();
  return s;
}

// Workspace of the culled path for chunks of up to `chunk` rays over meshes of up to `nb` patches.
using SplitIt = hipcub::TransformInputIterator<unsigned long long, BucketSplit, const uint32_t *>;
bzr_status ensure_work(bzr_ctx *ctx, uint32_t chunk, uint32_t nb, Work &w) {
  size_t cub_bytes = 0;
  const uint32_t hn = nb;  // histogram slots, one per patch
  BZR_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, cub_bytes, SplitIt(static_cast<const uint32_t *>(nullptr), BucketSplit()),
                                           static_cast<unsigned long long *>(nullptr), hn + 1, ctx->stream));
  const size_t cap = (size_t)kMaxCand * chunk;
  const size_t bytes = round256(32) + round256((size_t)(hn + 1) * 4) + round256((size_t)(hn + 1) * 8) + 2 * round256(cap * 4) +
                       round256((size_t)chunk * 4) + round256((size_t)chunk * 8) + round256(kSlotWords * cap * 4) +
                       round256((cap + 64 * ((size_t)nb + 1) + (BZR_TRAV_HYBRID ? cap : 0)) * 8) + round256(cap * 4) +
                       2 * round256((size_t)chunk * 4) + round256(((size_t)chunk + kAblockBlock - 1) / kAblockBlock * kAmaskWords * 8) +
                       (BZR_STAGED_AOS ? round256((size_t)chunk * 32) : 0) + round256(cub_bytes);
  const size_t had = ctx->work_bytes;
  if (bzr_status s = ensure_buffer(ctx->work, ctx->work_bytes, bytes)) return s;
  if (ctx->work_bytes != had) ctx->zero_ctr = nullptr;  // reallocated (possibly at the same address)
  Staging st{static_cast<char *>(ctx->work)};
  w.ctr = st.take<uint32_t>(8);
  w.hist = st.take<uint32_t>(hn + 1);
  w.offs = st.take<unsigned long long>(hn + 1);
  w.cand = st.take<uint32_t>(cap);
  w.rank = st.take<uint32_t>(cap);
  w.count = st.take<uint32_t>(chunk);
  w.key = st.take<unsigned long long>(chunk);
  w.slot = st.take<float>(kSlotWords * cap);
  // dense chunks (< 64 padding slots per patch) + sparse; then (BZR_TRAV_HYBRID) the in-wave follow requests' records
  w.pairs = st.take<uint2>(cap + 64 * ((size_t)nb + 1) + (BZR_TRAV_HYBRID ? cap : 0));
  w.fol = st.take<uint32_t>(cap);
  w.ovf = st.take<uint32_t>(chunk);
  w.dirty = st.take<uint32_t>(chunk);
  w.amask = st.take<unsigned long long>(((size_t)chunk + kAblockBlock - 1) / kAblockBlock * kAmaskWords);
  w.aos = BZR_STAGED_AOS ? st.take<float4>((size_t)2 * chunk) : nullptr;
  w.cub = st.take<char>(cub_bytes ? cub_bytes : 1);
  w.cub_bytes = cub_bytes;
  w.cap = static_cast<uint32_t>(cap);
  w.hbase = static_cast<uint32_t>(cap + 64 * ((size_t)nb + 1));
  w.hyb_t = hybrid_threshold();
  return BZR_OK;
}

// Rays per chunk of the staged path, whose workspace is ~2.7 KB per ray + 0.5 KB per patch: at most
// 2^BZR_CHUNK_LOG2 (8M rays, ~23 GB) and at most what a quarter of the device's free memory holds (at the
// context's first staged call), with the
// batch split into equal chunks (rounded to whole waves).  Measured on cfg5 (67M rays): 1M-ray chunks
// 28.3 ms per frame, 4M 21.4, 8M 20.0, 16M 20.0 -- small chunks leave the kernels short of waves.
#ifndef BZR_CHUNK_LOG2
#define BZR_CHUNK_LOG2 23
#endif
constexpr uint32_t kChunk = 1u << BZR_CHUNK_LOG2;
constexpr size_t kWorkBytesPerRay = (size_t)kMaxCand * (4 + 4 + 48 + 8 + 4 + (BZR_TRAV_HYBRID ? 8 : 0)) + 20 + (BZR_STAGED_AOS ? 32 : 0);
static_assert(BZR_CHUNK_LOG2 <= 26, "pair records hold a chunk's ray index in 26 bits");
static_assert((uint64_t)kMaxCand * kChunk * (BZR_TRAV_HYBRID ? 2 : 1) + 64ull * (kStagedPatchLimit + 1) < (1ull << 32),
              "32-bit pair indices");
static_assert(kMaxCand <= 64, "winner keys hold a list slot in 6 bits");
uint32_t chunk_for(bzr_ctx *ctx, uint64_t n) {
  if (!ctx->chunk_cap) {
    size_t free_b = 0, total_b = 0;
    uint64_t cap = kChunk;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b)
      cap = std::min<uint64_t>(cap, std::max<uint64_t>(free_b / 4 / kWorkBytesPerRay / 64 * 64, 64));
    ctx->chunk_cap = static_cast<uint32_t>(cap);
  }
  const uint64_t cap = ctx->chunk_cap, pieces = (n + cap - 1) / cap;
  if (pieces <= 1) return static_cast<uint32_t>(std::max<uint64_t>(n, 1));
  return static_cast<uint32_t>(std::min<uint64_t>(cap, ((n + pieces - 1) / pieces + 63) / 64 * 64));
}

// One BezierMesh::intersect per ray of rays [off, off + n) (+ refraction, per kMode).
template <int kMode, bool kFast>
bzr_status run_culled(bzr_ctx *ctx, const MeshView &mv, const float *rays, uint32_t ld, uint32_t off, uint32_t n,
                      const uint32_t *alive, const Out &o, Work &w) {
  const uint32_t nb = mv.n;
  const uint32_t hn = nb;
  const bool small_scan = hn + 1 <= kScanSmall;
  if (nb >= kStagedPatchLimit)  // (the automatic choice sends such meshes to the fused path, which takes any mesh)
    return set_error(BZR_ERR_INVALID_ARGUMENT, "staged path: mesh of " + std::to_string(nb) +
                                                   " patches, at or above 2^25; use BZR_PIPELINE_FUSED");
  if (!(ctx->zero_ctr == w.ctr && ctx->zero_hn >= hn))  // counters + histogram [0, hn] to zero
    BZR_HIP(hipMemsetAsync(w.ctr, 0, reinterpret_cast<char *>(w.hist + hn + 1) - reinterpret_cast<char *>(w.ctr),
                           ctx->stream));
  ctx->zero_ctr = nullptr;  // valid again only once this segment is fully enqueued
  unsigned long long *const ctr = (ctx->counting && ctx->counters) ? ctx->counters : nullptr;
  // BZR_ROWS_DIRECT: an intersect segment's Newton stage writes the hit rows itself (record_row)
  w.ro = RowOut{};
  if (kMode == kModeHits && BZR_ROWS_DIRECT && BZR_FINISH_NORAY && !BZR_TRAV_HYBRID)
    w.ro = RowOut{o.hits, ld, off, w.count, w.dirty, w.ctr + 4};
  if (BZR_TRAV_ABLOCK == 3 && mv.n_always > kAblockMin && mv.n_always <= kAblockMax) {  // pre-test kernel, then the walk
    Span sp(ctx, BZR_KERNEL_TRAVERSE);
    hipLaunchKernelGGL(k_always_mask, dim3((n + kAblockBlock - 1) / kAblockBlock), dim3(kAblockBlock), 0, ctx->stream, mv,
                       rays, ld, off, alive, n, w.amask);
    hipLaunchKernelGGL((k_traverse<kTravBlock, 3, kFast>), dim3((n + kTravBlock - 1) / kTravBlock), dim3(kTravBlock), 0,
                       ctx->stream, mv, rays, ld, off, alive, n, w, ctr);
  } else if (BZR_TRAV_ABLOCK && mv.n_always > kAblockMin && mv.n_always <= kAblockMax)  // block-level always-list pre-test
    launch_on(ctx, ctx->stream, dim3(kAblockBlock), BZR_KERNEL_TRAVERSE, k_traverse<kAblockBlock, BZR_TRAV_ABLOCK == 3 ? 1 : BZR_TRAV_ABLOCK, kFast>,
              dim3((n + kAblockBlock - 1) / kAblockBlock), mv, rays, ld, off, alive, n, w, ctr);
  else
    launch_on(ctx, ctx->stream, dim3(kTravBlock), BZR_KERNEL_TRAVERSE, k_traverse<kTravBlock, 0, kFast>,
              dim3((n + kTravBlock - 1) / kTravBlock), mv, rays, ld, off, alive, n, w, ctr);
  {
    Span sp(ctx, BZR_KERNEL_BUCKET);
    if (small_scan)
      hipLaunchKernelGGL(k_scan_small, dim3(1), dim3(kScanThreads), 0, ctx->stream, w.hist, w.offs, hn + 1);
    else
      BZR_HIP(hipcub::DeviceScan::ExclusiveSum(w.cub, w.cub_bytes, SplitIt(w.hist, BucketSplit()), w.offs, hn + 1,
                                               ctx->stream));
    launch(ctx, -1, k_place, dim3(grid_for(std::max(n, nb))), n, nb, w,
           (ctx->counting && ctx->counters) ? w.ctr + 3 : nullptr);
  }
  // persistent grid: the resident capacity of the device, never more than the worst-case chunk count
  const uint32_t gn = std::min<uint32_t>(std::max<uint32_t>((kMaxCand * n + kBlock - 1) / kBlock, 1u),
                                         resident_blocks(ctx, k_newton<kFast>) * newton_gridx(nb));
  launch(ctx, BZR_KERNEL_NEWTON, k_newton<kFast>, dim3(gn), mv.full, w.offs + hn, w.pairs, rays, ld, off, n, w.slot, w.key,
         w.fol, w.ctr, (const float4 *)w.aos, w.ro);
  launch(ctx, BZR_KERNEL_NEWTON_LANE, k_newton_lane<kFast>, dim3(std::min<uint32_t>(std::max<uint32_t>(n / 1024u, 1u), 1024u)),
         mv.full, w.offs + hn, w.pairs, rays, ld, off, n, w.slot, w.key, w.fol, w.ctr, (const float4 *)w.aos, w.ro);
  {  // follow retries + overflow rays (whose keys the Newton stage left untouched: their lists are empty)
    const uint64_t items = (uint64_t)n * ((nb + kOvfSlice - 1) / kOvfSlice);
    const uint32_t grid = std::max(std::min<uint32_t>(grid_for(n / 8 + 1), resolve_blocks()),
                                   (uint32_t)std::min<uint64_t>(items, BZR_OVERFLOW_BLOCKS));
    launch(ctx, BZR_KERNEL_FOLLOW, k_resolve<kFast>, dim3(std::max<uint32_t>(grid, 1u)), mv, rays, ld, off, n, w);
  }
  if (ctx->counting && ctx->counters)  // before k_finish, which clears the counters
    hipLaunchKernelGGL(k_count, dim3(1), dim3(64), 0, ctx->stream, w, nb, ctx->counters);
  if (kMode == kModeHits && BZR_FINISH_NORAY)  // the overflow rays first (k_finish clears their count)
    // (grid-stride over the overflow list, whose length only the device knows.  64 blocks: a batch whose rays all
    // lie beyond s_max re-evaluates them 16 K at a time, while k_resolve's full scan of the same rays costs a gate per
    // ray and patch; 512 blocks cost cfg3 frames ~1 % in launch for nothing on the bench configs)
    launch(ctx, BZR_KERNEL_FINISH, k_finish_ovf<kFast>, dim3(std::min<uint32_t>(grid_for(n), 64u)), mv, rays, ld, off,
           w, o);
  launch(ctx, BZR_KERNEL_FINISH, k_finish<kMode, kFast>, dim3(grid_for(n)), mv, rays, ld, off, n, w, o);
  BZR_HIP(hipGetLastError());
  ctx->zero_ctr = w.ctr;  // k_place cleared the histogram, k_finish the counters
  ctx->zero_hn = hn;
  return BZR_OK;
}

// The fused path: one k_trace launch for the whole job (no workspace, no chunking).
template <int kMode>
bzr_status run_fused(bzr_ctx *ctx, const LensSet &set, const TraceJob &job, uint32_t flags) {
  if (job.n == 0) return BZR_OK;
  const bool fast = use_fast(flags), count = ctx->counting && ctx->counters;
  const dim3 grid((job.n + kTraceBlock - 1) / kTraceBlock), block(kTraceBlock);
  TraceJob j = job;
  j.wave_clock = (ctx->wave_clock && ctx->wave_clock_cap >= (job.n + 63) / 64) ? ctx->wave_clock : nullptr;
  j.wave_real = ctx->wave_clock_real ? 1u : 0u;
  j.order = nullptr;
  j.cost = nullptr;
  const uint32_t tiles = grid.x;
  const bool sched = BZR_TRACE_SCHED && BZR_TRACE_RPL == 1 && tiles >= kSchedMinTiles;
  if (sched) {  // this call's tile costs; the order of the last call of the same size, if any
    if (ctx->sched_cap < tiles) {
      if (ctx->sched) BZR_HIP(hipFree(ctx->sched));
      ctx->sched = nullptr;
      ctx->sched_cap = ctx->sched_waves = 0;
      BZR_HIP(hipMalloc(&ctx->sched, ((size_t)2 * tiles + 2 * kSchedBins) * sizeof(uint32_t)));
      BZR_HIP(hipMemsetAsync(ctx->sched + (size_t)2 * tiles, 0, kSchedBins * sizeof(uint32_t), ctx->stream));
      ctx->sched_cap = tiles;
    }
    j.cost = ctx->sched;
    // the saved order belongs to a call of this size over the same lenses in the same mode (any other
    // call rebuilds it -- its bits would not change either way, the order is a permutation of whole tiles)
    uint64_t key = 0xcbf29ce484222325ull ^ (uint64_t)kMode;
    for (uint32_t l = 0; l < set.count; ++l)
      key = (key ^ reinterpret_cast<uintptr_t>(set.lens[l].full)) * 0x100000001b3ull;
    if (ctx->sched_key != key) {
      ctx->sched_key = key;
      ctx->sched_waves = 0;
    }
    if (ctx->sched_waves == tiles) {
      j.order = ctx->sched + ctx->sched_cap;
      ++ctx->sched_calls;
    } else {
      ctx->sched_calls = 0;
    }
  }
  const bool rebuild = sched && ctx->sched_calls % BZR_TRACE_SCHED_REFRESH == 0;
#if BZR_TRACE_RPL > 1
  constexpr uint32_t kRays = 64u * BZR_TRACE_RPL;  // rays per one-wave block (k_trace_r)
  const dim3 rgrid((job.n + kRays - 1) / kRays), rblock(64);
  auto go = [&](auto kernel) { launch_on(ctx, ctx->stream, rblock, BZR_KERNEL_TRACE, kernel, rgrid, set, j, ctx->counters); };
  (void)grid;
  (void)block;
  if (fast) {
    if (count) go(k_trace_r<kMode, BZR_TRACE_RPL, true, true>);
    else go(k_trace_r<kMode, BZR_TRACE_RPL, true, false>);
  } else {
    if (count) go(k_trace_r<kMode, BZR_TRACE_RPL, false, true>);
    else go(k_trace_r<kMode, BZR_TRACE_RPL, false, false>);
  }
#else
  auto go = [&](auto kernel) { launch_on(ctx, ctx->stream, block, BZR_KERNEL_TRACE, kernel, grid, set, j, ctx->counters); };
  if (fast) {
    if (count) go(k_trace<kMode, true, true>);
    else go(k_trace<kMode, true, false>);
  } else {
    if (count) go(k_trace<kMode, false, true>);
    else go(k_trace<kMode, false, false>);
  }
#endif
  BZR_HIP(hipGetLastError());
  if (rebuild) {  // the next calls' order: tiles longest-first (counting sort of the cost bins)
    uint32_t *order = ctx->sched + ctx->sched_cap, *hist = ctx->sched + (size_t)2 * ctx->sched_cap, *offs = hist + kSchedBins;
    const dim3 sg((tiles + kSchedThreads - 1) / kSchedThreads);
    hipLaunchKernelGGL(k_sched_count, sg, dim3(kSchedThreads), 0, ctx->stream, ctx->sched, tiles, hist);
    hipLaunchKernelGGL(k_sched_scan, dim3(1), dim3(kSchedBins), 0, ctx->stream, hist, offs);
    hipLaunchKernelGGL(k_sched_place, sg, dim3(kSchedThreads), 0, ctx->stream, ctx->sched, tiles, offs, order);
    BZR_HIP(hipGetLastError());
    ctx->sched_waves = tiles;
  }
  return BZR_OK;
}

uint32_t max_patches(const LensSet &set) {
  uint32_t nb = 0;
  for (uint32_t l = 0; l < set.count; ++l) nb = std::max(nb, set.lens[l].n);
  return nb;
}

LensSet single_lens(const MeshView &mv) {
  LensSet set{};
  set.count = 1;
  set.lens[0] = mv;
  return set;
}

template <int kMode>
bzr_status run_segment(bool fast, bzr_ctx *ctx, const MeshView &mv, const float *rays, uint32_t ld, uint32_t off,
                       uint32_t n, const uint32_t *alive, const Out &o, Work &w) {
  return fast ? run_culled<kMode, true>(ctx, mv, rays, ld, off, n, alive, o, w)
              : run_culled<kMode, false>(ctx, mv, rays, ld, off, n, alive, o, w);
}

}  // namespace

// ------------------------------------------------------------------- C ABI
extern "C" bzr_status bzr_device_count(int32_t *count) {
  if (!count) return set_error(BZR_ERR_INVALID_ARGUMENT, "null count");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) c = 0;
  *count = c;
  return BZR_OK;
}

extern "C" bzr_status bzr_ctx_create(int32_t device, bzr_ctx **out) {
  if (!out) return set_error(BZR_ERR_INVALID_ARGUMENT, "null out");
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
    return set_error(BZR_ERR_NO_DEVICE, "no HIP device visible: libbzr has no CPU path");
  if (device < 0 || device >= count) return set_error(BZR_ERR_INVALID_ARGUMENT, "device index out of range");
  DeviceGuard g(device);
  bzr_ctx *c = new (std::nothrow) bzr_ctx();
  if (!c) return set_error(BZR_ERR_OUT_OF_MEMORY, "context allocation");
  c->device = device;
  hipError_t e = hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking);
  if (e != hipSuccess) {
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
    return set_error(BZR_ERR_HIP, std::string("context streams: ") + hipGetErrorString(e));
  }
  c->stream = c->own;
  *out = c;
  return BZR_OK;
}

extern "C" bzr_status bzr_ctx_timing(bzr_ctx *ctx, int32_t enable) {
  if (!ctx) return set_error(BZR_ERR_INVALID_ARGUMENT, "null context");
  ctx->timing = enable != 0;
  return BZR_OK;
}

extern "C" bzr_status bzr_ctx_timing_report(bzr_ctx *ctx, float ms[BZR_KERNEL_COUNT], uint32_t calls[BZR_KERNEL_COUNT]) {
  if (!ctx || !ms || !calls) return set_error(BZR_ERR_INVALID_ARGUMENT, "null argument");
  DeviceGuard g(ctx->device);
  BZR_HIP(hipStreamSynchronize(ctx->stream));
  for (auto const &mk : ctx->marks) {
    float t = 0.0f;
    BZR_HIP(hipEventElapsedTime(&t, mk.start, mk.stop));
    ctx->ms[mk.kernel] += t;
    ctx->calls[mk.kernel] += 1;
    ctx->spare.push_back(mk.start);
    ctx->spare.push_back(mk.stop);
  }
  ctx->marks.clear();
  for (int k = 0; k < BZR_KERNEL_COUNT; ++k) {
    ms[k] = static_cast<float>(ctx->ms[k]);
    calls[k] = ctx->calls[k];
    ctx->ms[k] = 0.0;
    ctx->calls[k] = 0;
  }
  return BZR_OK;
}

extern "C" bzr_status bzr_ctx_counters(bzr_ctx *ctx, int32_t enable) {
  if (!ctx) return set_error(BZR_ERR_INVALID_ARGUMENT, "null context");
  DeviceGuard g(ctx->device);
  if (enable && !ctx->counters) {
    BZR_HIP(hipMalloc(&ctx->counters, kCounterReplicas * BZR_COUNTER_COUNT * sizeof(unsigned long long)));
    BZR_HIP(hipMemsetAsync(ctx->counters, 0, kCounterReplicas * BZR_COUNTER_COUNT * sizeof(unsigned long long),
                           ctx->stream));
  }
  ctx->counting = enable != 0;
  return BZR_OK;
}

extern "C" bzr_status bzr_ctx_counters_report(bzr_ctx *ctx, uint64_t counts[BZR_COUNTER_COUNT]) {
  if (!ctx || !counts) return set_error(BZR_ERR_INVALID_ARGUMENT, "null argument");
  for (int k = 0; k < BZR_COUNTER_COUNT; ++k) counts[k] = 0;
  if (!ctx->counters) return BZR_OK;
  DeviceGuard g(ctx->device);
  std::vector<unsigned long long> host((size_t)kCounterReplicas * BZR_COUNTER_COUNT);
  const size_t bytes = host.size() * sizeof(unsigned long long);
  BZR_HIP(hipMemcpyAsync(host.data(), ctx->counters, bytes, hipMemcpyDeviceToHost, ctx->stream));
  BZR_HIP(hipMemsetAsync(ctx->counters, 0, bytes, ctx->stream));
  BZR_HIP(hipStreamSynchronize(ctx->stream));
  for (uint32_t r = 0; r < kCounterReplicas; ++r)
    for (int k = 0; k < BZR_COUNTER_COUNT; ++k) counts[k] += host[(size_t)r * BZR_COUNTER_COUNT + k];
  return BZR_OK;
}

extern "C" bzr_status bzr_ctx_destroy(bzr_ctx *ctx) {
  if (!ctx) return BZR_OK;
  DeviceGuard g(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  (void)hipStreamSynchronize(ctx->own);
  for (auto const &mk : ctx->marks) {
    (void)hipEventDestroy(mk.start);
    (void)hipEventDestroy(mk.stop);
  }
  for (auto e : ctx->spare) (void)hipEventDestroy(e);
  if (ctx->handoff) (void)hipEventDestroy(ctx->handoff);
  if (ctx->scratch) (void)hipFree(ctx->scratch);
  if (ctx->work) (void)hipFree(ctx->work);
  if (ctx->counters) (void)hipFree(ctx->counters);
  if (ctx->pack) (void)hipFree(ctx->pack);
  if (ctx->sched) (void)hipFree(ctx->sched);
  (void)hipStreamDestroy(ctx->own);
  delete ctx;
  return BZR_OK;
}

namespace {
// Switch the context's stream; work already queued on the old stream (which shares the context's
// workspace) is ordered before anything launched on the new one.
bzr_status switch_stream(bzr_ctx *ctx, hipStream_t next) {
  if (next == ctx->stream) return BZR_OK;
  DeviceGuard g(ctx->device);
  if (!ctx->handoff) BZR_HIP(hipEventCreateWithFlags(&ctx->handoff, hipEventDisableTiming));
  BZR_HIP(hipEventRecord(ctx->handoff, ctx->stream));
  BZR_HIP(hipStreamWaitEvent(next, ctx->handoff, 0));
  ctx->stream = next;
  return BZR_OK;
}
}  // namespace

extern "C" bzr_status bzr_ctx_set_stream(bzr_ctx *ctx, void *stream) {
  if (!ctx) return set_error(BZR_ERR_INVALID_ARGUMENT, "null context");
  return switch_stream(ctx, reinterpret_cast<hipStream_t>(stream));
}

extern "C" bzr_status bzr_ctx_use_own_stream(bzr_ctx *ctx) {
  if (!ctx) return set_error(BZR_ERR_INVALID_ARGUMENT, "null context");
  return switch_stream(ctx, ctx->own);
}

extern "C" bzr_status bzr_ctx_get_stream(bzr_ctx *ctx, void **stream) {
  if (!ctx || !stream) return set_error(BZR_ERR_INVALID_ARGUMENT, "null argument");
  *stream = reinterpret_cast<void *>(ctx->stream);
  return BZR_OK;
}

extern "C" bzr_status bzr_sync(bzr_ctx *ctx) {
  if (!ctx) return set_error(BZR_ERR_INVALID_ARGUMENT, "null context");
  DeviceGuard g(ctx->device);
  BZR_HIP(hipStreamSynchronize(ctx->stream));
  return BZR_OK;
}

extern "C" bzr_status bzr_mesh_create(bzr_ctx *ctx, const void *patches, uint32_t n, uint32_t stride, bzr_mesh **out) {
  if (!ctx || !out || (!patches && n)) return set_error(BZR_ERR_INVALID_ARGUMENT, "null argument");
  if (stride < sizeof(bzr_patch)) return set_error(BZR_ERR_INVALID_ARGUMENT, "stride smaller than bzr_patch");
  *out = nullptr;
  DeviceGuard g(ctx->device);
  std::vector<float> full((size_t)n * rec::kWords);  // index order
  std::vector<float4> planar((size_t)n * 4);
  const char *src = static_cast<const char *>(patches);
  for (uint32_t i = 0; i < n; ++i) {
    float *r = &full[(size_t)i * rec::kWords];
    std::memcpy(r, src + (size_t)i * stride, sizeof(bzr_patch));
    const float *m = r + rec::kMinv;  // col-major: M(i,j) = m[j*3+i]
    planar[4 * i + 0] = make_float4(r[0], r[1], r[2], r[3]);
    planar[4 * i + 1] = make_float4(r[rec::kHin], r[rec::kHout], m[0], m[3]);
    planar[4 * i + 2] = make_float4(m[6], m[1], m[4], m[7]);
    planar[4 * i + 3] = make_float4(m[2], m[5], m[8], 0.0f);
  }
  bzr_host::Bvh bvh, bvh_near;
  try {
    bvh = bzr_host::build_bvh(full.data(), n, rec::kWords, bzr_host::kTierFar);
    bvh_near = bzr_host::build_bvh(full.data(), n, rec::kWords, bzr_host::kTierNear);
  } catch (std::exception const &e) {
    return set_error(BZR_ERR_OUT_OF_MEMORY, std::string("BVH build: ") + e.what());
  }
  auto leaves = [&](bzr_host::Bvh const &t) {  // BVH slot order, patch index in the last word
    std::vector<float4> leaf((size_t)n * 4);
    for (uint32_t k = 0; k < n; ++k) {
      uint32_t b = t.order[k];
      for (int j = 0; j < 4; ++j) leaf[4 * k + j] = planar[4 * b + j];
      std::memcpy(&leaf[4 * k + 3].w, &b, 4);
    }
    return leaf;
  };
  const std::vector<float4> leaf = leaves(bvh), leaf_near = leaves(bvh_near);
  auto kids_of = [](bzr_host::Bvh const &t) {  // node i, child c -> float4 pair 2 (4 i + c): lo.xyz ref, hi.xyz 0
    std::vector<float4> k(t.nodes4.size() * 8);
    for (size_t i = 0; i < t.nodes4.size(); ++i)
      for (int c = 0; c < 4; ++c) {
        auto const &nd = t.nodes4[i];
        float ref;
        std::memcpy(&ref, &nd.child[c], 4);
        k[8 * i + 2 * c] = make_float4(nd.lo[0][c], nd.lo[1][c], nd.lo[2][c], ref);
        k[8 * i + 2 * c + 1] = make_float4(nd.hi[0][c], nd.hi[1][c], nd.hi[2][c], 0.0f);
      }
    return k;
  };
  const std::vector<float4> kids = kids_of(bvh), kids_near = kids_of(bvh_near);
  // two levels per node (k_traverse's bundle walk, BZR_TRAV_WIDE; three with 2): slot 4 c + g of node i is
  // grandchild g of its child c when that child is an axis-aligned inner node, else (a leaf, an oriented-box
  // node) slot 4 c is the child itself and 4 c + 1..3 are empty.  A walk over these slots skips the children's own boxes,
  // so it reaches a superset of the leaves the 4-wide walk reaches (every leaf still takes its exact gate).
  auto wide_of = [](bzr_host::Bvh const &t) {
    constexpr uint32_t S = kWideSlots;
    float empty;
    const uint32_t e = bzr_host::kEmptyChild;
    std::memcpy(&empty, &e, 4);
    std::vector<float4> k(t.nodes4.size() * 2 * S, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    for (size_t s = 0; s < k.size(); s += 2) k[s].w = empty;
    // slots [base, base + span) of node i's record: child c of nd, expanded while span > 1 and it is an
    // axis-aligned inner node, else in the range's first slot
    std::function<void(size_t, uint32_t, uint32_t, const bzr_host::Bvh4Node &, int)> fill =
        [&](size_t i, uint32_t base, uint32_t span, const bzr_host::Bvh4Node &nd, int c) {
          const uint32_t ch = nd.child[c];
          const bool inner = ch != bzr_host::kEmptyChild && !(ch & (bzr_host::kLeafFlag | bzr_host::kObbFlag));
          if (!inner || span == 1u) {
            float ref;
            std::memcpy(&ref, &nd.child[c], 4);
            k[2 * (S * i + base)] = make_float4(nd.lo[0][c], nd.lo[1][c], nd.lo[2][c], ref);
            k[2 * (S * i + base) + 1] = make_float4(nd.hi[0][c], nd.hi[1][c], nd.hi[2][c], 0.0f);
            return;
          }
          for (int g = 0; g < 4; ++g) fill(i, base + g * (span / 4u), span / 4u, t.nodes4[ch], g);
        };
    for (size_t i = 0; i < t.nodes4.size(); ++i)
      for (int c = 0; c < 4; ++c) fill(i, c * (S / 4u), S / 4u, t.nodes4[i], c);
    return k;
  };
  const std::vector<float4> wide = BZR_TRAV_WIDE ? wide_of(bvh) : std::vector<float4>(),
                            wide_near = BZR_TRAV_WIDE ? wide_of(bvh_near) : std::vector<float4>();
  // the always list: the same patches in both tiers (whether a gate region is proven does not depend on
  // the tier's origin radius)
  if (bvh.always != bvh_near.always) return set_error(BZR_ERR_INVALID_ARGUMENT, "BVH tiers disagree on the always list");
  std::vector<float4> always(bvh.always.size() * kAlwaysQuads);
  for (size_t k = 0; k < bvh.always.size(); ++k) {
    const uint32_t b = bvh.always[k];
    for (int j = 0; j < 4; ++j) always[kAlwaysQuads * k + j] = planar[4 * b + j];
    std::memcpy(&always[kAlwaysQuads * k + 3].w, &b, 4);
    std::memcpy(&always[kAlwaysQuads * k + 4], &bvh.always_wedge[8 * k], 8 * sizeof(float));
  }
  bzr_mesh *mesh = new (std::nothrow) bzr_mesh();
  if (!mesh) return set_error(BZR_ERR_OUT_OF_MEMORY, "mesh allocation");
  mesh->device = ctx->device;
  mesh->n = n;
  mesh->nnodes = static_cast<uint32_t>(bvh.nodes4.size());
  mesh->n_always = static_cast<uint32_t>(bvh.always.size());
  mesh->s_max = bvh.s_max;
  mesh->s_near = std::min(bvh_near.s_max, bvh.s_max);
  for (int k = 0; k < 4; ++k) mesh->sphere[k] = bvh.sphere[k];
  struct Up {
    void **dst;
    const void *src;
    size_t bytes;
  } ups[] = {
      {reinterpret_cast<void **>(&mesh->planar), planar.data(), planar.size() * sizeof(float4)},
      {reinterpret_cast<void **>(&mesh->full), full.data(), full.size() * sizeof(float)},
      {reinterpret_cast<void **>(&mesh->nodes), bvh.nodes4.data(), bvh.nodes4.size() * sizeof(bzr_host::Bvh4Node)},
      {reinterpret_cast<void **>(&mesh->leaf), leaf.data(), leaf.size() * sizeof(float4)},
      {reinterpret_cast<void **>(&mesh->nodes_near), bvh_near.nodes4.data(),
       bvh_near.nodes4.size() * sizeof(bzr_host::Bvh4Node)},
      {reinterpret_cast<void **>(&mesh->leaf_near), leaf_near.data(), leaf_near.size() * sizeof(float4)},
      {reinterpret_cast<void **>(&mesh->obb), bvh.obb.data(), bvh.obb.size() * sizeof(bzr_host::Bvh4ObbNode)},
      {reinterpret_cast<void **>(&mesh->obb_near), bvh_near.obb.data(),
       bvh_near.obb.size() * sizeof(bzr_host::Bvh4ObbNode)},
      {reinterpret_cast<void **>(&mesh->always), always.data(), always.size() * sizeof(float4)},
      {reinterpret_cast<void **>(&mesh->kids), kids.data(), kids.size() * sizeof(float4)},
      {reinterpret_cast<void **>(&mesh->kids_near), kids_near.data(), kids_near.size() * sizeof(float4)},
      {reinterpret_cast<void **>(&mesh->wide), wide.data(), wide.size() * sizeof(float4)},
      {reinterpret_cast<void **>(&mesh->wide_near), wide_near.data(), wide_near.size() * sizeof(float4)},
  };
  hipError_t e = hipSuccess;
  for (auto &u : ups) {
    if (e == hipSuccess) e = hipMalloc(u.dst, u.bytes ? u.bytes : 16);
    if (e == hipSuccess && u.bytes) e = hipMemcpyAsync(*u.dst, u.src, u.bytes, hipMemcpyHostToDevice, ctx->stream);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) {
    for (auto &u : ups) (void)hipFree(*u.dst);
    delete mesh;
    return set_error(BZR_ERR_HIP, std::string("mesh upload: ") + hipGetErrorString(e));
  }
  *out = mesh;
  return BZR_OK;
}

extern "C" bzr_status bzr_mesh_destroy(bzr_mesh *mesh) {
  if (!mesh) return BZR_OK;
  DeviceGuard g(mesh->device);
  (void)hipDeviceSynchronize();
  (void)hipFree(mesh->planar);
  (void)hipFree(mesh->full);
  (void)hipFree(mesh->nodes);
  (void)hipFree(mesh->leaf);
  (void)hipFree(mesh->nodes_near);
  (void)hipFree(mesh->leaf_near);
  (void)hipFree(mesh->obb);
  (void)hipFree(mesh->obb_near);
  (void)hipFree(mesh->always);
  (void)hipFree(mesh->kids);
  (void)hipFree(mesh->kids_near);
  (void)hipFree(mesh->wide);
  (void)hipFree(mesh->wide_near);
  delete mesh;
  return BZR_OK;
}

extern "C" bzr_status bzr_mesh_size(const bzr_mesh *mesh, uint32_t *n) {
  if (!mesh || !n) return set_error(BZR_ERR_INVALID_ARGUMENT, "null argument");
  *n = mesh->n;
  return BZR_OK;
}

// BezierMesh::intersect of n rays given as device rows into device hit rows [13][n]: the body of bzr_intersect
// and bzr_intersect_records, on the context's stream.
static bzr_status intersect_rows(bzr_ctx *ctx, const bzr_mesh *mesh, const float *d_rays, uint32_t n, float *d_hits,
                                 uint32_t flags) {
  MeshView mv = view_of(mesh);
  if (use_scan(flags)) {
    launch(ctx, BZR_KERNEL_INTERSECT_SCAN, k_intersect_scan, dim3(grid_for(n)), mv, d_rays, n, d_hits);
  } else if (!use_staged(flags, n, mesh->n)) {
    TraceJob job{};
    job.rays = d_rays;
    job.hits = d_hits;
    job.n = job.ld = n;
    if (bzr_status s = run_fused<kModeHits>(ctx, single_lens(mv), job, flags)) return s;
  } else {
    Work w;
    const uint32_t ch = chunk_for(ctx, n);
    if (bzr_status s = ensure_work(ctx, ch, mesh->n, w)) return s;
    Out o{};
    o.hits = d_hits;
    for (uint32_t off = 0; off < n; off += ch)
      if (bzr_status s = run_segment<kModeHits>(use_fast(flags), ctx, mv, d_rays, n, off, std::min(ch, n - off), nullptr, o, w))
        return s;
  }
  BZR_HIP(hipGetLastError());
  return BZR_OK;
}

extern "C" bzr_status bzr_intersect(bzr_ctx *ctx, const bzr_mesh *mesh, const float *rays, uint32_t n, float *hits,
                                    uint32_t flags) {
  if (bzr_status s = check_flags(flags, true)) return s;
  if (bzr_status s = check_ctx_mesh(ctx, mesh)) return s;
  if (n == 0) return BZR_OK;
  if (!rays || !hits) return set_error(BZR_ERR_INVALID_ARGUMENT, "null buffer");
  DeviceGuard g(ctx->device);
  const float *d_rays = rays;
  float *d_hits = hits;
  const bool host = !(flags & BZR_DEVICE_PTRS), aos = (flags & BZR_RAYS_AOS) != 0;
  if (host || aos) {
    size_t rb = (size_t)n * 6 * sizeof(float), hb = (size_t)n * 13 * sizeof(float);
    if (bzr_status s = ensure_buffer(ctx->scratch, ctx->scratch_bytes,
                                     round256(rb) + (host ? round256(hb) : 0) + (host && aos ? round256(rb) : 0)))
      return s;
    Staging st{static_cast<char *>(ctx->scratch)};
    float *r = st.take<float>((size_t)n * 6);
    if (host) d_hits = st.take<float>((size_t)n * 13);
    float *tmp = host && aos ? st.take<float>((size_t)n * 6) : nullptr;
    if (bzr_status s = rays_in(ctx, rays, r, n, host, aos, tmp)) return s;
    d_rays = r;
  }
  if (bzr_status s = intersect_rows(ctx, mesh, d_rays, n, d_hits, flags)) return s;
  if (host) {
    BZR_HIP(hipMemcpyAsync(hits, d_hits, (size_t)n * 13 * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    BZR_HIP(hipStreamSynchronize(ctx->stream));
  }
  return BZR_OK;
}

extern "C" bzr_status bzr_intersect_records(bzr_ctx *ctx, const bzr_mesh *mesh, const float *rays, uint32_t n,
                                            bzr_hit_record *records, uint32_t *patch_index, uint32_t flags) {
  if (bzr_status s = check_flags(flags, true)) return s;
  if (bzr_status s = check_ctx_mesh(ctx, mesh)) return s;
  if (n == 0) return BZR_OK;
  if (!rays || !records) return set_error(BZR_ERR_INVALID_ARGUMENT, "null buffer");
  DeviceGuard g(ctx->device);
  const bool host = !(flags & BZR_DEVICE_PTRS), aos = (flags & BZR_RAYS_AOS) != 0;
  // staging: the rays' rows (unless the caller's device rows are used as they are), the hit rows, and for host
  // callers the records and patch words before their copies
  const size_t rb = (size_t)n * 24, hb = (size_t)n * 52, pb = (size_t)n * 4;
  const bool stage_rays = host || aos;
  if (bzr_status s = ensure_buffer(ctx->scratch, ctx->scratch_bytes,
                                   (stage_rays ? round256(rb) : 0) + (host && aos ? round256(rb) : 0) + round256(hb) +
                                       (host ? round256(hb) + round256(pb) : 0)))
    return s;
  Staging st{static_cast<char *>(ctx->scratch)};
  const float *d_rays = rays;
  if (stage_rays) {
    float *r = st.take<float>((size_t)n * 6);
    float *tmp = host && aos ? st.take<float>((size_t)n * 6) : nullptr;
    if (bzr_status s = rays_in(ctx, rays, r, n, host, aos, tmp)) return s;
    d_rays = r;
  }
  float *d_hits = st.take<float>((size_t)n * 13);
  void *d_rec = records;
  uint32_t *d_patch = patch_index;
  if (host) {
    d_rec = st.take<uint32_t>((size_t)n * 13);
    d_patch = patch_index ? st.take<uint32_t>(n) : nullptr;
  }
  if (bzr_status s = intersect_rows(ctx, mesh, d_rays, n, d_hits, flags)) return s;
  BZR_HIP(bzr_hits_to_records(ctx->stream, d_hits, n, d_rec, d_patch));
  if (host) {
    BZR_HIP(hipMemcpyAsync(records, d_rec, hb, hipMemcpyDeviceToHost, ctx->stream));
    if (patch_index) BZR_HIP(hipMemcpyAsync(patch_index, d_patch, pb, hipMemcpyDeviceToHost, ctx->stream));
    BZR_HIP(hipStreamSynchronize(ctx->stream));
  }
  return BZR_OK;
}

extern "C" bzr_status bzr_patch_intersect(bzr_ctx *ctx, const bzr_mesh *mesh, const uint32_t *idx, const uint32_t *limit,
                                          const float *rays, uint32_t n, float *hits, uint32_t flags) {
  if (bzr_status s = check_flags(flags)) return s;
  if (bzr_status s = check_ctx_mesh(ctx, mesh)) return s;
  if (n == 0) return BZR_OK;
  if (!idx || !limit || !rays || !hits) return set_error(BZR_ERR_INVALID_ARGUMENT, "null buffer");
  DeviceGuard g(ctx->device);
  const uint32_t *d_idx = idx, *d_lim = limit;
  const float *d_rays = rays;
  float *d_hits = hits;
  bool host = !(flags & BZR_DEVICE_PTRS);
  if (host) {
    size_t ib = (size_t)n * 4, rb = (size_t)n * 24, hb = (size_t)n * 52;
    if (bzr_status s = ensure_buffer(ctx->scratch, ctx->scratch_bytes, 2 * round256(ib) + round256(rb) + round256(hb)))
      return s;
    Staging st{static_cast<char *>(ctx->scratch)};
    uint32_t *a = st.take<uint32_t>(n), *b = st.take<uint32_t>(n);
    float *r = st.take<float>((size_t)n * 6);
    d_hits = st.take<float>((size_t)n * 13);
    BZR_HIP(hipMemcpyAsync(a, idx, ib, hipMemcpyHostToDevice, ctx->stream));
    BZR_HIP(hipMemcpyAsync(b, limit, ib, hipMemcpyHostToDevice, ctx->stream));
    BZR_HIP(hipMemcpyAsync(r, rays, rb, hipMemcpyHostToDevice, ctx->stream));
    d_idx = a;
    d_lim = b;
    d_rays = r;
  }
  auto *kp = use_fast(flags) ? &k_patch<true> : &k_patch<false>;
  launch(ctx, BZR_KERNEL_PATCH, kp, dim3(grid_for(n)), view_of(mesh), d_idx, d_lim, d_rays, n,
                     d_hits);
  BZR_HIP(hipGetLastError());
  if (host) {
    BZR_HIP(hipMemcpyAsync(hits, d_hits, (size_t)n * 52, hipMemcpyDeviceToHost, ctx->stream));
    BZR_HIP(hipStreamSynchronize(ctx->stream));
  }
  return BZR_OK;
}

extern "C" bzr_status bzr_refract(bzr_ctx *ctx, const bzr_mesh *mesh, float ri, const float *rays, const uint32_t *expected,
                                  uint32_t expected_all, uint32_t n, float *out_rays, uint32_t *out_status,
                                  uint32_t flags) {
  if (bzr_status s = check_flags(flags, true)) return s;
  if (bzr_status s = check_ctx_mesh(ctx, mesh)) return s;
  if (n == 0) return BZR_OK;
  if (!rays || !out_rays || !out_status) return set_error(BZR_ERR_INVALID_ARGUMENT, "null buffer");
  DeviceGuard g(ctx->device);
  const float *d_rays = rays;
  const uint32_t *d_exp = expected;
  float *d_out = out_rays;
  uint32_t *d_st = out_status;
  const bool host = !(flags & BZR_DEVICE_PTRS), aos = (flags & BZR_RAYS_AOS) != 0;
  float *tmp = nullptr;  // host + AoS: the records on the device, in and out
  if (host || aos) {
    size_t rb = (size_t)n * 24, ib = (size_t)n * 4;
    if (bzr_status s = ensure_buffer(ctx->scratch, ctx->scratch_bytes,
                                     2 * round256(rb) + (host ? 2 * round256(ib) : 0) + (host && aos ? round256(rb) : 0)))
      return s;
    Staging st{static_cast<char *>(ctx->scratch)};
    float *r = st.take<float>((size_t)n * 6);
    d_out = st.take<float>((size_t)n * 6);
    if (host) {
      uint32_t *e = st.take<uint32_t>(n);
      d_st = st.take<uint32_t>(n);
      if (expected) BZR_HIP(hipMemcpyAsync(e, expected, ib, hipMemcpyHostToDevice, ctx->stream));
      d_exp = expected ? e : nullptr;
    }
    if (host && aos) tmp = st.take<float>((size_t)n * 6);
    if (bzr_status s = rays_in(ctx, rays, r, n, host, aos, tmp)) return s;
    d_rays = r;
  }
  MeshView mv = view_of(mesh, ri);
  if (use_scan(flags)) {
    launch(ctx, BZR_KERNEL_REFRACT_SCAN, k_refract_scan, dim3(grid_for(n)), mv, d_rays, d_exp, expected_all,
                       n, d_out, d_st);
  } else if (!use_staged(flags, n, mesh->n)) {
    TraceJob job{};
    job.rays = d_rays;
    job.out_rays = d_out;
    job.status = d_st;
    job.expected = d_exp;
    job.expected_all = expected_all;
    job.n = job.ld = n;
    if (bzr_status s = run_fused<kModeRefract>(ctx, single_lens(mv), job, flags)) return s;
  } else {
    Work w;
    const uint32_t ch = chunk_for(ctx, n);
    if (bzr_status s = ensure_work(ctx, ch, mesh->n, w)) return s;
    Out o{};
    o.rays = d_out;
    o.expected = d_exp;
    o.expected_all = expected_all;
    o.status = d_st;
    o.ri = ri;
    for (uint32_t off = 0; off < n; off += ch)
      if (bzr_status s = run_segment<kModeRefract>(use_fast(flags), ctx, mv, d_rays, n, off, std::min(ch, n - off), nullptr, o, w))
        return s;
  }
  BZR_HIP(hipGetLastError());
  if (bzr_status s = rays_out(ctx, d_out, out_rays, n, host, aos, tmp)) return s;
  if (host) {
    BZR_HIP(hipMemcpyAsync(out_status, d_st, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream));
    BZR_HIP(hipStreamSynchronize(ctx->stream));
  }
  return BZR_OK;
}

extern "C" bzr_status bzr_trace_chain(bzr_ctx *ctx, const bzr_mesh *const *lenses, const float *ri, uint32_t nlens,
                                      const float *rays, uint32_t n, float *out_rays, uint32_t *out_status,
                                      uint32_t *out_segments, uint32_t flags) {
  if (bzr_status s = check_flags(flags, true)) return s;
  if (!ctx) return set_error(BZR_ERR_INVALID_ARGUMENT, "null context");
  if (nlens == 0 || nlens > kMaxLenses) return set_error(BZR_ERR_INVALID_ARGUMENT, "nlens must be 1..8");
  if (!lenses || !ri) return set_error(BZR_ERR_INVALID_ARGUMENT, "null lens list");
  LensSet set{};
  set.count = nlens;
  for (uint32_t l = 0; l < nlens; ++l) {
    if (bzr_status s = check_ctx_mesh(ctx, lenses[l])) return s;
    set.lens[l] = view_of(lenses[l], ri[l]);
  }
  if (n == 0) return BZR_OK;
  if (!rays || !out_rays || !out_status) return set_error(BZR_ERR_INVALID_ARGUMENT, "null buffer");
  if (rays == out_rays) return set_error(BZR_ERR_INVALID_ARGUMENT, "rays and out_rays must not alias");
  DeviceGuard g(ctx->device);
  const float *d_rays = rays;
  float *d_out = out_rays;
  uint32_t *d_st = out_status, *d_seg = out_segments;
  const bool host = !(flags & BZR_DEVICE_PTRS), aos = (flags & BZR_RAYS_AOS) != 0;
  float *tmp = nullptr;  // host + AoS: the records on the device, in and out
  if (host || aos) {
    size_t rb = (size_t)n * 24, ib = (size_t)n * 4;
    if (bzr_status s = ensure_buffer(ctx->scratch, ctx->scratch_bytes,
                                     2 * round256(rb) + (host ? 2 * round256(ib) : 0) + (host && aos ? round256(rb) : 0)))
      return s;
    Staging st{static_cast<char *>(ctx->scratch)};
    float *r = st.take<float>((size_t)n * 6);
    d_out = st.take<float>((size_t)n * 6);
    if (host) {
      d_st = st.take<uint32_t>(n);
      d_seg = st.take<uint32_t>(n);
    }
    if (host && aos) tmp = st.take<float>((size_t)n * 6);
    if (bzr_status s = rays_in(ctx, rays, r, n, host, aos, tmp)) return s;
    d_rays = r;
  }
  if (use_scan(flags)) {
    launch(ctx, BZR_KERNEL_CHAIN_SCAN, k_chain_scan, dim3(grid_for(n)), set, d_rays, n, d_out, d_st, d_seg);
    BZR_HIP(hipGetLastError());
  } else if (!use_staged(flags, n, max_patches(set))) {
    TraceJob job{};
    job.rays = d_rays;
    job.out_rays = d_out;
    job.status = d_st;
    job.segments = d_seg;
    job.n = job.ld = n;
    if (bzr_status s = run_fused<kModeStage>(ctx, set, job, flags)) return s;
  } else {
    // stage by stage: out_rays holds the rays in flight, out_status != NONE marks them alive
    uint32_t nb = 0;
    for (uint32_t l = 0; l < nlens; ++l) nb = std::max(nb, set.lens[l].n);
    Work w;
    const uint32_t ch = chunk_for(ctx, n);
    if (bzr_status s = ensure_work(ctx, ch, nb, w)) return s;
    // the first stage reads the caller's rays and writes every ray's ray / status / segments (no
    // copy or fill launches); later stages update the rays in flight in place, alive = status != NONE
    for (uint32_t off = 0; off < n; off += ch) {
      const uint32_t m = std::min(ch, n - off);
      for (uint32_t l = 0; l < nlens; ++l) {
        for (uint32_t j = 0; j < 2; ++j) {
          Out o{};
          o.rays = d_out;
          o.expected_all = j == 0 ? uint32_t(BZR_RR_INSIDE) : uint32_t(BZR_RR_OUTSIDE);
          o.status = d_st;
          o.segments = d_seg;
          o.ri = set.lens[l].ri;
          o.first = (l == 0 && j == 0) ? 1u : 0u;
          if (bzr_status s = run_segment<kModeStage>(use_fast(flags), ctx, set.lens[l], o.first ? d_rays : d_out, n, off,
                                                     m, o.first ? nullptr : d_st, o, w))
            return s;
        }
      }
    }
    BZR_HIP(hipGetLastError());
  }
  if (bzr_status s = rays_out(ctx, d_out, out_rays, n, host, aos, tmp)) return s;
  if (host) {
    BZR_HIP(hipMemcpyAsync(out_status, d_st, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream));
    if (out_segments)
      BZR_HIP(hipMemcpyAsync(out_segments, d_seg, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream));
    BZR_HIP(hipStreamSynchronize(ctx->stream));
  }
  return BZR_OK;
}

// ------------------------------------------------------------ test hook: normalized()
namespace {
// Row k of out (k < 3): the product's exact normalized() (patch_math.hpp unit_or_self, shared-reciprocal chain
// where its guard allows); rows 3..5: sqrt_rn / div_rn per component (the compiler's own lowering).
__global__ __launch_bounds__(kBlock) void k_debug_unit(const float *__restrict__ a, uint32_t n,
                                                       float *__restrict__ out) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const f3 v = mk(a[i], a[(size_t)n + i], a[(size_t)2 * n + i]);
  const f3 u = normalized(v);
  const float z = dot(v, v);
  f3 w = v;
  if (z > 0.0f) {
    const float s = sqrt_rn(z);
    w = mk(div_rn(v.x, s), div_rn(v.y, s), div_rn(v.z, s));
  }
  const float r[6] = {u.x, u.y, u.z, w.x, w.y, w.z};
#pragma unroll
  for (int k = 0; k < 6; ++k) out[(size_t)k * n + i] = r[k];
}
// newton_tail's bracket quotients (div_heights) beside one correctly rounded division each.
__global__ __launch_bounds__(kBlock) void k_debug_div_heights(const float *__restrict__ a, uint32_t n,
                                                              float *__restrict__ out) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const float hin = a[i], hout = a[(size_t)n + i], ic = a[(size_t)2 * n + i];
  float din, dout;
  div_heights(hin, hout, ic, din, dout);
  out[i] = din;
  out[(size_t)n + i] = dout;
  out[(size_t)2 * n + i] = div_rn(hin, ic);
  out[(size_t)3 * n + i] = div_rn(hout, ic);
}
}  // namespace

extern "C" bzr_status bzr_debug_div_heights(void *ctxp, const float *a, uint32_t n, float *out) {
  bzr_ctx *ctx = static_cast<bzr_ctx *>(ctxp);
  if (!ctx) return set_error(BZR_ERR_INVALID_ARGUMENT, "null context");
  if (n == 0) return BZR_OK;
  if (!a || !out) return set_error(BZR_ERR_INVALID_ARGUMENT, "null buffer");
  DeviceGuard g(ctx->device);
  hipLaunchKernelGGL(k_debug_div_heights, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, ctx->stream, a, n, out);
  BZR_HIP(hipGetLastError());
  return BZR_OK;
}

extern "C" bzr_status bzr_debug_wave_clock(void *ctxp, unsigned long long *clock, uint32_t waves) {
  bzr_ctx *ctx = static_cast<bzr_ctx *>(ctxp);
  if (!ctx) return set_error(BZR_ERR_INVALID_ARGUMENT, "null context");
  ctx->wave_clock = clock;
  ctx->wave_clock_cap = clock ? waves : 0u;
  ctx->wave_clock_real = false;
  return BZR_OK;
}

extern "C" bzr_status bzr_debug_wave_clock_rate(void *ctxp, unsigned long long *clock, uint32_t waves) {
  bzr_ctx *ctx = static_cast<bzr_ctx *>(ctxp);
  if (!ctx) return set_error(BZR_ERR_INVALID_ARGUMENT, "null context");
  ctx->wave_clock = clock;
  ctx->wave_clock_cap = clock ? waves : 0u;
  ctx->wave_clock_real = clock != nullptr;
  return BZR_OK;
}

extern "C" bzr_status bzr_debug_unit(void *ctxp, const float *a, uint32_t n, float *out) {
  bzr_ctx *ctx = static_cast<bzr_ctx *>(ctxp);
  if (!ctx) return set_error(BZR_ERR_INVALID_ARGUMENT, "null context");
  if (n == 0) return BZR_OK;
  if (!a || !out) return set_error(BZR_ERR_INVALID_ARGUMENT, "null buffer");
  DeviceGuard g(ctx->device);
  hipLaunchKernelGGL(k_debug_unit, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, ctx->stream, a, n, out);
  BZR_HIP(hipGetLastError());
  return BZR_OK;
}

// ------------------------------------------------------------ tessellation
extern "C" uint32_t bzr_internal_unit_subtriangles(int32_t divisor, float *out);  // host (patch_build.cpp)

namespace {
// BezierMesh::interpolate (reference/bezierMesh.cpp:55-66): output triangle t = k * nb + b is
// sub-triangle k of patch b; its three vertices are BezierTriangle::interpolate at the sub-triangle's
// barycentric corners (reference/bezierTriangle.cpp:105-121, patch_math.hpp `interpolate`).
__global__ __launch_bounds__(kBlock) void k_tessellate(const float *__restrict__ full, uint32_t nb,
                                                       const float *__restrict__ bary, uint64_t total,
                                                       float *__restrict__ out) {
  const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (t >= total) return;
  const uint32_t k = static_cast<uint32_t>(t / nb), b = static_cast<uint32_t>(t % nb);
  const PatchView<const float *> p{full + (size_t)rec::kWords * b};
  const float *bk = bary + (size_t)9 * k;
#pragma unroll
  for (int v = 0; v < 3; ++v) {
    const f3 q = interpolate(p, mk(bk[3 * v], bk[3 * v + 1], bk[3 * v + 2]));
    out[(size_t)9 * t + 3 * v] = q.x;
    out[(size_t)9 * t + 3 * v + 1] = q.y;
    out[(size_t)9 * t + 3 * v + 2] = q.z;
  }
}
}  // namespace

extern "C" bzr_status bzr_mesh_interpolate(bzr_ctx *ctx, const bzr_mesh *mesh, int32_t divisor, float *out_xyz,
                                           uint32_t flags) {
  if (bzr_status s = check_flags(flags)) return s;
  if (bzr_status s = check_ctx_mesh(ctx, mesh)) return s;
  if (divisor < 1 || divisor > 4096) return set_error(BZR_ERR_INVALID_ARGUMENT, "divisor must be 1..4096");
  const uint32_t K = static_cast<uint32_t>(divisor) * static_cast<uint32_t>(divisor);
  const uint64_t total = (uint64_t)K * mesh->n;
  if (total == 0) return BZR_OK;
  if (!out_xyz) return set_error(BZR_ERR_INVALID_ARGUMENT, "null buffer");
  DeviceGuard g(ctx->device);
  std::vector<float> bary((size_t)K * 9);
  if (bzr_internal_unit_subtriangles(divisor, bary.data()) != K)
    return set_error(BZR_ERR_INVALID_ARGUMENT, "sub-triangle count mismatch");
  const bool host = !(flags & BZR_DEVICE_PTRS);
  const size_t bb = round256(bary.size() * 4), ob = (size_t)total * 9 * 4;
  if (bzr_status s = ensure_buffer(ctx->scratch, ctx->scratch_bytes, bb + (host ? round256(ob) : 0))) return s;
  Staging st{static_cast<char *>(ctx->scratch)};
  float *d_bary = st.take<float>(bary.size());
  float *d_out = host ? st.take<float>((size_t)total * 9) : out_xyz;
  BZR_HIP(hipMemcpyAsync(d_bary, bary.data(), bary.size() * 4, hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(k_tessellate, dim3(static_cast<uint32_t>((total + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     ctx->stream, mesh->full, mesh->n, d_bary, total, d_out);
  BZR_HIP(hipGetLastError());
  if (host) BZR_HIP(hipMemcpyAsync(out_xyz, d_out, ob, hipMemcpyDeviceToHost, ctx->stream));
  // the staged sub-triangle table must outlive the kernel: this call is synchronous
  BZR_HIP(hipStreamSynchronize(ctx->stream));
  return BZR_OK;
}

// ------------------------------------------------------------ illumination
namespace {
// Rays first .. first+n-1 of the emitter into rays [6][ld].  With `status`: rays that cannot meet the
// first lens's bounding sphere (over its proven gate regions) and pass none of its always-listed patches'
// planar gates start as NONE (culled, never traced), the others INSIDE (the chain's first refraction
// expects to enter the lens); stats[EMITTED], stats[CULLED] count them.
__global__ __launch_bounds__(kBlock) void k_emit(bzr_emitter em, BeltTable bt, uint64_t first, uint32_t n, uint32_t ld,
                                                 float *__restrict__ rays, uint32_t *__restrict__ patch,
                                                 uint32_t *__restrict__ status, uint32_t *__restrict__ segments,
                                                 float4 sphere, const float4 *__restrict__ always, uint32_t n_always,
                                                 unsigned long long *__restrict__ stats) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  bool culled = false;
  f3 o = mk(0.0f, 0.0f, 0.0f), d = o;
  if (i < n) {
    uint32_t p;
    emit_ray(em, bt, first + i, o, d, p);
    store_ray(rays, ld, i, o, d);
    if (patch) patch[i] = p;
    if (status) {
      const float sp[4] = {sphere.x, sphere.y, sphere.z, sphere.w};
      culled = !may_hit_sphere(o, d, sp);
    }
  }
  if (status) {
    // the always list has no box inside the sphere: a ray outside it is kept if any of those gates passes
    for (uint32_t k = 0; k < n_always && __any(culled); ++k) {
      uint32_t b;
      if (always_gate(always, k, culled, o, d, b)) culled = false;
    }
    if (i < n) {
      status[i] = culled ? BZR_RR_NONE : BZR_RR_INSIDE;
      if (segments) segments[i] = 0u;
    }
  }
  if (stats) {
    const unsigned long long made = __ballot(i < n), cut = __ballot(culled);
    if ((threadIdx.x & 63u) == 0u) {
      if (made) atomicAdd(&stats[BZR_ILLUM_EMITTED], (unsigned long long)__popcll(made));
      if (cut) atomicAdd(&stats[BZR_ILLUM_CULLED], (unsigned long long)__popcll(cut));
    }
  }
}

// Rays that left the last lens (status OUTSIDE) meet the target plane: one count per landed ray.
__global__ __launch_bounds__(kBlock) void k_land(bzr_target tg, float4 plane, float cell_u, float cell_v,
                                                 const float *__restrict__ rays, uint32_t ld, uint32_t n,
                                                 const uint32_t *__restrict__ status, uint32_t *__restrict__ hist,
                                                 unsigned long long *__restrict__ stats) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  bool exited = false, landed = false;
  if (i < n && status[i] == BZR_RR_OUTSIDE) {
    exited = true;
    f3 s, d;
    load_ray(rays, ld, i, s, d);
    const int32_t cell = target_cell(tg, mk(plane.x, plane.y, plane.z), plane.w, cell_u, cell_v, s, d);
    if (cell >= 0) {
      landed = true;
      atomicAdd(&hist[cell], 1u);
    }
  }
  const unsigned long long ex = __ballot(exited), la = __ballot(landed);
  if ((threadIdx.x & 63u) == 0u) {
    if (ex) atomicAdd(&stats[BZR_ILLUM_EXITED], (unsigned long long)__popcll(ex));
    if (la) atomicAdd(&stats[BZR_ILLUM_LANDED], (unsigned long long)__popcll(la));
  }
}

// UniformHemisphere(belts)'s patch table (reference/hostUtil.cpp:3-14, same float expressions) and the
// belt boundaries cos(i * width) the device compares cos(incidence) against.
bzr_status belt_tables(uint32_t belts, std::vector<float> &cos_lo, std::vector<uint32_t> &count,
                       std::vector<uint32_t> &first) {
  if (belts == 0 || belts > 4096) return set_error(BZR_ERR_INVALID_ARGUMENT, "belts must be 1..4096");
  constexpr float kPi = 3.14159265358979323846f;  // cgPi, reference/3dGeomUtil.h:19
  const float width = kPi / 2.0f / (float)belts;
  cos_lo.assign(belts, 1.0f);
  count.resize(belts);
  first.resize(belts);
  uint32_t so_far = 0;
  for (uint32_t i = 0; i < belts; ++i) {
    count[i] = (uint32_t)std::ceil(static_cast<double>(4.0f * (float)belts) *
                                   std::sin(static_cast<double>((2.0f * (float)i + 1.0f) / (4.0f * (float)belts) * kPi)));
    first[i] = so_far;
    so_far += count[i];
    if (i) cos_lo[i] = std::cos((float)i * width);
  }
  return BZR_OK;
}

bzr_status check_emitter(const bzr_emitter *em) {
  if (!em) return set_error(BZR_ERR_INVALID_ARGUMENT, "null emitter");
  if (!em->parts_u || !em->parts_v || !em->points_per_part || !em->rays_per_point)
    return set_error(BZR_ERR_INVALID_ARGUMENT, "emitter counts must be positive");
  return BZR_OK;
}

// The belt tables in device memory (carved from `st`), as the kernels' BeltTable.
bzr_status upload_belts(bzr_ctx *ctx, const bzr_emitter *em, Staging &st, BeltTable &bt, std::vector<float> &cos_lo,
                        std::vector<uint32_t> &count, std::vector<uint32_t> &first) {
  if (bzr_status s = belt_tables(em->belts, cos_lo, count, first)) return s;
  float *c = st.take<float>(em->belts);
  uint32_t *k = st.take<uint32_t>(em->belts), *f = st.take<uint32_t>(em->belts);
  BZR_HIP(hipMemcpyAsync(c, cos_lo.data(), em->belts * 4, hipMemcpyHostToDevice, ctx->stream));
  BZR_HIP(hipMemcpyAsync(k, count.data(), em->belts * 4, hipMemcpyHostToDevice, ctx->stream));
  BZR_HIP(hipMemcpyAsync(f, first.data(), em->belts * 4, hipMemcpyHostToDevice, ctx->stream));
  bt = BeltTable{c, k, f, em->belts};
  return BZR_OK;
}
size_t belt_bytes(uint32_t belts) { return 3 * round256((size_t)belts * 4); }
}  // namespace

extern "C" bzr_status bzr_mesh_bounding_sphere(const bzr_mesh *mesh, float out[4]) {
  if (!mesh || !out) return set_error(BZR_ERR_INVALID_ARGUMENT, "null argument");
  for (int k = 0; k < 4; ++k) out[k] = mesh->sphere[k];
  return BZR_OK;
}

extern "C" bzr_status bzr_emit(bzr_ctx *ctx, const bzr_emitter *em, uint64_t first, uint32_t n, float *rays_soa,
                               uint32_t *patch_index, uint32_t flags) {
  if (!ctx) return set_error(BZR_ERR_INVALID_ARGUMENT, "null context");
  if (bzr_status s = check_emitter(em)) return s;
  if (n == 0) return BZR_OK;
  if (!rays_soa) return set_error(BZR_ERR_INVALID_ARGUMENT, "null buffer");
  DeviceGuard g(ctx->device);
  const bool host = !(flags & BZR_DEVICE_PTRS);
  const size_t rb = (size_t)n * 24, pb = (size_t)n * 4;
  if (bzr_status s = ensure_buffer(ctx->scratch, ctx->scratch_bytes,
                                   belt_bytes(em->belts) + (host ? round256(rb) + round256(pb) : 0)))
    return s;
  Staging st{static_cast<char *>(ctx->scratch)};
  BeltTable bt;
  std::vector<float> cos_lo;
  std::vector<uint32_t> count, firsts;
  if (bzr_status s = upload_belts(ctx, em, st, bt, cos_lo, count, firsts)) return s;
  float *d_rays = host ? st.take<float>((size_t)n * 6) : rays_soa;
  uint32_t *d_patch = host ? (patch_index ? st.take<uint32_t>(n) : nullptr) : patch_index;
  hipLaunchKernelGGL(k_emit, dim3(grid_for(n)), dim3(kBlock), 0, ctx->stream, *em, bt, first, n, n, d_rays, d_patch,
                     (uint32_t *)nullptr, (uint32_t *)nullptr, make_float4(0.0f, 0.0f, 0.0f, 0.0f),
                     (const float4 *)nullptr, 0u, (unsigned long long *)nullptr);
  BZR_HIP(hipGetLastError());
  if (host) {
    BZR_HIP(hipMemcpyAsync(rays_soa, d_rays, rb, hipMemcpyDeviceToHost, ctx->stream));
    if (patch_index) BZR_HIP(hipMemcpyAsync(patch_index, d_patch, pb, hipMemcpyDeviceToHost, ctx->stream));
  }
  BZR_HIP(hipStreamSynchronize(ctx->stream));  // the staged belt tables must outlive the kernel
  return BZR_OK;
}

extern "C" bzr_status bzr_illuminate(bzr_ctx *ctx, const bzr_mesh *const *lenses, const float *ri, uint32_t nlens,
                                     const bzr_emitter *em, uint64_t total_rays, const bzr_target *tg, uint32_t *hist,
                                     uint64_t stats[4], uint32_t flags) {
  if (!ctx) return set_error(BZR_ERR_INVALID_ARGUMENT, "null context");
  if (nlens == 0 || nlens > kMaxLenses) return set_error(BZR_ERR_INVALID_ARGUMENT, "nlens must be 1..8");
  if (!lenses || !ri || !tg || !hist) return set_error(BZR_ERR_INVALID_ARGUMENT, "null argument");
  if (bzr_status s = check_emitter(em)) return s;
  if (!tg->bins_u || !tg->bins_v || !(tg->size_u > 0.0f) || !(tg->size_v > 0.0f))
    return set_error(BZR_ERR_INVALID_ARGUMENT, "target bins and sizes must be positive");
  if (bzr_status s = check_flags(flags)) return s;
  LensSet set{};
  set.count = nlens;
  uint32_t nb = 0;
  for (uint32_t l = 0; l < nlens; ++l) {
    if (bzr_status s = check_ctx_mesh(ctx, lenses[l])) return s;
    set.lens[l] = view_of(lenses[l], ri[l]);
    nb = std::max(nb, set.lens[l].n);
  }
  DeviceGuard g(ctx->device);
  // target plane (normal = axis_u x axis_v normalised, constant = n . origin) and cell sizes, in the
  // oracle's operation order
  const float *au = tg->axis_u, *av = tg->axis_v;
  f3 pn{au[1] * av[2] - au[2] * av[1], au[2] * av[0] - au[0] * av[2], au[0] * av[1] - au[1] * av[0]};
  {
    const float z = pn.x * pn.x + (pn.y * pn.y + pn.z * pn.z);
    if (z > 0.0f) {
      const float s = std::sqrt(z);
      pn = f3{pn.x / s, pn.y / s, pn.z / s};
    }
  }
  const float pc = pn.x * tg->origin[0] + (pn.y * tg->origin[1] + pn.z * tg->origin[2]);
  const float cell_u = tg->size_u / (float)tg->bins_u, cell_v = tg->size_v / (float)tg->bins_v;
  const size_t cells = (size_t)tg->bins_u * tg->bins_v;
  const bool host = !(flags & BZR_DEVICE_PTRS);
  const uint32_t B = chunk_for(ctx, total_rays);
  if (bzr_status s = ensure_buffer(ctx->scratch, ctx->scratch_bytes,
                                   belt_bytes(em->belts) + round256((size_t)B * 24) + 2 * round256((size_t)B * 4) +
                                       round256(32) + (host ? round256(cells * 4) : 0)))
    return s;
  Staging st{static_cast<char *>(ctx->scratch)};
  BeltTable bt;
  std::vector<float> cos_lo;
  std::vector<uint32_t> count, firsts;
  if (bzr_status s = upload_belts(ctx, em, st, bt, cos_lo, count, firsts)) return s;
  float *d_rays = st.take<float>((size_t)B * 6);
  uint32_t *d_st = st.take<uint32_t>(B), *d_seg = st.take<uint32_t>(B);
  unsigned long long *d_stats = st.take<unsigned long long>(4);
  uint32_t *d_hist = host ? st.take<uint32_t>(cells) : hist;
  BZR_HIP(hipMemsetAsync(d_stats, 0, 32, ctx->stream));
  if (host) BZR_HIP(hipMemsetAsync(d_hist, 0, cells * 4, ctx->stream));
  Work w;
  const bool staged = use_staged(flags, B, nb);
  if (staged)
    if (bzr_status s = ensure_work(ctx, B, nb, w)) return s;
  const float4 sphere = make_float4(lenses[0]->sphere[0], lenses[0]->sphere[1], lenses[0]->sphere[2],
                                    lenses[0]->sphere[3]);
  for (uint64_t first = 0; first < total_rays; first += B) {
    const uint32_t m = (uint32_t)std::min<uint64_t>(B, total_rays - first);
    hipLaunchKernelGGL(k_emit, dim3(grid_for(m)), dim3(kBlock), 0, ctx->stream, *em, bt, first, m, B, d_rays,
                       (uint32_t *)nullptr, d_st, d_seg, sphere, set.lens[0].always, set.lens[0].n_always, d_stats);
    if (!staged) {  // the chain in place over the batch; culled rays (status NONE) are skipped
      TraceJob job{};
      job.rays = d_rays;
      job.out_rays = d_rays;
      job.status = d_st;
      job.segments = d_seg;
      job.alive_in = d_st;
      job.n = m;
      job.ld = B;
      if (bzr_status s = run_fused<kModeStage>(ctx, set, job, flags)) return s;
    } else {
      for (uint32_t l = 0; l < nlens; ++l)
        for (uint32_t j = 0; j < 2; ++j) {
          Out o{};
          o.rays = d_rays;
          o.expected_all = j == 0 ? uint32_t(BZR_RR_INSIDE) : uint32_t(BZR_RR_OUTSIDE);
          o.status = d_st;
          o.segments = d_seg;
          o.ri = set.lens[l].ri;
          if (bzr_status s = run_segment<kModeStage>(use_fast(flags), ctx, set.lens[l], d_rays, B, 0, m, d_st, o, w)) return s;
        }
    }
    hipLaunchKernelGGL(k_land, dim3(grid_for(m)), dim3(kBlock), 0, ctx->stream, *tg, make_float4(pn.x, pn.y, pn.z, pc),
                       cell_u, cell_v, d_rays, B, m, d_st, d_hist, d_stats);
    BZR_HIP(hipGetLastError());
  }
  unsigned long long hs[4];
  BZR_HIP(hipMemcpyAsync(hs, d_stats, 32, hipMemcpyDeviceToHost, ctx->stream));
  std::vector<uint32_t> hh(host ? cells : 0);
  if (host) BZR_HIP(hipMemcpyAsync(hh.data(), d_hist, cells * 4, hipMemcpyDeviceToHost, ctx->stream));
  BZR_HIP(hipStreamSynchronize(ctx->stream));
  if (host)
    for (size_t k = 0; k < cells; ++k) hist[k] += hh[k];
  if (stats)
    for (int k = 0; k < 4; ++k) stats[k] = hs[k];
  return BZR_OK;
}
