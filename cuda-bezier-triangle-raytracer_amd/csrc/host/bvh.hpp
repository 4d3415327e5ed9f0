// bvh.hpp -- culling structure of one lens mesh (see bvh.cpp for why it is exact-preserving).
#pragma once
#include <array>
#include <cstdint>
#include <vector>

namespace bzr_host {

constexpr uint32_t kLeafFlag = 0x80000000u;

struct Box {
  std::array<float, 3> lo, hi;
  bool empty = false;
};

// 32-byte node, read with scalar loads: inner (a = left, b = right), leaf (a = first, b = kLeafFlag | count)
struct BvhNode {
  float lo[3];
  uint32_t a;
  float hi[3];
  uint32_t b;
};

// 4-wide node of the device BVH (128 bytes, read with scalar loads): the gate boxes of up to four
// children, SoA by coordinate.  child: inner node index, kLeafFlag | leaf slot (one patch), or
// kEmptyChild (no child, or a subtree whose gate regions are all empty).
constexpr uint32_t kEmptyChild = 0xFFFFFFFFu;
struct Bvh4Node {
  float lo[3][4];
  float hi[3][4];
  uint32_t child[4];
  uint32_t pad[4];
};
static_assert(sizeof(Bvh4Node) == 128, "Bvh4Node layout");

// 4-wide node of the wide-patch subtree (256 bytes, read with four 64-byte scalar loads): each child is
// bounded by an oriented box -- centre c, orthonormal axes u v w, half extents h -- instead of an AABB.
// The wide patches' gate regions are long thin needles in planes through (nearly) the origin (SURVEY.md
// 0.4): their AABBs span the scene, their oriented boxes do not.  One 64-byte record per child (AoS, one
// scalar load each): c.xyz u.xyz v.xyz w.xyz h.xyz, then the child ref.  A child ref with kObbFlag set
// names one of these nodes (index in Bvh::obb).
constexpr uint32_t kObbFlag = 0x40000000u;
struct Bvh4ObbChild {
  float f[15];
  uint32_t child;
};
struct Bvh4ObbNode {
  Bvh4ObbChild c[4];
};
static_assert(sizeof(Bvh4ObbNode) == 256, "Bvh4ObbNode layout");

struct Bvh {
  std::vector<Bvh4Node> nodes4;    // device BVH, root = 0 (always present)
  std::vector<Bvh4ObbNode> obb;    // the wide subtree's nodes (refs kObbFlag | index)
  std::vector<float> patch_obb;    // per patch (mesh order): c, u, v, w, h (15 floats) + 1 if it has one
  std::vector<BvhNode> nodes;      // binary build tree (one patch per leaf), root = 0
  std::vector<uint32_t> order;     // leaf ranges index this: patch index in mesh order; the tree's slots
                                   // are [0, n - always.size()), the always-tested patches follow
  std::vector<uint32_t> always;    // patches whose gate region has no proven bound (bvh.cpp), ascending:
                                   // not in the tree, every wave-segment gate-tests them
  std::vector<float> always_wedge; // per always patch, 8 floats: w.xyz, L, H, B, C, 0 -- the in-plane wedge a
                                   // passing float plane point p lies in, L - B|p| - C(|s|+|p|) <= w.p <=
                                   // H + B|p| + C(|s|+|p|) (inf-norms; bvh.cpp always_wedge): a proven
                                   // pre-test that skips most always-list gates
  std::vector<float> patch_box;    // per order slot: lo.xyz, 0, hi.xyz, 0 (the gate-region box)
  float extent = 0.0f;             // max |coordinate| of any finite box
  float s_max = 0.0f;              // rays with |origin|_inf > s_max take the brute-force path
  float sphere[4] = {0, 0, 0, 0};  // Ritter sphere over the gate-region boxes: centre, radius
};

void ritter_sphere(std::vector<Box> const &box, float out[4]);

// Two trees per lens, built from the same patches for two origin radii (the gate-region boxes' rounding
// slack grows with the radius the ray origins may have):
//   kTierFar   s_max = max(1e3, 100 x span): every ray the culled path takes (farther -> full scan)
//   kTierNear  s_max = max(1, 8 x span): tighter boxes, for waves whose rays all start within it
//              (refracted segments start on the lens; primaries usually start near it)
// span = the largest |control-point coordinate| of the mesh.
constexpr int kTierFar = 0, kTierNear = 1;
// records: n patch records of stride_words floats (bzr_patch layout, 66 words)
Bvh build_bvh(const float *records, uint32_t n, uint32_t stride_words, int tier = kTierFar);

}  // namespace bzr_host
