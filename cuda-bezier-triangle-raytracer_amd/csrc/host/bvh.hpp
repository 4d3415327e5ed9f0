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

struct Bvh {
  std::vector<Bvh4Node> nodes4;    // device BVH, root = 0 (always present)
  std::vector<BvhNode> nodes;      // binary build tree (one patch per leaf), root = 0
  std::vector<uint32_t> order;     // leaf ranges index this: patch index in mesh order
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
