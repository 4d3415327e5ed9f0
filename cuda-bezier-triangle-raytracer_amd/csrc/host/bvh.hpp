// bvh.hpp -- culling structure of one lens mesh (see bvh.cpp for why it is exact-preserving).
#pragma once
#include <array>
#include <cstdint>
#include <vector>

namespace bzr_host {

constexpr uint32_t kLeafSize = 4;
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

struct Bvh {
  std::vector<BvhNode> nodes;      // root = 0
  std::vector<uint32_t> order;     // leaf ranges index this: patch index in mesh order
  std::vector<float> patch_box;    // per order slot: lo.xyz, 0, hi.xyz, 0 (the gate-region box)
  float extent = 0.0f;             // max |coordinate| of any finite box
  float s_max = 0.0f;              // rays with |origin|_inf > s_max take the brute-force path
};

// records: n patch records of stride_words floats (bzr_patch layout, 66 words)
Bvh build_bvh(const float *records, uint32_t n, uint32_t stride_words);

}  // namespace bzr_host
