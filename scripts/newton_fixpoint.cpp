// How often the Newton loop of BezierTriangle::intersect (reference/bezierTriangle.cpp:155-164,
// csRootSearchIterations = 4) reaches a bitwise fixed point before its last iteration, per lane and per
// patch-uniform pass of 64 lanes (an 8x8 wave's lanes whose planar gate passed the patch).  The loop state
// is (middle, pdir): once an iteration leaves both bit-identical, every later iteration recomputes the same
// hit, so a pass could stop there with the same output bits.  Host only: the product's own arithmetic
// (single_ray.cpp, patch_math_body.inc) with a probe at the end of each iteration; cfg4's chain (both lenses,
// inside then outside), sampled 8x8 waves of the 4096^2 frame.
// build: g++ -O2 -std=c++17 -ffp-contract=off scripts/newton_fixpoint.cpp -Iinclude -Iinclude/bzr \
//          -Icuda-bezier-triangle-raytracer_amd/csrc/host -Icuda-bezier-triangle-raytracer_amd/csrc/device \
//          -Lcuda-bezier-triangle-raytracer_amd/lib -lbzr -Wl,-rpath,$PWD/cuda-bezier-triangle-raytracer_amd/lib
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <random>
#include <vector>

static int g_conv = -1;             // iteration at whose end the state stopped changing (4: never), -1: no Newton
static float g_prev[4];
static void probe(int i, float m, float x, float y, float z) {
  const float cur[4] = {m, x, y, z};
  if (i == 0) g_conv = 4;
  else if (g_conv == 4 && std::memcmp(cur, g_prev, sizeof cur) == 0) g_conv = i;
  std::memcpy(g_prev, cur, sizeof cur);
}
#define BZR_NEWTON_PROBE(i, m, d) probe(i, m, (d).x, (d).y, (d).z)
#include "../cuda-bezier-triangle-raytracer_amd/csrc/host/single_ray.cpp"

#include "bzr/bzr.hpp"

int main(int argc, char **argv) {
  const int waves = argc > 1 ? std::atoi(argv[1]) : 300, side = 4096;
  auto makeLens = [](float x) {
    Mesh m;
    m.makeEllipsoid(32, 16, Vector(1.0f, 4.0f, 2.0f));
    m += Vector{x, 0.0f, 0.0f};
    m.standardizeVertices();
    m.standardizeNormals();
    return BezierLens(1.3f, BezierMesh(m));
  };
  BezierLens lens[2] = {makeLens(10.0f), makeLens(13.0f)};
  std::mt19937 rng(7);
  const float y0 = -4.2f, y1 = 4.2f, z0 = -2.1f, z1 = 2.1f, s = static_cast<float>(side);
  long lanes = 0, passes = 0, lane_hist[5] = {0, 0, 0, 0, 0}, pass_hist[5] = {0, 0, 0, 0, 0};
  long saved_iters = 0, lane_slots = 0;
  int sampled = 0;
  while (sampled < waves) {
    const int br = rng() % (side / 8), bc = rng() % (side / 8);
    const float yc = y0 + (y1 - y0) * ((bc * 8 + 4) / s), zc = z0 + (z1 - z0) * ((br * 8 + 4) / s);
    if ((yc / 4) * (yc / 4) + (zc / 2) * (zc / 2) > 1.0f) continue;  // inside the lens outline
    ++sampled;
    std::vector<Ray> ray(64);
    std::vector<int> alive(64, 1);
    for (int w = 0; w < 64; ++w) {
      const float y = y0 + (y1 - y0) * ((static_cast<float>(bc * 8 + w % 8) + 0.5f) / s);
      const float z = z0 + (z1 - z0) * ((static_cast<float>(br * 8 + w / 8) + 0.5f) / s);
      ray[w] = Ray(Vertex{0.0f, y, z}, Vector{1.0f, 0.0f, 0.0f});
    }
    for (int seg = 0; seg < 4; ++seg) {
      BezierMesh const &mesh = lens[seg / 2].getMesh();
      std::map<uint32_t, int> pass_conv;  // patch -> the pass's last converging lane
      for (int w = 0; w < 64; ++w) {
        if (!alive[w]) continue;
        for (uint32_t b = 0; b < mesh.size(); ++b) {
          g_conv = -1;
          (void)bzr::host::patchIntersect(mesh[b], ray[w], false);
          if (g_conv < 0) continue;
          ++lanes;
          ++lane_hist[g_conv];
          auto it = pass_conv.find(b);
          if (it == pass_conv.end()) pass_conv[b] = g_conv;
          else it->second = std::max(it->second, g_conv);
        }
      }
      for (auto const &kv : pass_conv) {
        ++passes;
        ++pass_hist[kv.second];
        if (kv.second < 3) saved_iters += 3 - kv.second;
      }
      lane_slots += (long)pass_conv.size();
      for (int w = 0; w < 64; ++w) {
        if (!alive[w]) continue;
        auto r = bzr::host::lensRefract(&mesh[0], mesh.size(), 1.3f, ray[w],
                                        seg % 2 == 0 ? RefractionResult::cInside : RefractionResult::cOutside);
        if (r.second == RefractionResult::cNone) alive[w] = 0;
        else ray[w] = r.first;
      }
    }
  }
  std::printf("{\"waves\": %d, \"newton_lanes\": %ld, \"passes\": %ld, \"lane_fixed_after_iter\": [%ld, %ld, %ld, %ld], "
              "\"lane_never\": %ld, \"pass_fixed_after_iter\": [%ld, %ld, %ld, %ld], \"pass_never\": %ld, "
              "\"pass_iterations_saved_frac\": %.4f}\n",
              waves, lanes, passes, lane_hist[0], lane_hist[1], lane_hist[2], lane_hist[3], lane_hist[4], pass_hist[0],
              pass_hist[1], pass_hist[2], pass_hist[3], pass_hist[4], passes ? (double)saved_iters / (4.0 * passes) : 0.0);
  return 0;
}
