// bvh.cpp -- exact-preserving culling structure for one lens mesh (host build, device use).
//
// BezierMesh::intersect (reference/bezierMesh.cpp:206-227) scans every patch.  A patch can
// only contribute when its planar gate passes (reference/bezierTriangle.cpp:124-131): the
// ray/plane point p satisfies 0 <= M p <= 1 componentwise (M = mBarycentricInverse).  That set,
// intersected with the underlying plane, is a convex polygon -- usually the flat triangle
// (cp0, cp1, cp2), but much larger when the plane passes near the origin and M is
// ill-conditioned, so it is computed here in double precision by clipping the
// plane against the six half-spaces of M's rows, loosened by the rounding slack of the float
// gate.  Its inflated AABB is the patch's culling box; a median-split BVH over those boxes is
// traversed on the GPU.  A ray that misses a box cannot pass that patch's gate, so the set of
// patches that reach the Newton stage -- and therefore every output bit -- is the brute-force
// scan's.  The per-ray part of the slack (ray origin magnitude) is added on the device.
#include "bvh.hpp"

#include <algorithm>
#include <exception>
#include <cfloat>
#include <array>
#include <cmath>
#include <cstring>
#include <numeric>
#include <stdexcept>

namespace bzr_host {
namespace {

using d3 = std::array<double, 3>;
d3 sub(d3 a, d3 b) { return {a[0] - b[0], a[1] - b[1], a[2] - b[2]}; }
d3 addm(d3 a, d3 b, double s) { return {a[0] + s * b[0], a[1] + s * b[1], a[2] + s * b[2]}; }
double dotd(d3 a, d3 b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
d3 crossd(d3 a, d3 b) { return {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]}; }
double normd(d3 a) { return std::sqrt(dotd(a, a)); }

// Rounding allowances of the float planar gate (u = 2^-24; X bounds |x|_inf over the region, s_max
// |origin|_inf; n, c the record's plane, nu = |n|).  plane_ray computes D^ = fl(n.s), t^ = fl(fl(c - D^) /
// fl(d.n)) and p^ = fl(s + fl(d t^)).  With p~ = s + d t^ (exact), n.p~ - c = (n.s - D^) + (c - D^) d12 -
// eta t^ (|d12| <= gamma_2, |eta| <= gamma_3 sum |d_i n_i|), and |p^_i - p~_i| <= u (|d_i t^| + |p^_i|);
// bounding each term with |s| <= s_max, |p^|, |p~ - s| <= sqrt3 (X + s_max) gives
//   off-plane distance |n.p^ - c| / nu <= u (sqrt3 (9 s_max + 5 X) + 2 |c| / nu) <= 16 u (X + s_max)
//   distance of p^ from the ray line    <= |p^ - p~| <= 2 sqrt3 u (X + s_max)
// (measured over 2e5 random and grazing rays on cfg5's patches: at most 4.6 u and 1.6 u -- tests/
// test_culling_conservative.py pins both).  Allowances:
//   kEps    the plane slab: 24 u (X + s_max), 1.5x the bound
//   kPad    the box padding for the ray-line distance plus the float slab test's own rounding
//           (t = fma(lo, 1/d, -s/d): ~4 u (X + s_max) in space): 16 u (X + s_max), 2x the sum
//   kSlack  the barycentric slack: fl(M_k p) differs from M_k p by at most gamma_3 sum_l |M_kl| |p_l|
//           (gamma_3 = 3.0000002 u) -- 2^-21 = 8 u is 2.7x that (proven allowance, see gate_region_box)
// The rounding-dominated patches, whose gate no bound covers, get no box at all: they are left out of
// the tree and gate-tested by every wave-segment (Bvh::always), so culling is exact by construction.
#ifndef BZR_BVH_EPS_U
#define BZR_BVH_EPS_U 24.0
#endif
#ifndef BZR_BVH_PAD_U
#define BZR_BVH_PAD_U 16.0
#endif
#ifndef BZR_BVH_KSLACK_LOG2
#define BZR_BVH_KSLACK_LOG2 21
#endif
constexpr double kEps = BZR_BVH_EPS_U / 16777216.0;
constexpr double kPad = BZR_BVH_PAD_U / 16777216.0;
constexpr double kSlack = 1.0 / (1 << BZR_BVH_KSLACK_LOG2);

// Clip convex polygon `poly` (plane points) to { x : g.x + h >= 0 }.
std::vector<d3> clip(std::vector<d3> const &poly, d3 g, double h) {
  std::vector<d3> out;
  std::size_t m = poly.size();
  for (std::size_t i = 0; i < m; ++i) {
    d3 a = poly[i], b = poly[(i + 1) % m];
    double fa = dotd(g, a) + h, fb = dotd(g, b) + h;
    if (fa >= 0) out.push_back(a);
    if ((fa >= 0) != (fb >= 0)) {
      double t = fa / (fa - fb);
      out.push_back(addm(a, sub(b, a), t));
    }
  }
  return out;
}

// Conservative AABB of the region where the float planar gate of one patch can pass, for rays whose
// origin satisfies |s|_inf <= s_max.  The gate accepts p when 0 <= fl(M p) <= 1; p is the float
// ray/plane point, within eps of the plane and within pad of the ray.  So the region is the
// parallelepiped P = { x : -slack <= M_i x <= 1 + slack } cut by the slab |n.x - c| <= eps:
// its AABB is spanned by the two slab-face slices of P and the vertices of P inside the slab.
struct Region {       // the gate region's extreme points (double) and the ray-point padding
  enum Kind { kEmpty, kFinite, kUnbounded };
  Kind kind = kUnbounded;  // kEmpty: never a candidate; kUnbounded: non-finite record data
  bool proven = false;     // the region is a proven bound (else: the patch goes to the always list)
  std::vector<d3> pts;
  double pad = 0.0;
};

Box gate_region_box(const float *rec, double s_max, Region *region = nullptr) {
  d3 n{rec[0], rec[1], rec[2]};
  double c = rec[3];
  const float *m = rec + 49;  // col-major
  d3 row[3];
  for (int i = 0; i < 3; ++i) row[i] = {m[i], m[3 + i], m[6 + i]};
  Box all;
  all.lo = {-HUGE_VALF, -HUGE_VALF, -HUGE_VALF};
  all.hi = {HUGE_VALF, HUGE_VALF, HUGE_VALF};
  double nn = normd(n);
  if (!(nn > 0) || !std::isfinite(c)) return all;
  for (auto const &r : row)
    if (!std::isfinite(r[0]) || !std::isfinite(r[1]) || !std::isfinite(r[2])) return all;
  d3 nu = {n[0] / nn, n[1] / nn, n[2] / nn};
  double cu = c / nn;
  d3 helper = std::fabs(nu[0]) < 0.6 ? d3{1, 0, 0} : (std::fabs(nu[1]) < 0.6 ? d3{0, 1, 0} : d3{0, 0, 1});
  d3 u = crossd(nu, helper);
  double un = normd(u);
  u = {u[0] / un, u[1] / un, u[2] / un};
  d3 v = crossd(nu, u);
  // Q = M^-1 (double): P's vertices are Q b, b in {-slack, 1+slack}^3
  double md[9];
  for (int i = 0; i < 9; ++i) md[i] = m[i];
  auto at = [&md](int i, int j) { return md[j * 3 + i]; };
  double det = at(0, 0) * (at(1, 1) * at(2, 2) - at(1, 2) * at(2, 1)) - at(0, 1) * (at(1, 0) * at(2, 2) - at(1, 2) * at(2, 0)) +
               at(0, 2) * (at(1, 0) * at(2, 1) - at(1, 1) * at(2, 0));
  if (!(std::fabs(det) > 0) || !std::isfinite(det)) return all;
  d3 q[3];
  double ext = std::fabs(cu) + 1.0;
  for (int k = 0; k < 3; ++k) {  // column k of M^-1: inv(i,k) = cof(k,i) / det
    for (int i = 0; i < 3; ++i) {
      int r1 = (k + 1) % 3, r2 = (k + 2) % 3, c1 = (i + 1) % 3, c2 = (i + 2) % 3;
      q[k][i] = (at(r1, c1) * at(r2, c2) - at(r1, c2) * at(r2, c1)) / det;
    }
    ext += 2.0 * normd(q[k]);
  }
  if (!std::isfinite(ext)) return all;
  // Where can a passing float p lie?  fl(M_k p) = M_k p + e_k with |e_k| <= gamma_3 sum_l |M_kl| |p_l|
  // (gamma_3 = 3.0000002 u, u = 2^-24), and the gate needs fl(M p) in [0,1]^3.  With Q = M^-1,
  // p = Q (b - e) for some b in [0,1]^3, so componentwise |p| <= |Q| 1 + G |p| with G = gamma_3 |Q| |M|.
  // When I - G is a nonsingular M-matrix (spectral radius of G < 1; checked by its leading principal
  // minors) that gives |p| <= P = (I - G)^-1 |Q| 1, hence |e_k| <= gamma_3 sum_l |M_kl| P_l, and
  // slack_k = kSlack (sum_l |M_kl| P_l + 1) (kSlack = 2.7 gamma_3) is a proven allowance; X = max(max P,
  // ext) bounds |p|_inf.  |Q| is the double-precision inverse widened by its residual.  Otherwise (the
  // rounding-dominated patches: the rows of M nearly parallel to the normal, fl(M p) is rounding noise
  // near the plane) no bound exists -- along M's near-null direction the noise of fl(M p)
  // grows with |p| and can land in [0,1]^3 arbitrarily far out -- so the patch gets no box: it returns
  // the always-hit box with region->proven false, and build_bvh moves it to the always list.
  const double g3 = 3.0000002 / 16777216.0;
  double rn = 0.0;  // max column sum of |I - M Q~|
  for (int j = 0; j < 3; ++j) {
    double cs = 0.0;
    for (int i = 0; i < 3; ++i) {
      double mq = 0.0;
      for (int k = 0; k < 3; ++k) mq += row[i][k] * q[j][k];
      cs += std::fabs((i == j ? 1.0 : 0.0) - mq);
    }
    rn = std::max(rn, cs);
  }
  double qa[3][3];  // |Q| bound, [i][k] = row i, column k
  for (int i = 0; i < 3; ++i) {
    const double rmax = std::max({std::fabs(q[0][i]), std::fabs(q[1][i]), std::fabs(q[2][i])});
    for (int k = 0; k < 3; ++k) qa[i][k] = std::fabs(q[k][i]) * (1.0 + 1e-12) + 4.0 * rn * rmax;
  }
  double A[3][3];  // I - G
  for (int i = 0; i < 3; ++i)
    for (int l = 0; l < 3; ++l) {
      double gil = 0.0;
      for (int k = 0; k < 3; ++k) gil += qa[i][k] * std::fabs(row[k][l]);
      A[i][l] = (i == l ? 1.0 : 0.0) - g3 * gil * (1.0 + 1e-12);
    }
  const double m1 = A[0][0], m2 = A[0][0] * A[1][1] - A[0][1] * A[1][0];
  const double m3 = A[0][0] * (A[1][1] * A[2][2] - A[1][2] * A[2][1]) - A[0][1] * (A[1][0] * A[2][2] - A[1][2] * A[2][0]) +
                    A[0][2] * (A[1][0] * A[2][1] - A[1][1] * A[2][0]);
  double P[3] = {0.0, 0.0, 0.0};
  bool proven = rn < 1e-4 && m1 > 1e-9 && m2 > 1e-9 && m3 > 1e-9;
  if (proven) {  // P = A^-1 (|Q| 1) by the adjugate (A is a Z-matrix with positive leading minors: an
                 // M-matrix, so A^-1 >= 0; |.| only guards the rounding of entries that are ~0)
    const double qs[3] = {qa[0][0] + qa[0][1] + qa[0][2], qa[1][0] + qa[1][1] + qa[1][2], qa[2][0] + qa[2][1] + qa[2][2]};
    for (int i = 0; i < 3 && proven; ++i) {
      double acc = 0.0;
      for (int l = 0; l < 3; ++l) {
        const int r1 = (l + 1) % 3, r2 = (l + 2) % 3, c1 = (i + 1) % 3, c2 = (i + 2) % 3;
        acc += std::fabs((A[r1][c1] * A[r2][c2] - A[r1][c2] * A[r2][c1]) / m3) * qs[l];  // |(A^-1)[i][l]| (|Q| 1)_l
      }
      P[i] = acc * (1.0 + 1e-9);
      if (!std::isfinite(P[i])) proven = false;
    }
  }
  if (!proven) return all;
  const double X = std::max({ext, P[0], P[1], P[2]});
  if (!std::isfinite(X)) return all;
  if (region) region->proven = true;
  double slack[3];
  for (int k = 0; k < 3; ++k)
    slack[k] = kSlack * (std::fabs(row[k][0]) * P[0] + std::fabs(row[k][1]) * P[1] + std::fabs(row[k][2]) * P[2] + 1.0);
  const double eps = kEps * (X + s_max);  // off-plane distance of the float plane point
  std::vector<d3> pts;
  // the initial square must contain the whole slab slice of the slack-inflated parallelepiped
  double qn = 0.0, smax_slack = std::max({slack[0], slack[1], slack[2]});
  for (int k = 0; k < 3; ++k) qn += normd(q[k]);
  const double e = 2.0 * (qn * (1.0 + 2.0 * smax_slack) + std::fabs(cu) + eps);
  for (double off : {-eps, eps}) {
    d3 x0 = {nu[0] * (cu + off), nu[1] * (cu + off), nu[2] * (cu + off)};
    std::vector<d3> poly = {addm(addm(x0, u, -e), v, -e), addm(addm(x0, u, e), v, -e),
                            addm(addm(x0, u, e), v, e), addm(addm(x0, u, -e), v, e)};
    for (int i = 0; i < 3 && !poly.empty(); ++i) {
      poly = clip(poly, row[i], slack[i]);                                                   // M_i x >= -slack
      if (!poly.empty()) poly = clip(poly, {-row[i][0], -row[i][1], -row[i][2]}, 1.0 + slack[i]);  // <= 1+slack
    }
    pts.insert(pts.end(), poly.begin(), poly.end());
  }
  for (int corner = 0; corner < 8; ++corner) {
    d3 b;
    for (int k = 0; k < 3; ++k) b[k] = (corner >> k) & 1 ? 1.0 + slack[k] : -slack[k];
    d3 p{0, 0, 0};
    for (int k = 0; k < 3; ++k) p = addm(p, q[k], b[k]);
    if (std::fabs(dotd(nu, p) - cu) <= eps) pts.push_back(p);
  }
  d3 lo{HUGE_VAL, HUGE_VAL, HUGE_VAL}, hi{-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
  bool any = false;
  for (auto const &p : pts) {
    any = true;
    if (region) region->pts.push_back(p);
    for (int a = 0; a < 3; ++a) {
      lo[a] = std::min(lo[a], p[a]);
      hi[a] = std::max(hi[a], p[a]);
    }
  }
  Box bx;
  if (region) region->kind = any ? Region::kFinite : Region::kEmpty;
  if (!any) {  // no point of the slab passes the gate even with slack: never a candidate
    bx.lo = {1.0f, 1.0f, 1.0f};
    bx.hi = {0.0f, 0.0f, 0.0f};
    bx.empty = true;
    return bx;
  }
  double pad = kPad * (X + s_max) + 1e-6;  // ray-line distance of the plane point and slab-test rounding
  if (region) region->pad = pad;
  for (int a = 0; a < 3; ++a) {
    bx.lo[a] = static_cast<float>(std::nextafter(lo[a] - pad, -HUGE_VAL));
    bx.hi[a] = static_cast<float>(std::nextafter(hi[a] + pad, HUGE_VAL));
  }
  return bx;
}

#ifndef BZR_BVH_SAH
#define BZR_BVH_SAH 1
#endif

struct Builder {
  std::vector<Box> const &box;
  std::vector<std::array<float, 3>> centre;
  std::vector<uint32_t> &order;
  std::vector<BvhNode> &nodes;

  // Binned surface-area-heuristic split of order[first, first+count) (16 centroid bins per axis):
  // minimises sum over both sides of (box half-area x patches).  The gate-region boxes differ in
  // size by orders of magnitude (ill-conditioned patches have huge ones), which a median split
  // spreads over many subtrees.  Returns the left side's size after partitioning, 0 for "no useful
  // split" (the caller falls back to the median).  Any split keeps the culling exact.
  uint32_t sah_split(uint32_t first, uint32_t count, std::array<float, 3> const &clo, std::array<float, 3> const &chi) {
    constexpr int kBins = 16;
    constexpr double kHuge = 1e30;
    auto area = [](std::array<double, 3> const &lo, std::array<double, 3> const &hi) {
      double e[3];
      for (int a = 0; a < 3; ++a) e[a] = std::max(0.0, hi[a] - lo[a]);
      double s = e[0] * e[1] + e[1] * e[2] + e[2] * e[0];
      return std::isfinite(s) ? s : kHuge;
    };
    double best = HUGE_VAL;
    int best_axis = -1, best_bin = 0;
    for (int a = 0; a < 3; ++a) {
      const double ext = (double)chi[a] - (double)clo[a];
      if (!(ext > 0.0) || !std::isfinite(ext)) continue;
      struct Bin {
        std::array<double, 3> lo{HUGE_VAL, HUGE_VAL, HUGE_VAL}, hi{-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
        uint32_t n = 0;
      } bins[kBins];
      for (uint32_t k = first; k < first + count; ++k) {
        const uint32_t p = order[k];
        int b = (int)((centre[p][a] - (double)clo[a]) / ext * kBins);
        b = std::min(std::max(b, 0), kBins - 1);
        bins[b].n++;
        if (box[p].empty) continue;
        for (int d = 0; d < 3; ++d) {
          bins[b].lo[d] = std::min(bins[b].lo[d], (double)box[p].lo[d]);
          bins[b].hi[d] = std::max(bins[b].hi[d], (double)box[p].hi[d]);
        }
      }
      // sweep: right-side areas / counts from the top, then left side from the bottom
      double right_area[kBins];
      uint32_t right_n[kBins];
      std::array<double, 3> lo{HUGE_VAL, HUGE_VAL, HUGE_VAL}, hi{-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
      uint32_t nr = 0;
      for (int b = kBins - 1; b > 0; --b) {
        for (int d = 0; d < 3; ++d) {
          lo[d] = std::min(lo[d], bins[b].lo[d]);
          hi[d] = std::max(hi[d], bins[b].hi[d]);
        }
        nr += bins[b].n;
        right_area[b] = area(lo, hi);
        right_n[b] = nr;
      }
      lo = {HUGE_VAL, HUGE_VAL, HUGE_VAL};
      hi = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
      uint32_t nl = 0;
      for (int b = 1; b < kBins; ++b) {  // split between bin b-1 and b
        for (int d = 0; d < 3; ++d) {
          lo[d] = std::min(lo[d], bins[b - 1].lo[d]);
          hi[d] = std::max(hi[d], bins[b - 1].hi[d]);
        }
        nl += bins[b - 1].n;
        if (nl == 0 || right_n[b] == 0) continue;
        const double cost = area(lo, hi) * nl + right_area[b] * right_n[b];
        if (cost < best) {
          best = cost;
          best_axis = a;
          best_bin = b;
        }
      }
    }
    if (best_axis < 0) return 0;
    const double ext = (double)chi[best_axis] - (double)clo[best_axis];
    auto mid = std::partition(order.begin() + first, order.begin() + first + count, [&](uint32_t p) {
      int b = (int)((centre[p][best_axis] - (double)clo[best_axis]) / ext * kBins);
      return std::min(std::max(b, 0), kBins - 1) < best_bin;
    });
    const uint32_t cut = static_cast<uint32_t>(mid - (order.begin() + first));
    return (cut == 0 || cut == count) ? 0u : cut;
  }

  uint32_t build(uint32_t first, uint32_t count) {
    uint32_t id = static_cast<uint32_t>(nodes.size());
    nodes.push_back({});
    Box bb;
    bb.lo = {HUGE_VALF, HUGE_VALF, HUGE_VALF};
    bb.hi = {-HUGE_VALF, -HUGE_VALF, -HUGE_VALF};
    std::array<float, 3> clo{HUGE_VALF, HUGE_VALF, HUGE_VALF}, chi{-HUGE_VALF, -HUGE_VALF, -HUGE_VALF};
    for (uint32_t k = first; k < first + count; ++k) {
      Box const &b = box[order[k]];
      for (int a = 0; a < 3; ++a) {
        if (!b.empty) {
          bb.lo[a] = std::min(bb.lo[a], b.lo[a]);
          bb.hi[a] = std::max(bb.hi[a], b.hi[a]);
        }
        clo[a] = std::min(clo[a], centre[order[k]][a]);
        chi[a] = std::max(chi[a], centre[order[k]][a]);
      }
    }
    BvhNode nd;
    std::memcpy(nd.lo, bb.lo.data(), 12);
    std::memcpy(nd.hi, bb.hi.data(), 12);
    if (count <= 1) {
      nd.a = first;
      nd.b = kLeafFlag | count;
      nodes[id] = nd;
      return id;
    }
#if BZR_BVH_SAH
    if (uint32_t cut = sah_split(first, count, clo, chi)) {
      uint32_t left = build(first, cut);
      uint32_t right = build(first + cut, count - cut);
      nd.a = left;
      nd.b = right;
      nodes[id] = nd;
      return id;
    }
#endif
    int axis = 0;
    for (int a = 1; a < 3; ++a)
      if (chi[a] - clo[a] > chi[axis] - clo[axis]) axis = a;
    uint32_t half = count / 2;
    std::nth_element(order.begin() + first, order.begin() + first + half, order.begin() + first + count,
                     [&](uint32_t x, uint32_t y) {
                       return centre[x][axis] < centre[y][axis] || (centre[x][axis] == centre[y][axis] && x < y);
                     });
    uint32_t left = build(first, half);
    uint32_t right = build(first + half, count - half);
    nd.a = left;
    nd.b = right;
    nodes[id] = nd;
    return id;
  }
};

bool box_empty(BvhNode const &nd) { return !(nd.lo[0] <= nd.hi[0] && nd.lo[1] <= nd.hi[1] && nd.lo[2] <= nd.hi[2]); }

// Eigenvectors of a symmetric 3x3 matrix (cyclic Jacobi), columns of v, by decreasing eigenvalue.
void eigen_sym3(double a[3][3], double v[3][3]) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) v[i][j] = i == j ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 32; ++sweep) {
    double off = std::fabs(a[0][1]) + std::fabs(a[0][2]) + std::fabs(a[1][2]);
    if (!(off > 1e-300)) break;
    for (int p = 0; p < 2; ++p)
      for (int q = p + 1; q < 3; ++q) {
        if (std::fabs(a[p][q]) < 1e-300) continue;
        const double th = 0.5 * std::atan2(2.0 * a[p][q], a[q][q] - a[p][p]);
        const double c = std::cos(th), sn = std::sin(th);
        for (int k = 0; k < 3; ++k) {  // A <- J^T A J
          const double akp = a[k][p], akq = a[k][q];
          a[k][p] = c * akp - sn * akq;
          a[k][q] = sn * akp + c * akq;
        }
        for (int k = 0; k < 3; ++k) {
          const double apk = a[p][k], aqk = a[q][k];
          a[p][k] = c * apk - sn * aqk;
          a[q][k] = sn * apk + c * aqk;
        }
        for (int k = 0; k < 3; ++k) {
          const double vkp = v[k][p], vkq = v[k][q];
          v[k][p] = c * vkp - sn * vkq;
          v[k][q] = sn * vkp + c * vkq;
        }
      }
  }
  int ord[3] = {0, 1, 2};
  std::sort(ord, ord + 3, [&](int x, int y) { return a[x][x] > a[y][y]; });
  double w[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) w[i][j] = v[i][ord[j]];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) v[i][j] = w[i][j];
}

// Oriented box (15 floats: c, u, v, w, h) enclosing `pts` inflated by `pad` on every axis.  The axes are
// the points' principal directions, rounded to float; the centre and half extents are computed in double
// against the ROUNDED axes, then widened by `pad` and rounded outward, so the float box contains every
// point in exact arithmetic; the device test's own float error is covered by the pad (bvh.cpp header).
bool fit_obb(std::vector<d3> const &pts, double pad, float out[15]) {
  // the "always hit" box for regions without a finite description (non-finite records: full scan semantics)
  for (int k = 0; k < 15; ++k) out[k] = 0.0f;
  out[3] = out[7] = out[11] = 1.0f;
  out[12] = out[13] = out[14] = HUGE_VALF;
  if (pts.empty()) return false;
  for (auto const &p : pts)
    if (!std::isfinite(p[0]) || !std::isfinite(p[1]) || !std::isfinite(p[2])) return false;
  d3 mean{0, 0, 0};
  for (auto const &p : pts)
    for (int k = 0; k < 3; ++k) mean[k] += p[k];
  for (int k = 0; k < 3; ++k) mean[k] /= (double)pts.size();
  double cov[3][3] = {};
  for (auto const &p : pts)
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) cov[i][j] += (p[i] - mean[i]) * (p[j] - mean[j]);
  double ev[3][3];
  eigen_sym3(cov, ev);
  float ax[3][3];
  d3 u{ev[0][0], ev[1][0], ev[2][0]}, w{ev[0][2], ev[1][2], ev[2][2]};
  double un = normd(u);
  if (!(un > 0) || !std::isfinite(un)) return false;
  u = {u[0] / un, u[1] / un, u[2] / un};
  w = sub(w, {u[0] * dotd(w, u), u[1] * dotd(w, u), u[2] * dotd(w, u)});
  double wn = normd(w);
  if (!(wn > 1e-12)) {  // degenerate spread: any axis perpendicular to u
    d3 helper = std::fabs(u[0]) < 0.6 ? d3{1, 0, 0} : d3{0, 1, 0};
    w = crossd(u, helper);
    wn = normd(w);
  }
  w = {w[0] / wn, w[1] / wn, w[2] / wn};
  d3 v = crossd(w, u);
  const d3 axes[3] = {u, v, w};
  for (int a = 0; a < 3; ++a)
    for (int k = 0; k < 3; ++k) ax[a][k] = static_cast<float>(axes[a][k]);
  for (int a = 0; a < 3; ++a) {
    double lo = HUGE_VAL, hi = -HUGE_VAL;
    for (auto const &p : pts) {
      const double t = p[0] * ax[a][0] + p[1] * ax[a][1] + p[2] * ax[a][2];
      lo = std::min(lo, t);
      hi = std::max(hi, t);
    }
    if (!std::isfinite(lo) || !std::isfinite(hi)) return false;
    (void)lo;
  }
  // centre = mean rounded to float; half extents from the rounded centre along the rounded axes
  float c[3];
  for (int k = 0; k < 3; ++k) c[k] = static_cast<float>(mean[k]);
  float h[3];
  for (int a = 0; a < 3; ++a) {
    double m = 0.0;
    for (auto const &p : pts) {
      const double t = (p[0] - c[0]) * ax[a][0] + (p[1] - c[1]) * ax[a][1] + (p[2] - c[2]) * ax[a][2];
      m = std::max(m, std::fabs(t));
    }
    h[a] = static_cast<float>(std::nextafter(m + pad, HUGE_VAL));
    if (!std::isfinite(h[a])) return false;
  }
  for (int k = 0; k < 3; ++k) out[k] = c[k];
  for (int a = 0; a < 3; ++a)
    for (int k = 0; k < 3; ++k) out[3 + 3 * a + k] = ax[a][k];
  for (int a = 0; a < 3; ++a) out[12 + a] = h[a];
  return true;
}

double half_area(BvhNode const &nd) {
  double e[3];
  for (int a = 0; a < 3; ++a) e[a] = std::max(0.0, (double)nd.hi[a] - (double)nd.lo[a]);
  return e[0] * e[1] + e[1] * e[2] + e[2] * e[0];
}

// Oriented boxes of the wide subtree: binary nodes [wide_first, ...) belong to it (the builder appends
// them after the narrow subtree's); each covers order[range] and its box encloses the gate-region points
// of those patches.
struct ObbBuild {
  uint32_t wide_first = 0xFFFFFFFFu;              // binary nodes from here on are in the wide subtree
  uint32_t max_obb_patches = 4;                   // only nodes over at most this many patches get oriented boxes
  std::vector<std::pair<uint32_t, uint32_t>> range;  // per binary node: (first, count) of order[]
  std::vector<Region> const *region = nullptr;       // per patch (mesh order)
  std::vector<uint32_t> const *order = nullptr;
  std::vector<Bvh4ObbNode> *obb = nullptr;
  bool obb_of(uint32_t n2, float out[15]) const {
    std::vector<d3> pts;
    double pad = 0.0;
    for (uint32_t k = range[n2].first; k < range[n2].first + range[n2].second; ++k) {
      Region const &r = (*region)[(*order)[k]];
      if (r.kind == Region::kEmpty) continue;  // never a candidate
      if (r.kind == Region::kUnbounded) {      // no finite gate region: cannot bound it
        fit_obb({}, 0.0, out);
        return false;
      }
      pts.insert(pts.end(), r.pts.begin(), r.pts.end());
      pad = std::max(pad, r.pad);
    }
    return fit_obb(pts, 2.0 * pad, out);  // 2x: the rotated slab test's own rounding (header)
  }
};

std::pair<uint32_t, uint32_t> fill_ranges(std::vector<BvhNode> const &bin, uint32_t n2,
                                          std::vector<std::pair<uint32_t, uint32_t>> &range) {
  if (bin[n2].b & kLeafFlag) return range[n2] = {bin[n2].a, bin[n2].b & ~kLeafFlag};
  const auto l = fill_ranges(bin, bin[n2].a, range), r = fill_ranges(bin, bin[n2].b, range);
  return range[n2] = {std::min(l.first, r.first), l.second + r.second};
}

// Collapse the binary tree under `n2` into 4-wide nodes: repeatedly open the child with the largest
// box until four children remain.  Subtrees with empty boxes (no patch whose gate can pass) drop out.
// Nodes of the wide subtree become Bvh4ObbNode (ref kObbFlag | index).
uint32_t collapse(std::vector<BvhNode> const &bin, uint32_t n2, std::vector<Bvh4Node> &out, ObbBuild const &ob) {
  if (n2 >= ob.wide_first && !(bin[n2].b & kLeafFlag) && ob.range[n2].second <= ob.max_obb_patches) {
    std::vector<uint32_t> kids = {bin[n2].a, bin[n2].b};
    while (kids.size() < 4) {
      int best = -1;
      double area = -1.0;
      for (int i = 0; i < (int)kids.size(); ++i) {
        BvhNode const &k = bin[kids[i]];
        if ((k.b & kLeafFlag) || box_empty(k)) continue;
        double ar = half_area(k);
        if (ar > area || std::isnan(ar)) {
          area = ar;
          best = i;
        }
      }
      if (best < 0) break;
      uint32_t x = kids[best];
      kids.erase(kids.begin() + best);
      kids.push_back(bin[x].a);
      kids.push_back(bin[x].b);
    }
    const uint32_t id = static_cast<uint32_t>(ob.obb->size());
    ob.obb->push_back({});
    Bvh4ObbNode nd{};
    for (int c = 0; c < 4; ++c) {
      nd.c[c].child = kEmptyChild;
      fit_obb({}, 0.0, nd.c[c].f);  // (unused slots: never tested, their ref is empty)
    }
    for (int c = 0; c < (int)kids.size(); ++c) {
      BvhNode const &k = bin[kids[c]];
      if (box_empty(k)) continue;
      ob.obb_of(kids[c], nd.c[c].f);  // on failure: the always-hit box
      nd.c[c].child = (k.b & kLeafFlag) ? (kLeafFlag | k.a) : collapse(bin, kids[c], out, ob);
    }
    (*ob.obb)[id] = nd;
    return kObbFlag | id;
  }
  uint32_t id = static_cast<uint32_t>(out.size());
  out.push_back({});
  std::vector<uint32_t> kids;
  if (bin[n2].b & kLeafFlag)
    kids.push_back(n2);
  else
    kids = {bin[n2].a, bin[n2].b};
  while (kids.size() < 4) {
    int best = -1;
    double area = -1.0;
    for (int i = 0; i < (int)kids.size(); ++i) {
      BvhNode const &k = bin[kids[i]];
      if ((k.b & kLeafFlag) || box_empty(k)) continue;
      double ar = half_area(k);
      if (ar > area || std::isnan(ar)) {
        area = ar;
        best = i;
      }
    }
    if (best < 0) break;
    uint32_t x = kids[best];
    kids.erase(kids.begin() + best);
    kids.push_back(bin[x].a);
    kids.push_back(bin[x].b);
  }
  Bvh4Node nd{};
  for (int c = 0; c < 4; ++c) nd.child[c] = kEmptyChild;
  for (int c = 0; c < (int)kids.size(); ++c) {
    BvhNode const &k = bin[kids[c]];
    if (box_empty(k)) continue;
    for (int a = 0; a < 3; ++a) {
      nd.lo[a][c] = k.lo[a];
      nd.hi[a][c] = k.hi[a];
    }
    nd.child[c] = (k.b & kLeafFlag) ? (kLeafFlag | k.a) : collapse(bin, kids[c], out, ob);
  }
  out[id] = nd;
  return id;
}

// Wedge pre-test of an always-listed patch (8 floats: w.xyz, L, H, B, C, 0; Bvh::always_wedge).  No box
// bounds where its float gate passes, but a slab does once |p| is known: for any direction w and
// g = M^-T w (so M^T g = w + r), a passing float plane point p has y = M p with y_k = b_k - e_k, b_k in
// [0,1], |e_k| <= gamma_3 |M_k|_1 |p|_inf, hence
//   w.p = g.y - r.p  in  [L - B |p|_inf, H + B |p|_inf],  L = sum min(0, g_k), H = sum max(0, g_k),
//   B = gamma_3 sum_k |g_k| |M_k|_1 + |r|_1.
// w = M's middle right singular vector (eigenvector of M^T M) makes the slab a thin in-plane wedge
// around M's near-null direction (the one the gate's rounding noise runs along): on cfg5 it rejects ~97 %
// of (ray, patch) pairs before the division.  The device evaluates w.p~ at p~ = s + d (num x rcp(cs)),
// within 14 u (|s| + |p~|) of the gate's own p (inf-norm; u = 2^-24; plane_ray's rounding plus v_rcp_f32's
// 1 ulp), so it widens both sides by C (|s| + |p~|), C = 32 u + 14 u B (also covering its own dot
// product).  Any direction is valid, so the eigenvector's accuracy only affects tightness; g's is
// covered by the residual r.  Open wedge (L = -inf, H = +inf) when M or its inverse is not finite.
void always_wedge(const float *rec, float out[8]) {
  out[0] = out[1] = out[2] = 0.0f;
  out[3] = -HUGE_VALF;
  out[4] = HUGE_VALF;
  out[5] = out[6] = out[7] = 0.0f;
  const float *m = rec + 49;  // col-major
  double M[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) M[i][j] = m[j * 3 + i];
  for (auto const &r : M)
    for (double x : r)
      if (!std::isfinite(x)) return;
  double det = M[0][0] * (M[1][1] * M[2][2] - M[1][2] * M[2][1]) - M[0][1] * (M[1][0] * M[2][2] - M[1][2] * M[2][0]) +
               M[0][2] * (M[1][0] * M[2][1] - M[1][1] * M[2][0]);
  if (!(std::fabs(det) > 0) || !std::isfinite(det)) return;
  double Q[3][3];  // M^-1 by cofactors
  for (int i = 0; i < 3; ++i)
    for (int k = 0; k < 3; ++k) {
      const int r1 = (k + 1) % 3, r2 = (k + 2) % 3, c1 = (i + 1) % 3, c2 = (i + 2) % 3;
      Q[i][k] = (M[r1][c1] * M[r2][c2] - M[r1][c2] * M[r2][c1]) / det;
    }
  double A[3][3], V[3][3];  // M^T M and its eigenvectors (columns, decreasing eigenvalue)
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) A[i][j] = M[0][i] * M[0][j] + M[1][i] * M[1][j] + M[2][i] * M[2][j];
  eigen_sym3(A, V);
  double w[3] = {V[0][1], V[1][1], V[2][1]};
  const double wn = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  if (!(wn > 0)) return;
  for (double &x : w) x = static_cast<float>(x / wn);  // the float direction the device uses, exactly
  double g[3];  // g = Q^T w
  for (int k = 0; k < 3; ++k) g[k] = Q[0][k] * w[0] + Q[1][k] * w[1] + Q[2][k] * w[2];
  double r1 = 0.0, gm = 0.0;  // |M^T g - w|_1, and a scale for the double rounding of that residual
  for (int l = 0; l < 3; ++l) {
    double acc = -w[l], mag = std::fabs(w[l]);
    for (int k = 0; k < 3; ++k) {
      acc += M[k][l] * g[k];
      mag += std::fabs(M[k][l] * g[k]);
    }
    r1 += std::fabs(acc);
    gm = std::max(gm, mag);
  }
  const double g3 = 3.0000002 / 16777216.0, u = 1.0 / 16777216.0;
  double L = 0.0, H = 0.0, B = r1 + 1e-12 * gm;
  for (int k = 0; k < 3; ++k) {
    L += std::min(0.0, g[k]);
    H += std::max(0.0, g[k]);
    B += g3 * std::fabs(g[k]) * (std::fabs(M[k][0]) + std::fabs(M[k][1]) + std::fabs(M[k][2]));
  }
  L -= 1e-9 * (std::fabs(L) + 1.0);
  H += 1e-9 * (std::fabs(H) + 1.0);
  B = B * (1.0 + 1e-9) + 1e-30;
  const double C = 32.0 * u + 14.0 * u * B;
  if (!std::isfinite(L) || !std::isfinite(H) || !std::isfinite(B)) return;
  out[0] = static_cast<float>(w[0]);
  out[1] = static_cast<float>(w[1]);
  out[2] = static_cast<float>(w[2]);
  out[3] = std::nextafter(static_cast<float>(L), -HUGE_VALF);
  out[4] = std::nextafter(static_cast<float>(H), HUGE_VALF);
  out[5] = std::nextafter(static_cast<float>(B), HUGE_VALF);
  out[6] = std::nextafter(static_cast<float>(C), HUGE_VALF);
}

}  // namespace

// Patches whose gate-region box exceeds kWideRatio x their triangle's extent go to the wide subtree
// (meshes of at least kWideMinPatches patches).
// (64: the fewest node visits per wave on cfg5 in the host replay bzr_debug_traverse, ratios 4..512 tried.)
constexpr float kWideRatio = 64.0f;
constexpr uint32_t kWideMinPatches = 64;

Bvh build_bvh(const float *records, uint32_t n, uint32_t stride_words, int tier) {
  Bvh out;
  std::vector<Box> box(n);
  Builder bld{box, std::vector<std::array<float, 3>>(n), out.order, out.nodes};
  // ray origins up to s_max use this tree (far tier: 100x the mesh's control-point extent, at least
  // 1e3, farther origins are routed to the brute-force scan by the kernel; near tier: 8x, see bvh.hpp)
  double span = 0.0;
  for (uint32_t i = 0; i < n; ++i)
    for (int k = 0; k < 30; ++k) {
      double x = std::fabs(records[(size_t)i * stride_words + 19 + k]);
      if (std::isfinite(x)) span = std::max(span, x);
    }
  out.s_max = static_cast<float>(tier == kTierNear ? std::max(1.0, 8.0 * span) : std::max(1e3, 100.0 * span));
  out.extent = 0.0f;
  std::vector<Region> region(n);
  for (uint32_t i = 0; i < n; ++i) {
    box[i] = gate_region_box(records + (size_t)i * stride_words, out.s_max, &region[i]);
    for (int a = 0; a < 3; ++a) {
      float lo = box[i].lo[a], hi = box[i].hi[a];
      bld.centre[i][a] = box[i].empty ? 0.0f : (std::isfinite(lo) && std::isfinite(hi) ? 0.5f * (lo + hi) : 0.0f);
      if (!box[i].empty) out.extent = std::max({out.extent, std::fabs(lo), std::fabs(hi)});
    }
  }
  if (!std::isfinite(out.extent)) out.extent = HUGE_VALF;
  out.order.resize(n);
  std::iota(out.order.begin(), out.order.end(), 0u);
  // Patches without a proven gate region (rounding-dominated or non-finite records) leave the tree for the
  // always list: order = [tree slots..., always...], the tree is built over the first n_tree slots.
  {
    auto mid = std::stable_partition(out.order.begin(), out.order.end(), [&](uint32_t i) { return region[i].proven; });
    out.always.assign(mid, out.order.end());
    std::sort(out.always.begin(), out.always.end());
    out.always_wedge.assign(out.always.size() * 8, 0.0f);
    for (size_t k = 0; k < out.always.size(); ++k)
      always_wedge(records + (size_t)out.always[k] * stride_words, &out.always_wedge[8 * k]);
  }
  const uint32_t n_tree = n - static_cast<uint32_t>(out.always.size());
  // Wide patches: gate regions much larger than their own triangle (planes through or near the
  // origin make M ill-conditioned).  Mixed into the tree their boxes would inflate
  // every ancestor's box and send most rays into those subtrees, so they get a subtree of their own
  // beside the narrow patches' (root = (narrow, wide)).
  uint32_t n_narrow = n_tree;
  if (n_tree >= kWideMinPatches) {
    auto wide = [&](uint32_t i) {
      Box const &b = box[i];
      if (b.empty) return false;
      const float *cp = records + (size_t)i * stride_words + 19;
      float tri = 0.0f, ext = 0.0f;
      for (int a = 0; a < 3; ++a) {
        const float lo = std::min({cp[a], cp[3 + a], cp[6 + a]}), hi = std::max({cp[a], cp[3 + a], cp[6 + a]});
        tri = std::max(tri, hi - lo);
        ext = std::max(ext, b.hi[a] - b.lo[a]);
      }
      return !(ext <= kWideRatio * tri);  // also non-finite boxes
    };
    auto mid = std::stable_partition(out.order.begin(), out.order.begin() + n_tree, [&](uint32_t i) { return !wide(i); });
    n_narrow = static_cast<uint32_t>(mid - out.order.begin());
  }
  ObbBuild ob;
  if (n_tree && n_narrow > 0 && n_narrow < n_tree) {
    out.nodes.push_back({});  // root, filled below
    const uint32_t l = bld.build(0, n_narrow);
// BZR_BVH_OBB (A/B knob, default 0): oriented boxes for the wide subtree (nodes over at most
// BZR_BVH_OBB_MAX patches).  Measured on cfg5 (8192^2, staged): k_traverse 34.6 ms with them vs 24.4 ms
// without -- fewer node and leaf visits (host replay 86 + 63 vs 97 + 105 per wave) but a 256-byte node
// costs four dependent scalar loads within the SGPR budget, where an AABB node costs one.
#ifndef BZR_BVH_OBB
#define BZR_BVH_OBB 0
#endif
    if (BZR_BVH_OBB) ob.wide_first = static_cast<uint32_t>(out.nodes.size());
#ifdef BZR_BVH_OBB_MAX
    ob.max_obb_patches = BZR_BVH_OBB_MAX;
#endif
    const uint32_t r = bld.build(n_narrow, n_tree - n_narrow);
    BvhNode root;
    for (int a = 0; a < 3; ++a) {
      root.lo[a] = std::min(out.nodes[l].lo[a], out.nodes[r].lo[a]);
      root.hi[a] = std::max(out.nodes[l].hi[a], out.nodes[r].hi[a]);
    }
    root.a = l;
    root.b = r;
    out.nodes[0] = root;
  } else if (n_tree) {
    bld.build(0, n_tree);
  }
  if (n_tree) {
    ob.range.resize(out.nodes.size());
    fill_ranges(out.nodes, 0, ob.range);
    ob.region = &region;
    ob.order = &out.order;
    ob.obb = &out.obb;
    collapse(out.nodes, 0, out.nodes4, ob);
    // Exact by construction: every leaf the device can reach holds a patch with a proven gate region.
    std::vector<uint32_t> todo{0u};
    while (!todo.empty()) {
      const uint32_t ref = todo.back();
      todo.pop_back();
      for (int c = 0; c < 4; ++c) {
        const uint32_t ch = (ref & kObbFlag) ? out.obb[ref & ~kObbFlag].c[c].child : out.nodes4[ref].child[c];
        if (ch == kEmptyChild) continue;
        if (ch & kLeafFlag) {
          const uint32_t slot = ch & ~kLeafFlag;
          if (slot >= n_tree || !region[out.order[slot]].proven)
            throw std::logic_error("BVH leaf without a proven gate region");
        } else {
          todo.push_back(ch);
        }
      }
    }
  } else {
    Bvh4Node root{};
    for (int c = 0; c < 4; ++c) root.child[c] = kEmptyChild;
    out.nodes4.push_back(root);
  }
  out.patch_box.resize((size_t)n * 8);
  for (uint32_t k = 0; k < n; ++k) {
    Box const &b = box[out.order[k]];
    float *d = &out.patch_box[(size_t)k * 8];
    d[0] = b.lo[0]; d[1] = b.lo[1]; d[2] = b.lo[2]; d[3] = 0.0f;
    d[4] = b.hi[0]; d[5] = b.hi[1]; d[6] = b.hi[2]; d[7] = 0.0f;
  }
  out.patch_obb.assign((size_t)n * 16, 0.0f);
  if (ob.wide_first != 0xFFFFFFFFu)
    for (uint32_t k = n_narrow; k < n_tree; ++k) {  // the wide patches' own boxes (what their parents test)
      const uint32_t p = out.order[k];
      if (region[p].kind == Region::kEmpty) continue;
      fit_obb(region[p].pts, 2.0 * region[p].pad, &out.patch_obb[(size_t)p * 16]);  // always-hit if unbounded
      out.patch_obb[(size_t)p * 16 + 15] = 1.0f;
    }
  {  // the sphere over the tree's (proven) boxes only: the always list has no box (bzr_illuminate tests it
     // behind the sphere per ray instead), so one unproven patch does not disable the cull
    std::vector<Box> proven;
    for (uint32_t p = 0; p < n; ++p)
      if (region[p].proven) proven.push_back(box[p]);
    ritter_sphere(proven, out.sphere);
  }
  return out;
}

// Ritter's bounding sphere (the README's pre-cull, reference/README.md:194) over the corners of every
// non-empty gate-region box given (build_bvh: the proven ones): a ray that misses it cannot meet any of
// those gate regions, so it passes none of their planar gates.  Any non-finite corner disables the cull
// (radius +inf).  The radius is padded by 1e-6 relative so the float-rounded centre and radius still
// enclose every corner.
void ritter_sphere(std::vector<Box> const &box, float out[4]) {
  std::vector<std::array<double, 3>> pts;
  bool finite = true;
  for (Box const &b : box) {
    if (b.empty) continue;
    for (int c = 0; c < 8; ++c) {
      std::array<double, 3> p{(c & 1) ? b.hi[0] : b.lo[0], (c & 2) ? b.hi[1] : b.lo[1], (c & 4) ? b.hi[2] : b.lo[2]};
      finite = finite && std::isfinite(p[0]) && std::isfinite(p[1]) && std::isfinite(p[2]);
      pts.push_back(p);
    }
  }
  out[0] = out[1] = out[2] = 0.0f;
  out[3] = pts.empty() ? 0.0f : HUGE_VALF;
  if (pts.empty() || !finite) return;
  auto d2 = [](std::array<double, 3> const &a, std::array<double, 3> const &b) {
    return (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]);
  };
  auto farthest = [&](std::array<double, 3> const &from) {
    size_t best = 0;
    for (size_t i = 1; i < pts.size(); ++i)
      if (d2(pts[i], from) > d2(pts[best], from)) best = i;
    return pts[best];
  };
  std::array<double, 3> y = farthest(pts[0]), z = farthest(y);
  std::array<double, 3> c{0.5 * (y[0] + z[0]), 0.5 * (y[1] + z[1]), 0.5 * (y[2] + z[2])};
  double r = 0.5 * std::sqrt(d2(y, z));
  for (auto const &p : pts) {  // grow to take every point outside (Ritter's second pass)
    double d = std::sqrt(d2(p, c));
    if (d > r) {
      double nr = 0.5 * (r + d), k = (nr - r) / d;
      for (int a = 0; a < 3; ++a) c[a] += (p[a] - c[a]) * k;
      r = nr;
    }
  }
  double need = 0.0;  // exact enclosing radius about the float-rounded centre
  std::array<double, 3> cf{(double)(float)c[0], (double)(float)c[1], (double)(float)c[2]};
  for (auto const &p : pts) need = std::max(need, std::sqrt(d2(p, cf)));
  for (int a = 0; a < 3; ++a) out[a] = static_cast<float>(cf[a]);
  out[3] = static_cast<float>(std::nextafter(need * (1.0 + 1e-6) + 1e-6, HUGE_VAL));
}

}  // namespace bzr_host

// ---- debug / test entry point (include/bzr_debug.h) ----
extern "C" void bzr_internal_set_error(const char *msg);
extern "C" int32_t bzr_debug_gate_boxes_tier(const void *patches, uint32_t n, uint32_t stride, int32_t tier,
                                             float *boxes, float *s_max) {
  try {
  if ((!patches && n) || (!boxes && n) || !s_max || stride % 4 || stride < 264) return 1;
  if (tier != bzr_host::kTierFar && tier != bzr_host::kTierNear) return 1;
  bzr_host::Bvh bvh = bzr_host::build_bvh(static_cast<const float *>(patches), n, stride / 4, tier);
  for (uint32_t k = 0; k < n; ++k) {
    uint32_t p = bvh.order[k];
    for (int a = 0; a < 3; ++a) {
      boxes[(size_t)p * 6 + a] = bvh.patch_box[(size_t)k * 8 + a];
      boxes[(size_t)p * 6 + 3 + a] = bvh.patch_box[(size_t)k * 8 + 4 + a];
    }
  }
  *s_max = bvh.s_max;
  return 0;
  } catch (std::exception const &e) {  // build_bvh's invariant checks: a status, not a throw across the C ABI
    bzr_internal_set_error(e.what());
    return 2;
  }
}

extern "C" int32_t bzr_debug_gate_boxes(const void *patches, uint32_t n, uint32_t stride, float *boxes, float *s_max) {
  return bzr_debug_gate_boxes_tier(patches, n, stride, bzr_host::kTierFar, boxes, s_max);
}

namespace {
float safe_inv_h(float x) { return 1.0f / (std::fabs(x) < 1e-20f ? std::copysign(1e-20f, x) : x); }
// same operation order as the device slab() in trace.hip (BZR_SLAB_FMA: fma(lo, inv, -s*inv))
bool slab_h(const float lo[3], const float hi[3], const float s[3], const float inv[3]) {
  float a[3], b[3];
  for (int k = 0; k < 3; ++k) {
    const float sinv = s[k] * inv[k];
    a[k] = std::fma(lo[k], inv[k], -sinv);
    b[k] = std::fma(hi[k], inv[k], -sinv);
  }
  float tnear = std::fmax(std::fmax(std::fmin(a[0], b[0]), std::fmin(a[1], b[1])), std::fmin(a[2], b[2]));
  float tfar = std::fmin(std::fmin(std::fmax(a[0], b[0]), std::fmax(a[1], b[1])), std::fmax(a[2], b[2]));
  return tnear <= tfar && tfar >= 0.0f;
}
}  // namespace

namespace {
// host mirror of the device obb_hit (trace.hip; 1/x where the device uses v_rcp_f32: statistics only)
bool obb_h(const float f[15], const float s[3], const float d[3]) {
  const float r[3] = {s[0] - f[0], s[1] - f[1], s[2] - f[2]};
  float tnear = -FLT_MAX, tfar = FLT_MAX;
  for (int a = 0; a < 3; ++a) {
    const float *u = f + 3 + 3 * a;
    const float o = std::fma(r[0], u[0], std::fma(r[1], u[1], r[2] * u[2]));
    const float dd = std::fma(d[0], u[0], std::fma(d[1], u[1], d[2] * u[2]));
    const float inv = 1.0f / (std::fabs(dd) < 1e-20f ? std::copysign(1e-20f, dd) : dd);
    const float h = f[12 + a], t1 = (-h - o) * inv, t2 = (h - o) * inv;
    tnear = std::fmax(tnear, std::fmin(t1, t2));
    tfar = std::fmin(tfar, std::fmax(t1, t2));
  }
  return tnear <= tfar && tfar >= 0.0f;
}
}  // namespace

// Per patch (mesh order): its oriented gate-region box (c, u, v, w, h) and a flag word 1.0f when the patch
// is in the wide subtree (the box its parent node tests), else 16 zeros.
extern "C" int32_t bzr_debug_gate_obbs(const void *patches, uint32_t n, uint32_t stride, int32_t tier, float *out) {
  try {
  if ((!patches && n) || (!out && n) || stride % 4 || stride < 264) return 1;
  if (tier != bzr_host::kTierFar && tier != bzr_host::kTierNear) return 1;
  bzr_host::Bvh bvh = bzr_host::build_bvh(static_cast<const float *>(patches), n, stride / 4, tier);
  std::copy(bvh.patch_obb.begin(), bvh.patch_obb.begin() + (size_t)n * 16, out);  // (memcpy from an empty vector is UB)
  return 0;
  } catch (std::exception const &e) {  // build_bvh's invariant checks: a status, not a throw across the C ABI
    bzr_internal_set_error(e.what());
    return 2;
  }
}

extern "C" int32_t bzr_debug_traverse(const void *patches, uint32_t n, uint32_t stride, const float *rays, uint32_t nr,
                                      uint8_t *hits, uint64_t stats[4]) {
  try {
  if ((!patches && n) || (!rays && nr) || !stats || stride % 4 || stride < 264) return 1;
  bzr_host::Bvh far = bzr_host::build_bvh(static_cast<const float *>(patches), n, stride / 4, bzr_host::kTierFar);
  bzr_host::Bvh near = bzr_host::build_bvh(static_cast<const float *>(patches), n, stride / 4, bzr_host::kTierNear);
  for (int k = 0; k < 4; ++k) stats[k] = 0;
  for (uint32_t w0 = 0; w0 < nr; w0 += 64) {
    uint32_t lanes = std::min<uint32_t>(64, nr - w0);
    float s[64][3], d[64][3], inv[64][3];
    bool active[64];
    for (uint32_t l = 0; l < lanes; ++l) {
      uint32_t r = w0 + l;
      for (int k = 0; k < 3; ++k) {
        s[l][k] = rays[(size_t)k * nr + r];
        d[l][k] = rays[(size_t)(3 + k) * nr + r];
        inv[l][k] = safe_inv_h(d[l][k]);
      }
      active[l] = std::fmax(std::fmax(std::fabs(s[l][0]), std::fabs(s[l][1])), std::fabs(s[l][2])) <= far.s_max;
    }
    bool all_near = true;  // the kernel's wave-uniform tier choice
    for (uint32_t l = 0; l < lanes; ++l)
      all_near &= !active[l] || std::fmax(std::fmax(std::fabs(s[l][0]), std::fabs(s[l][1])), std::fabs(s[l][2])) <= near.s_max;
    bzr_host::Bvh const &bvh = all_near ? near : far;
    stats[3] += 1;
    if (!n) continue;
    std::vector<uint32_t> stack{0u};
    while (!stack.empty()) {
      uint32_t node = stack.back();
      stack.pop_back();
      stats[0] += 1;
      const bool is_obb = node & bzr_host::kObbFlag;
      bzr_host::Bvh4Node const *nd = is_obb ? nullptr : &bvh.nodes4[node];
      bzr_host::Bvh4ObbNode const *od = is_obb ? &bvh.obb[node & ~bzr_host::kObbFlag] : nullptr;
      for (int c = 0; c < 4; ++c) {
        const uint32_t child = is_obb ? od->c[c].child : nd->child[c];
        if (child == bzr_host::kEmptyChild) continue;
        bool any = false;
        bool hit[64];
        if (is_obb) {
          for (uint32_t l = 0; l < lanes; ++l) any |= (hit[l] = active[l] && obb_h(od->c[c].f, s[l], d[l]));
        } else {
          float lo[3] = {nd->lo[0][c], nd->lo[1][c], nd->lo[2][c]}, hi[3] = {nd->hi[0][c], nd->hi[1][c], nd->hi[2][c]};
          for (uint32_t l = 0; l < lanes; ++l) any |= (hit[l] = active[l] && slab_h(lo, hi, s[l], inv[l]));
        }
        if (!any) continue;
        if (child & bzr_host::kLeafFlag) {
          uint32_t b = bvh.order[child & ~bzr_host::kLeafFlag];
          stats[1] += 1;
          for (uint32_t l = 0; l < lanes; ++l)
            if (hit[l]) {
              stats[2] += 1;
              if (hits) hits[(size_t)(w0 + l) * n + b] = 1;
            }
        } else {
          stack.push_back(child);
        }
      }
    }
    for (uint32_t b : bvh.always) {  // gate-tested by every wave-segment (the kernel's always loop)
      stats[1] += 1;
      for (uint32_t l = 0; l < lanes; ++l)
        if (active[l]) {
          stats[2] += 1;
          if (hits) hits[(size_t)(w0 + l) * n + b] = 1;
        }
    }
  }
  return 0;
  } catch (std::exception const &e) {  // build_bvh's invariant checks: a status, not a throw across the C ABI
    bzr_internal_set_error(e.what());
    return 2;
  }
}

namespace {
// Host mirror of the device's wave-bundle box test (trace.hip bundle_box): origins in [sl, sh], directions in
// [dl, dh] (per axis); see there for the derivation.  rl / rh: 1 / the clamped direction bounds, mixed: the
// axis's clamped bounds straddle zero.
struct BundleH {
  float sl[3], sh[3], rl[3], rh[3];
  bool mixed[3];
  bool finite;
};
BundleH bundle_h(const float (*s)[3], const float (*d)[3], const bool *act, uint32_t lanes) {
  BundleH b{};
  const float inf = HUGE_VALF;
  float dl[3], dh[3];
  for (int a = 0; a < 3; ++a) b.sl[a] = dl[a] = inf, b.sh[a] = dh[a] = -inf;
  for (uint32_t l = 0; l < lanes; ++l)
    if (act[l])
      for (int a = 0; a < 3; ++a) {
        b.sl[a] = std::fmin(b.sl[a], s[l][a]);
        b.sh[a] = std::fmax(b.sh[a], s[l][a]);
        dl[a] = std::fmin(dl[a], d[l][a]);
        dh[a] = std::fmax(dh[a], d[l][a]);
      }
  b.finite = true;
  for (int a = 0; a < 3; ++a) {
    b.finite &= std::fabs(b.sl[a]) <= 1e30f && std::fabs(b.sh[a]) <= 1e30f && std::fabs(dl[a]) <= 1e30f && std::fabs(dh[a]) <= 1e30f;
    const float lo = dl[a] > 1e-20f ? dl[a] : std::fmin(dl[a], -1e-20f);
    const float hi = dh[a] < -1e-20f ? dh[a] : std::fmax(dh[a], 1e-20f);
    b.rl[a] = 1.0f / lo;
    b.rh[a] = 1.0f / hi;
    b.mixed[a] = lo < 0.0f && hi > 0.0f;
  }
  return b;
}
// The wave's bundle width measure of the walk choice (trace.hip bundle_spread): the largest direction
// interval over the three axes.
float bundle_spread_h(const float (*s)[3], const float (*d)[3], const bool *act, uint32_t lanes) {
  (void)s;
  float w = 0.0f;
  for (int a = 0; a < 3; ++a) {
    float lo = HUGE_VALF, hi = -HUGE_VALF;
    for (uint32_t l = 0; l < lanes; ++l)
      if (act[l]) lo = std::fmin(lo, d[l][a]), hi = std::fmax(hi, d[l][a]);
    w = std::fmax(w, hi - lo);
  }
  return w;
}
bool bundle_box_h(const BundleH &b, const float lo[3], const float hi[3]) {
  if (!b.finite) return true;
  float tn = -HUGE_VALF, tf = HUGE_VALF;
  for (int a = 0; a < 3; ++a) {
    const float A = (hi[a] - b.sl[a]) * b.rl[a], B = (lo[a] - b.sh[a]) * b.rh[a];
    tn = std::fmax(tn, b.mixed[a] ? std::fmax(A, B) : std::fmin(A, B));
    tf = std::fmin(tf, b.mixed[a] ? HUGE_VALF : std::fmax(A, B));
  }
  tn -= std::fabs(tn) * 0x1p-21f + 0x1p-126f;
  tf += std::fabs(tf) * 0x1p-21f + 0x1p-126f;
  return !(tn > tf) && !(tf < 0.0f);  // NaN keeps the box
}
}  // namespace

// Host mirror of the device planar gate (trace.hip planar_gate, BZR_GATE_FLAT; built with -ffp-contract=off
// like the device code, so the same float operations in the same order): q = the 16-float planar record.
bool planar_gate_h(const float q[16], const float s[3], const float d[3]) {
  const float cs = d[0] * q[0] + (d[1] * q[1] + d[2] * q[2]);
  const float t = (q[3] - (q[0] * s[0] + (q[1] * s[1] + q[2] * s[2]))) / cs;
  const float ip[3] = {s[0] + d[0] * t, s[1] + d[1] * t, s[2] + d[2] * t};
  const bool valid = (std::fabs(cs) >= 0.00001f) & (t > 0.0f) & (std::fabs(t) > -q[4]) & (std::fabs(t) > q[5]);
  const float b0 = q[6] * ip[0] + (q[7] * ip[1] + q[8] * ip[2]);
  const float b1 = q[9] * ip[0] + (q[10] * ip[1] + q[11] * ip[2]);
  const float b2 = q[12] * ip[0] + (q[13] * ip[1] + q[14] * ip[2]);
  return valid & (b0 >= 0.0f) & (b0 <= 1.0f) & (b1 >= 0.0f) & (b1 <= 1.0f) & (b2 >= 0.0f) & (b2 <= 1.0f);
}
// The planar record of patch record r (66 words): the device's `planar` / leaf layout.
void planar_of(const float *r, float q[16]) {
  const float *m = r + 49;  // col-major M
  const float v[16] = {r[0], r[1], r[2], r[3], r[58], r[59], m[0], m[3], m[6], m[1], m[4], m[7], m[2], m[5], m[8], 0.0f};
  std::memcpy(q, v, sizeof v);
}
void ivdot_h(const float n[3], const float lo[3], const float hi[3], float &a, float &b) {
  a = (n[0] >= 0.0f ? n[0] * lo[0] : n[0] * hi[0]) + (n[1] >= 0.0f ? n[1] * lo[1] : n[1] * hi[1]) +
      (n[2] >= 0.0f ? n[2] * lo[2] : n[2] * hi[2]);
  b = (n[0] >= 0.0f ? n[0] * hi[0] : n[0] * lo[0]) + (n[1] >= 0.0f ? n[1] * hi[1] : n[1] * lo[1]) +
      (n[2] >= 0.0f ? n[2] * hi[2] : n[2] * lo[2]);
}
float amax_h(float lo, float hi) { return std::fmax(std::fabs(lo), std::fabs(hi)); }
// Host mirror of the device leaf pre-test (trace.hip bundle_gate_keep): false only when no ray of the
// bundle (origins [sl, sh], directions [dl, dh]) can pass the leaf's planar gate.  1/x where the device
// uses v_rcp_f32 (the 6u widening covers both).
bool bundle_gate_keep_h(const BundleH &b, const float dl[3], const float dh[3], const float q[16]) {
  if (!b.finite) return true;
  constexpr float u = 0x1p-24f;
  const float n[3] = {q[0], q[1], q[2]};
  float csl, csh, nsl, nsh;
  ivdot_h(n, dl, dh, csl, csh);
  ivdot_h(n, b.sl, b.sh, nsl, nsh);
  const float mc = 8.0f * u * (std::fabs(n[0]) * amax_h(dl[0], dh[0]) + std::fabs(n[1]) * amax_h(dl[1], dh[1]) +
                               std::fabs(n[2]) * amax_h(dl[2], dh[2]));
  const float ms = 8.0f * u * (std::fabs(n[0]) * amax_h(b.sl[0], b.sh[0]) + std::fabs(n[1]) * amax_h(b.sl[1], b.sh[1]) +
                               std::fabs(n[2]) * amax_h(b.sl[2], b.sh[2]) + std::fabs(q[3]));
  csl -= mc;
  csh += mc;
  const float numl = (q[3] - nsh) - ms, numh = (q[3] - nsl) + ms;
  if (csl > -0.00001f && csh < 0.00001f) return false;
  if (!(csl > 0.0f || csh < 0.0f)) return true;
  const float r1 = 1.0f / csl, r2 = 1.0f / csh;
  const float a1 = numl * r1, a2 = numl * r2, a3 = numh * r1, a4 = numh * r2;
  float tlo = std::fmin(std::fmin(a1, a2), std::fmin(a3, a4)), thi = std::fmax(std::fmax(a1, a2), std::fmax(a3, a4));
  tlo -= 6.0f * u * std::fabs(tlo);
  thi += 6.0f * u * std::fabs(thi);
  if (!(thi <= 1e30f)) return true;
  if (thi <= std::fmax(std::fmax(-q[4], q[5]), 0.0f)) return false;  // t > max(0, -hin, hout) for no ray
  tlo = std::fmax(tlo, 0.0f);
  float pl[3], ph[3], pm0 = 0.0f, smax = 0.0f;
  for (int a = 0; a < 3; ++a) {
    const float x1 = dl[a] * tlo, x2 = dl[a] * thi, x3 = dh[a] * tlo, x4 = dh[a] * thi;
    pl[a] = b.sl[a] + std::fmin(std::fmin(x1, x2), std::fmin(x3, x4));
    ph[a] = b.sh[a] + std::fmax(std::fmax(x1, x2), std::fmax(x3, x4));
    pm0 = std::fmax(pm0, amax_h(pl[a], ph[a]));
    smax = std::fmax(smax, amax_h(b.sl[a], b.sh[a]));
  }
  const float e = 8.0f * u * (smax + pm0);
  for (int k = 0; k < 3; ++k) {
    const float mrow[3] = {q[6 + 3 * k], q[7 + 3 * k], q[8 + 3 * k]};
    float lo, hi;
    ivdot_h(mrow, pl, ph, lo, hi);
    const float eb = (std::fabs(mrow[0]) + std::fabs(mrow[1]) + std::fabs(mrow[2])) * (e + 8.0f * u * pm0) + 1e-30f;
    if (hi + eb < 0.0f || lo - eb > 1.0f) return false;
  }
  return true;
}

// Host replay of a wave-bundle walk (diagnostic): per 64-ray wave, the tree is walked in batches of up to
// 16 nodes (64 child slots, one per lane) with the bundle box test instead of each lane's slab test, and
// compared with the per-lane walk of bzr_debug_traverse.  stats: [0] waves, [1] bundle batches, [2] bundle
// leaves, [3] per-lane node visits, [4] per-lane leaves, [5] per-lane leaves the bundle missed (must be 0),
// [6] child slots tested, [7] deepest work stack (nodes).  Oriented-box nodes are walked per lane in both.
extern "C" int32_t bzr_debug_traverse_bundle(const void *patches, uint32_t n, uint32_t stride, const float *rays,
                                             uint32_t nr, float max_spread, uint64_t stats[12]) {
  try {
  if ((!patches && n) || (!rays && nr) || !stats || stride % 4 || stride < 264) return 1;
  bzr_host::Bvh far = bzr_host::build_bvh(static_cast<const float *>(patches), n, stride / 4, bzr_host::kTierFar);
  bzr_host::Bvh near = bzr_host::build_bvh(static_cast<const float *>(patches), n, stride / 4, bzr_host::kTierNear);
  for (int k = 0; k < 12; ++k) stats[k] = 0;
  for (uint32_t w0 = 0; w0 < nr; w0 += 64) {
    const uint32_t lanes = std::min<uint32_t>(64, nr - w0);
    float s[64][3], d[64][3], inv[64][3];
    bool active[64];
    bool any_act = false;
    for (uint32_t l = 0; l < lanes; ++l) {
      for (int k = 0; k < 3; ++k) {
        s[l][k] = rays[(size_t)k * nr + w0 + l];
        d[l][k] = rays[(size_t)(3 + k) * nr + w0 + l];
        inv[l][k] = safe_inv_h(d[l][k]);
      }
      const float am = std::fmax(std::fmax(std::fabs(s[l][0]), std::fabs(s[l][1])), std::fabs(s[l][2]));
      active[l] = am <= far.s_max && std::isfinite(d[l][0]) && (d[l][0] != 0.0f || d[l][1] != 0.0f || d[l][2] != 0.0f);
      any_act |= active[l];
    }
    if (!any_act || !n) continue;
    bool all_near = true;
    for (uint32_t l = 0; l < lanes; ++l)
      all_near &= !active[l] || std::fmax(std::fmax(std::fabs(s[l][0]), std::fabs(s[l][1])), std::fabs(s[l][2])) <= near.s_max;
    bzr_host::Bvh const &bvh = all_near ? near : far;
    stats[0] += 1;
    // per-lane walk: leaves any lane reaches
    std::vector<uint32_t> lane_leaves, stack{0u};
    while (!stack.empty()) {
      const uint32_t node = stack.back();
      stack.pop_back();
      stats[3] += 1;
      const bool is_obb = node & bzr_host::kObbFlag;
      for (int c = 0; c < 4; ++c) {
        const uint32_t child = is_obb ? bvh.obb[node & ~bzr_host::kObbFlag].c[c].child : bvh.nodes4[node].child[c];
        if (child == bzr_host::kEmptyChild) continue;
        bool any = false;
        for (uint32_t l = 0; l < lanes && !any; ++l) {
          if (!active[l]) continue;
          if (is_obb) any = obb_h(bvh.obb[node & ~bzr_host::kObbFlag].c[c].f, s[l], d[l]);
          else {
            auto const &nd = bvh.nodes4[node];
            const float lo[3] = {nd.lo[0][c], nd.lo[1][c], nd.lo[2][c]}, hi[3] = {nd.hi[0][c], nd.hi[1][c], nd.hi[2][c]};
            any = slab_h(lo, hi, s[l], inv[l]);
          }
        }
        if (!any) continue;
        if (child & bzr_host::kLeafFlag) lane_leaves.push_back(child & ~bzr_host::kLeafFlag);
        else stack.push_back(child);
      }
    }
    stats[4] += lane_leaves.size();
    // bundle walk in batches of up to 16 nodes (or, for a bundle wider than max_spread, the per-lane walk)
    const BundleH b = bundle_h(s, d, active, lanes);
    if (bundle_spread_h(s, d, active, lanes) > max_spread) {
      stats[8] += 1;
      stats[1] += 0;
      stats[2] += lane_leaves.size();
      continue;
    }
    std::vector<uint32_t> bundle_leaves, work{0u};
    while (!work.empty()) {
      const long room = (64 - (long)work.size()) / 3;  // the device's kStack = 64 rule (trace.hip bundle_batch)
      const size_t take = std::min<size_t>(std::min<size_t>(16, work.size()), (size_t)std::max(room, 1L));
      std::vector<uint32_t> batch(work.end() - take, work.end());
      work.resize(work.size() - take);
      stats[1] += 1;
      stats[7] = std::max<uint64_t>(stats[7], work.size() + take);
      size_t pushed = 0;
      for (uint32_t node : batch) {
        const bool is_obb = node & bzr_host::kObbFlag;
        for (int c = 0; c < 4; ++c) {
          const uint32_t child = is_obb ? bvh.obb[node & ~bzr_host::kObbFlag].c[c].child : bvh.nodes4[node].child[c];
          if (child == bzr_host::kEmptyChild) continue;
          stats[6] += 1;
          bool hit = false;
          if (is_obb) {
            for (uint32_t l = 0; l < lanes && !hit; ++l) hit = active[l] && obb_h(bvh.obb[node & ~bzr_host::kObbFlag].c[c].f, s[l], d[l]);
          } else {
            auto const &nd = bvh.nodes4[node];
            const float lo[3] = {nd.lo[0][c], nd.lo[1][c], nd.lo[2][c]}, hi[3] = {nd.hi[0][c], nd.hi[1][c], nd.hi[2][c]};
            hit = bundle_box_h(b, lo, hi);
          }
          if (!hit) continue;
          if (child & bzr_host::kLeafFlag) bundle_leaves.push_back(child & ~bzr_host::kLeafFlag);
          else {
            work.push_back(child);
            ++pushed;
          }
        }
      }
      if (work.size() > 64) stats[9] += 1;  // the device's stack would overflow here
    }
    stats[2] += bundle_leaves.size();
    // the leaf pre-test: which admitted leaves a bundle-level gate keeps; none whose exact gate some lane
    // passes may be rejected
    float dl[3], dh[3];
    for (int a = 0; a < 3; ++a) {
      dl[a] = HUGE_VALF;
      dh[a] = -HUGE_VALF;
      for (uint32_t l = 0; l < lanes; ++l)
        if (active[l]) dl[a] = std::fmin(dl[a], d[l][a]), dh[a] = std::fmax(dh[a], d[l][a]);
    }
    for (uint32_t slot : bundle_leaves) {
      float q[16];
      planar_of(static_cast<const float *>(patches) + (size_t)(stride / 4) * bvh.order[slot], q);
      const bool keep = bundle_gate_keep_h(b, dl, dh, q);
      stats[10] += keep;
      if (!keep)
        for (uint32_t l = 0; l < lanes; ++l)
          if (active[l] && planar_gate_h(q, s[l], d[l])) {
            stats[11] += 1;
            break;
          }
    }
    std::sort(bundle_leaves.begin(), bundle_leaves.end());
    for (uint32_t x : lane_leaves) stats[5] += !std::binary_search(bundle_leaves.begin(), bundle_leaves.end(), x);
  }
  return 0;
  } catch (std::exception const &e) {  // build_bvh's invariant checks: a status, not a throw across the C ABI
    bzr_internal_set_error(e.what());
    return 2;
  }
}

// The always list of one tier (patches without a proven gate region, ascending): count, and the indices
// when `out` is not null.
extern "C" int32_t bzr_debug_always_list(const void *patches, uint32_t n, uint32_t stride, int32_t tier, uint32_t *out,
                                         uint32_t *count) {
  try {
  if ((!patches && n) || !count || stride % 4 || stride < 264) return 1;
  if (tier != bzr_host::kTierFar && tier != bzr_host::kTierNear) return 1;
  bzr_host::Bvh bvh = bzr_host::build_bvh(static_cast<const float *>(patches), n, stride / 4, tier);
  *count = static_cast<uint32_t>(bvh.always.size());
  if (out) std::copy(bvh.always.begin(), bvh.always.end(), out);
  return 0;
  } catch (std::exception const &e) {  // build_bvh's invariant checks: a status, not a throw across the C ABI
    bzr_internal_set_error(e.what());
    return 2;
  }
}

// The always list's wedge pre-test words (bvh.hpp Bvh::always_wedge), 8 floats per always-listed patch.
extern "C" int32_t bzr_debug_always_wedges(const void *patches, uint32_t n, uint32_t stride, int32_t tier, float *out) {
  try {
  if ((!patches && n) || !out || stride % 4 || stride < 264) return 1;
  if (tier != bzr_host::kTierFar && tier != bzr_host::kTierNear) return 1;
  bzr_host::Bvh bvh = bzr_host::build_bvh(static_cast<const float *>(patches), n, stride / 4, tier);
  std::copy(bvh.always_wedge.begin(), bvh.always_wedge.end(), out);
  return 0;
  } catch (std::exception const &e) {  // build_bvh's invariant checks: a status, not a throw across the C ABI
    bzr_internal_set_error(e.what());
    return 2;
  }
}

extern "C" int32_t bzr_debug_bounding_sphere(const void *patches, uint32_t n, uint32_t stride, float out[4]) {
  try {
  if ((!patches && n) || !out || stride % 4 || stride < 264) return 1;
  bzr_host::Bvh bvh = bzr_host::build_bvh(static_cast<const float *>(patches), n, stride / 4);
  for (int k = 0; k < 4; ++k) out[k] = bvh.sphere[k];
  return 0;
  } catch (std::exception const &e) {  // build_bvh's invariant checks: a status, not a throw across the C ABI
    bzr_internal_set_error(e.what());
    return 2;
  }
}
