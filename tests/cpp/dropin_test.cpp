// dropin_test.cpp -- a reference-style caller compiled against the drop-in headers.
//
// It includes the reference's header names (include/bzr/*.h) and uses the reference's API the way
// reference/test.cpp and reference/googleTest.cpp do.  Part 1 restates the googleTest L1 cases
// (reference/googleTest.cpp:46-353, cgEpsilon = 1e-4) on the product's value types; part 2 runs the
// host preprocessing API; part 3 (only with a HIP device) runs BezierMesh::intersect,
// BezierTriangle::intersect and BezierLens::refract through libbzr and checks them bit-for-bit against
// the oracle (test infrastructure, linked only into this test program).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "3dGeomUtil.h"
#include "bezierLens.h"
#include "bezierMesh.h"
#include "mesh.h"
#include "hostUtil.h"
#include "bzr_oracle.h"

static int g_fail = 0, g_checks = 0;
#define CHECK(cond)                                                          \
  do {                                                                       \
    ++g_checks;                                                              \
    if (!(cond)) {                                                           \
      ++g_fail;                                                              \
      std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
    }                                                                        \
  } while (0)

constexpr float cgEpsilon = 0.0001f;
static bool eq(Vector const &a, Vector const &b) { return (a - b).norm() < cgEpsilon; }

static Vertex planesNormals(Vertex p, Vector d1, Vector d2, Vector d3) {
  Vector n1 = d1.normalized(), n2 = d2.normalized(), n3 = d3.normalized();
  return Plane::intersect(Plane(n1, n1.dot(p)), Plane(n2, n2.dot(p)), Plane(n3, n3.dot(p)));
}

static void l1_geometry() {
  // vector.getAperpendicular
  for (Vector v : {Vector{1, 0, 0}, Vector{1, 1, 0}, Vector{1, 0, 1}, Vector{1, -1, -1}}) {
    v.normalize();
    CHECK(std::fabs(util::getAperpendicular(v).dot(v)) < 1e-6f);
  }
  // ray.averageErrorSquared
  Ray ray({0.0f, 0.0f, 0.0f}, {1.0f, 0.0f, 0.0f});
  CHECK(ray.getAverageErrorSquared({}) == 0.0f);
  CHECK(ray.getAverageErrorSquared({{2.0f, 0.0f, 0.0f}, {-3.0f, 0.0f, 0.0f}}) == 0.0f);
  CHECK(ray.getAverageErrorSquared({{2.0f, 1.0f, 0.0f}, {-3.0f, 0.0f, 1.0f}}) > 0.0f);
  // planeIntersection.Normals
  CHECK(eq(planesNormals({1, 2, 3}, {1, 2, 3}, {3, 1, 2}, {3, 2, 1}), Vertex{1, 2, 3}));
  CHECK(eq(planesNormals({3, -2, 1}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}), Vertex{3, -2, 1}));
  CHECK(eq(planesNormals({3, -2, -1}, {1, -2, 3}, {-1, 2, 3}, {1, 2, -3}), Vertex{3, -2, -1}));
  // planeIntersection.Proportion
  auto prop = [](Vertex c, float p1, Vertex o1, float p2, Vertex o2, float p3, Vertex o3) {
    return Plane::intersect(Plane::createFrom1proportion2points(p1, o1, o1 + 1.0f / p1 * (c - o1)),
                            Plane::createFrom1proportion2points(p2, o2, o2 + 1.0f / p2 * (c - o2)),
                            Plane::createFrom1proportion2points(p3, o3, o3 + 1.0f / p3 * (c - o3)));
  };
  CHECK(eq(prop({0, 0, 0}, 0.5f, {1, 0, 0}, 0.2f, {0, 1, 0}, 0.1f, {0, 0, 1}), Vertex{0, 0, 0}));
  CHECK(eq(prop({-1, 2, 3}, 0.1f, {10, 10, 0}, 0.2f, {0, -10, 10}, 0.3f, {-10, 0, 10}), Vertex{-1, 2, 3}));
  // planeIntersection.Vertices
  Vertex common{1, 2, 3};
  for (auto o : {std::array<Vertex, 3>{Vertex{10, 0, 0}, Vertex{0, 10, 0}, Vertex{0, 0, 10}},
                 std::array<Vertex, 3>{Vertex{-10, 0, 0}, Vertex{0, -10, 0}, Vertex{0, 0, -10}}}) {
    CHECK(eq(Plane::intersect(Plane::createFrom3points(o[0], o[1], common), Plane::createFrom3points(o[1], o[2], common),
                              Plane::createFrom3points(o[0], o[2], common)),
             common));
  }
  // planeIntersection.VectorPoints
  Vertex c2{1, 2, -3};
  CHECK(eq(Plane::intersect(Plane::createFrom1vector2points({-4, 1, 1}, {10, 0, 0}, c2),
                            Plane::createFrom1vector2points({1, -4, -1}, {0, 10, 0}, c2),
                            Plane::createFrom1vector2points({1, 1, -4}, {0, 0, 10}, c2)),
           c2));
  // planeIntersection.Ray (second case: deviation D1 -- mValid false, negative distance reported)
  {
    Ray r(Vertex{1, 2, -3}, Vector{1, 1, 1});
    Plane p = Plane::createFrom3points(Vertex{10, 1, 2}, Vertex{11, 11.1f, 2}, Vertex{12, 1.1f, 4.4f});
    CHECK(p.intersect(r).mValid);
    Ray r2(Vertex{1, 2, -3}, Vector{-1, 2, 3});
    auto i2 = p.intersect(r2);
    CHECK(!i2.mValid && i2.mDistance < 0.0f);
    Ray r3(Vertex{1, 2, -3}, Vector{0, 2, 0});
    Plane p3 = Plane::createFrom3points(Vertex{10, 10, 2}, Vertex{0, 10, 2}, Vertex{10, 10, 10.4f});
    auto i3 = p3.intersect(r3);
    CHECK(i3.mValid && (i3.mPoint - Vertex{1, 10, -3}).norm() < 0.00001f && std::fabs(i3.mCosIncidence) > 0.9999f);
  }
  // planeProjection.Point / planeDistance.Point
  Plane pp = Plane::createFrom3points({3, 2, 3}, {1, 4, 3}, {1, 2, 5});
  CHECK(eq(pp.project({1, 2, 3}), Vertex(1.666666f, 2.666666f, 3.666666f)));
  CHECK(std::fabs(std::fabs(pp.distance({1, 2, 3})) - 1.15468f) < cgEpsilon);
  // toWhichSide.Points
  Vertex t0{3, 2, 5}, t1{1, 4, 5}, t2{6, 5, 5};
  Vertex start = (t0 + t1 + t2) / 3.0f;
  Matrix conv = util::getBarycentricInverse(t0, t1, t2);
  CHECK(util::toWhichSide(conv * start, conv * (start + Vector{1, 0, 0})) == 2u);
  CHECK(util::toWhichSide(conv * start, conv * (start + Vector{0, 1, 0})) == 1u);
  CHECK(util::toWhichSide(conv * start, conv * (start + Vector{-1, -1, 0})) == 0u);
  // Eigen-surface idioms used by reference callers
  Vertex v;
  v << -1.0f, 0.0f, 0.0f;
  CHECK(v(0) == -1.0f && v[1] == 0.0f);
  Transform shrink = Transform::Identity() * 0.5f;
  CHECK(eq(shrink * Vertex{2, 4, 6}, Vertex{1, 2, 3}));
  CHECK(Vertex::Zero() == Vertex(0, 0, 0));
  CHECK(eq(Vertex{{1.0f, 2.0f, 3.0f}}, Vertex(1, 2, 3)));
}

static void preprocessing(Mesh &lens) {
  lens.makeEllipsoid(32, 16, Vector(1.0f, 4.0f, 2.0f));
  CHECK(lens.size() == 1024u);
  lens += Vector{10.0f, 0.0f, 0.0f};
  lens.standardizeVertices();
  lens.standardizeNormals();
  CHECK(lens.getFace2neighbours().size() == 1024u);
  CHECK(lens.getVertex2averageNormals().size() == 514u);  // 514 vertices
  CHECK(lens.getVertices().size() == 514u);
  BezierMesh bezier(lens);
  CHECK(bezier.size() == 3072u);
  CHECK(bezier.dumpControlPoints().size() == 30720u);
  Mesh tess = bezier.interpolate(2);
  CHECK(tess.size() == 4u * 3072u);
  Mesh thick = bezier.splitThickBezierTriangles();
  CHECK(thick.size() >= lens.size());
  // parity of the drop-in's construction with the oracle's
  omesh om;
  orc_mesh_init(&om);
  orc_mesh_make_ellipsoid(&om, 32, 16, ov3{1.0f, 4.0f, 2.0f});
  float id[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  orc_mesh_transform(&om, id, ov3{10.0f, 0.0f, 0.0f});
  orc_mesh_standardize_vertices(&om);
  CHECK(orc_mesh_standardize_normals(&om) == 0);
  std::vector<opatch> op(om.n * 3);
  CHECK(orc_bezier_build(&om, op.data()) == 0);
  CHECK(std::memcmp(op.data(), &bezier[0], sizeof(opatch) * op.size()) == 0);
  orc_mesh_free(&om);
}

static void hot_path(Mesh const &lensMesh) {
  BezierMesh bezier(lensMesh);
  std::vector<opatch> op(bezier.size());
  std::memcpy(op.data(), &bezier[0], sizeof(opatch) * op.size());
  BezierLens lens(1.3f, bezier);
  // a small image, single-ray calls like reference/test.cpp:376-401, and the batch overloads
  std::vector<Ray> rays;
  for (int i = 0; i < 24; ++i)
    for (int j = 0; j < 24; ++j)
      rays.emplace_back(Vertex{0.0f, -4.2f + 8.4f * (j + 0.5f) / 24, -2.1f + 4.2f * (i + 0.5f) / 24}, Vector{1, 0, 0});
  int hits = 0, exits = 0;
  std::vector<BezierIntersection> batch(rays.size());
  std::vector<uint32_t> patch(rays.size());
  bezier.intersect(rays.data(), rays.size(), batch.data(), patch.data());
  for (std::size_t r = 0; r < rays.size(); ++r) {
    oray orr{ov3{rays[r].mStart(0), rays[r].mStart(1), rays[r].mStart(2)},
             ov3{rays[r].mDirection(0), rays[r].mDirection(1), rays[r].mDirection(2)}};
    ohit want = orc_mesh_intersect(op.data(), op.size(), &orr);
    BezierIntersection got = r % 37 == 0 ? bezier.intersect(rays[r]) : batch[r];
    CHECK(static_cast<uint32_t>(got.mWhat) == want.what);
    if (want.what == ORC_INTERSECT) {
      ++hits;
      CHECK(patch[r] == want.patch);
      CHECK(std::memcmp(&got.mIntersection.mDistance, &want.t, 4) == 0);
      CHECK(std::memcmp(got.mBarycentric.data(), &want.bary, 12) == 0);
      CHECK(std::memcmp(got.mNormal.data(), &want.normal, 12) == 0);
      // the single-patch API gives the same hit for the winning patch
      BezierIntersection one = bezier[patch[r]].intersect(rays[r], BezierTriangle::LimitPlaneIntersection::cNone);
      CHECK(one.mWhat == BezierIntersection::What::cIntersect);
    }
    Ray cur = rays[r];
    RefractionResult st = RefractionResult::cNone;
    for (uint32_t j = 0; j < 2u; ++j) {
      RefractionResult expect = j == 0 ? RefractionResult::cInside : RefractionResult::cOutside;
      auto res = lens.refract(cur, expect);
      oray oo;
      uint32_t ost = orc_lens_refract(op.data(), op.size(), 1.3f, &orr, static_cast<uint32_t>(expect), &oo);
      CHECK(static_cast<uint32_t>(res.second) == ost);
      st = res.second;
      if (st == RefractionResult::cNone) break;
      CHECK(std::memcmp(res.first.mDirection.data(), &oo.dir, 12) == 0);
      cur = res.first;
      orr = oo;
    }
    exits += st == RefractionResult::cOutside;
  }
  CHECK(hits > 150 && exits > 100);
  // the whole chain in one call
  std::vector<Ray> out(rays.size());
  std::vector<RefractionResult> status(rays.size());
  std::vector<uint32_t> seg(rays.size());
  bzr::traceChain({&lens}, rays.data(), rays.size(), out.data(), status.data(), seg.data());
  int chainExits = 0;
  for (auto s : status) chainExits += s == RefractionResult::cOutside;
  CHECK(chainExits == exits);
  // the same chain dealt over two contexts (two streams / host threads on device 0), tiles of 100 rays
  bzr::Context c0(0), c1(0);
  std::vector<Ray> outT(rays.size());
  std::vector<RefractionResult> statusT(rays.size());
  std::vector<uint32_t> segT(rays.size());
  bzr::traceChainTiled({&c0, &c1}, {&lens}, rays.data(), rays.size(), outT.data(), statusT.data(), segT.data(), 100);
  CHECK(statusT == status && segT == seg);
  CHECK(std::memcmp(outT.data(), out.data(), out.size() * sizeof(Ray)) == 0);
  std::printf("hot path: %d hits, %d exits of %zu rays\n", hits, exits, rays.size());
}

// UniformHemisphere (reference/hostUtil.cpp) through the drop-in header vs the oracle's restatement of
// the same std::ranlux24_base stream: patch counts and the first 5000 draws, bit for bit.
static void hemisphere() {
  for (uint32_t belts : {1u, 3u, 8u, 16u}) {
    UniformHemisphere h(belts);
    orc_hemisphere *o = orc_hemisphere_create(belts);
    CHECK(h.getPatchCount() == orc_hemisphere_patch_count(o));
    int same = 0;
    for (int k = 0; k < 5000; ++k) {
      auto [d, idx] = h.getRandom();
      float od[3];
      uint32_t oidx = orc_hemisphere_random(o, od);
      same += std::memcmp(&d(0), &od[0], 4) == 0 && std::memcmp(&d(1), &od[1], 4) == 0 &&
              std::memcmp(&d(2), &od[2], 4) == 0 && idx == oidx && idx < h.getPatchCount();
    }
    CHECK(same == 5000);
    orc_hemisphere_free(o);
  }
}

int main() {
  hemisphere();
  l1_geometry();
  Mesh lens;
  preprocessing(lens);
  int32_t devices = 0;
  bzr_device_count(&devices);
  if (devices > 0) hot_path(lens);
  else std::printf("no HIP device: hot-path part skipped\n");
  std::printf("%d checks, %d failed\n", g_checks, g_fail);
  return g_fail ? 1 : 0;
}
