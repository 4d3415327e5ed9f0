// dropin_test.cpp -- a reference-style caller compiled against the drop-in headers.
//
// It includes the reference's header names (include/bzr/*.h) and uses the reference's API the way
// reference/test.cpp and reference/googleTest.cpp do.  Part 1 restates the googleTest L1 cases
// (reference/googleTest.cpp:46-353, cgEpsilon = 1e-4) on the product's value types; part 2 runs the
// host preprocessing API; part 3 runs the single-ray BezierMesh::intersect, BezierTriangle::intersect and
// BezierLens::refract (host arithmetic of the product, single_ray.cpp) against the oracle (test
// infrastructure, linked only into this test program); part 4 (only with a HIP device) runs the batch
// overloads, the chain and the multi-device calls through libbzr and checks them bit-for-bit against the
// single-ray results and the oracle, and times one ray through each path.
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <thread>
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

static bool same_hit(BezierIntersection const &a, BezierIntersection const &b) {
  return a.mWhat == b.mWhat && a.mIntersection.mValid == b.mIntersection.mValid &&
         std::memcmp(&a.mIntersection.mDistance, &b.mIntersection.mDistance, 4) == 0 &&
         std::memcmp(&a.mIntersection.mCosIncidence, &b.mIntersection.mCosIncidence, 4) == 0 &&
         std::memcmp(a.mIntersection.mPoint.data(), b.mIntersection.mPoint.data(), 12) == 0 &&
         std::memcmp(a.mBarycentric.data(), b.mBarycentric.data(), 12) == 0 &&
         std::memcmp(a.mNormal.data(), b.mNormal.data(), 12) == 0;
}
static bool same_ray(Ray const &a, Ray const &b) {
  return std::memcmp(a.mStart.data(), b.mStart.data(), 12) == 0 && std::memcmp(a.mDirection.data(), b.mDirection.data(), 12) == 0;
}

// cfg2's primary rays: plane x = 0, y in [-4.2, 4.2], z in [-2.1, 2.1], along +x
static std::vector<Ray> cfg2_rays(int side) {
  std::vector<Ray> rays;
  for (int i = 0; i < side; ++i)
    for (int j = 0; j < side; ++j)
      rays.emplace_back(Vertex{0.0f, -4.2f + 8.4f * (j + 0.5f) / side, -2.1f + 4.2f * (i + 0.5f) / side}, Vector{1, 0, 0});
  return rays;
}

template <typename F>
static double us_per_call(F &&f, int calls) {
  auto t0 = std::chrono::steady_clock::now();
  for (int k = 0; k < calls; ++k) f(k);
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / calls;
}

// Part 3: the reference's single-ray calls (reference/test.cpp:268,281,380), on the host, vs the oracle.
static void single_ray(Mesh const &lensMesh) {
  BezierMesh bezier(lensMesh);
  std::vector<opatch> op(bezier.size());
  std::memcpy(op.data(), &bezier[0], sizeof(opatch) * op.size());
  BezierLens lens(1.3f, bezier);
  std::vector<Ray> rays = cfg2_rays(24);
  int hits = 0, exits = 0;
  for (std::size_t r = 0; r < rays.size(); ++r) {
    oray orr{ov3{rays[r].mStart(0), rays[r].mStart(1), rays[r].mStart(2)},
             ov3{rays[r].mDirection(0), rays[r].mDirection(1), rays[r].mDirection(2)}};
    ohit want = orc_mesh_intersect(op.data(), op.size(), &orr);
    BezierIntersection got = bezier.intersect(rays[r]);
    CHECK(static_cast<uint32_t>(got.mWhat) == want.what);
    if (want.what == ORC_INTERSECT) {
      ++hits;
      CHECK(std::memcmp(&got.mIntersection.mDistance, &want.t, 4) == 0);
      CHECK(std::memcmp(got.mBarycentric.data(), &want.bary, 12) == 0);
      CHECK(std::memcmp(got.mNormal.data(), &want.normal, 12) == 0);
      // the single-patch API gives the same hit for the winning patch
      BezierIntersection one = bezier[want.patch].intersect(rays[r], BezierTriangle::LimitPlaneIntersection::cNone);
      CHECK(one.mWhat == BezierIntersection::What::cIntersect);
      CHECK(std::memcmp(&one.mIntersection.mDistance, &want.t, 4) == 0);
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
      CHECK(std::memcmp(res.first.mStart.data(), &oo.start, 12) == 0);
      CHECK(std::memcmp(res.first.mDirection.data(), &oo.dir, 12) == 0);
      cur = res.first;
      orr = oo;
    }
    exits += st == RefractionResult::cOutside;
  }
  CHECK(hits > 150 && exits > 100);
  std::printf("single ray (host): %d hits, %d exits of %zu rays\n", hits, exits, rays.size());
}

// Part 4: the GPU batch paths vs the host single-ray path, bit for bit, and the per-call latency of both.
static void hot_path(Mesh const &lensMesh) {
  BezierMesh bezier(lensMesh);
  BezierLens lens(1.3f, bezier);
  std::vector<Ray> rays = cfg2_rays(64);
  const std::size_t n = rays.size();
  // BezierMesh::intersect: GPU batch == host single ray, every field and the patch index
  std::vector<BezierIntersection> batch(n);
  std::vector<uint32_t> patch(n);
  bezier.intersect(rays.data(), n, batch.data(), patch.data());
  int hits = 0, same = 0;
  for (std::size_t r = 0; r < n; ++r) {
    uint32_t hp = 0;
    BezierIntersection one = bezier.intersect(rays[r], &hp);
    same += same_hit(one, batch[r]) && hp == patch[r];
    hits += batch[r].mWhat == BezierIntersection::What::cIntersect;
  }
  CHECK(same == static_cast<int>(n));
  CHECK(hits > 1000);
  // BezierTriangle::intersect: host vs bzr_patch_intersect, both limits, for every ray's winning (or first) patch
  {
    std::vector<uint32_t> idx(n), lim(n);
    std::vector<float> soa(6 * n), h(13 * n);
    for (std::size_t r = 0; r < n; ++r) {
      idx[r] = patch[r] == 0xFFFFFFFFu ? static_cast<uint32_t>(r % bezier.size()) : patch[r];
      lim[r] = static_cast<uint32_t>(r & 1u);
      for (int k = 0; k < 3; ++k) {
        soa[k * n + r] = rays[r].mStart(k);
        soa[(3 + k) * n + r] = rays[r].mDirection(k);
      }
    }
    bzr::Context &c = bzr::defaultContext();
    bzr::check(bzr_patch_intersect(c.get(), bezier.device(c), idx.data(), lim.data(), soa.data(), static_cast<uint32_t>(n),
                                   h.data(), BZR_HOST_PTRS));
    int agree = 0;
    for (std::size_t r = 0; r < n; ++r) {
      BezierIntersection one = bezier[idx[r]].intersect(rays[r], static_cast<BezierTriangle::LimitPlaneIntersection>(lim[r]));
      uint32_t what;
      std::memcpy(&what, &h[11 * n + r], 4);
      agree += static_cast<uint32_t>(one.mWhat) == what && std::memcmp(&one.mIntersection.mDistance, &h[r], 4) == 0 &&
               std::memcmp(one.mBarycentric.data(), &h[5 * n + r], 4) == 0 &&
               std::memcmp(one.mBarycentric.data() + 1, &h[6 * n + r], 4) == 0 &&
               std::memcmp(one.mBarycentric.data() + 2, &h[7 * n + r], 4) == 0 &&
               std::memcmp(one.mNormal.data(), &h[8 * n + r], 4) == 0;
    }
    CHECK(agree == static_cast<int>(n));
  }
  // BezierLens::refract: GPU batch == host single ray (both steps of the chain)
  std::vector<Ray> cur = rays, next(n);
  std::vector<RefractionResult> expect(n, RefractionResult::cInside), st(n);
  int refr_same = 0, exits = 0;
  for (uint32_t j = 0; j < 2u; ++j) {
    std::fill(expect.begin(), expect.end(), j == 0 ? RefractionResult::cInside : RefractionResult::cOutside);
    lens.refract(cur.data(), expect.data(), n, next.data(), st.data());
    for (std::size_t r = 0; r < n; ++r) {
      auto one = lens.refract(cur[r], expect[r]);
      refr_same += one.second == st[r] && same_ray(one.first, next[r]);
      if (j == 1) exits += st[r] == RefractionResult::cOutside;
    }
    cur = next;
  }
  CHECK(refr_same == static_cast<int>(2 * n));
  // the whole chain in one call
  std::vector<Ray> out(n);
  std::vector<RefractionResult> status(n);
  std::vector<uint32_t> seg(n);
  bzr::traceChain({&lens}, rays.data(), n, out.data(), status.data(), seg.data());
  int chainExits = 0;
  for (auto s : status) chainExits += s == RefractionResult::cOutside;
  CHECK(chainExits > 0);
  // four host threads sharing the default context, each calling the batch overloads three times: the context's
  // lock serialises them (its staging buffers are per context), every result equals the sequential one
  {
    std::atomic<int> agree{0};
    std::vector<std::thread> pool;
    for (int k = 0; k < 4; ++k)
      pool.emplace_back([&] {
        for (int rep = 0; rep < 3; ++rep) {
          std::vector<Ray> o(n);
          std::vector<RefractionResult> so(n);
          std::vector<uint32_t> sg(n);
          bzr::traceChain({&lens}, rays.data(), n, o.data(), so.data(), sg.data());
          std::vector<BezierIntersection> hb(n);
          std::vector<uint32_t> hp(n);
          bezier.intersect(rays.data(), n, hb.data(), hp.data());
          bool same = so == status && sg == seg && std::memcmp(o.data(), out.data(), n * sizeof(Ray)) == 0 && hp == patch;
          for (std::size_t r = 0; r < n && same; ++r) same = same_hit(hb[r], batch[r]);
          agree += same ? 1 : 0;
        }
      });
    for (auto &t : pool) t.join();
    CHECK(agree == 12);
  }
  // the same chain dealt over two contexts on device 0, gathered on the device (peer path), tiles of 100 rays
  bzr::Context c0(0), c1(0);
  std::vector<Ray> outT(n);
  std::vector<RefractionResult> statusT(n);
  std::vector<uint32_t> segT(n);
  bzr::traceChainTiled({&c0, &c1}, {&lens}, rays.data(), n, outT.data(), statusT.data(), segT.data(), 100);
  CHECK(statusT == status && segT == seg);
  CHECK(std::memcmp(outT.data(), out.data(), out.size() * sizeof(Ray)) == 0);
  // frame after frame: a TiledChain plan, 2 slots x 2 contexts on device 0, host outputs
  {
    bzr::Context s00(0), s01(0), s10(0), s11(0);
    bzr::TiledChain frames({{&s00, &s01}, {&s10, &s11}}, {&lens}, n, 512);
    CHECK(frames.transport() == BZR_GATHER_PEER);
    frames.setRays(rays.data());
    for (int k = 0; k < 4; ++k) {
      if (k == 2) CHECK(frames.calibrate() > 0u);  // the last two frames gather only the refracted rays
      std::vector<Ray> o(n);
      std::vector<RefractionResult> so(n);
      std::vector<uint32_t> sg(n);
      frames.trace(o.data(), so.data(), sg.data());
      CHECK(so == status && sg == seg);
      CHECK(std::memcmp(o.data(), out.data(), out.size() * sizeof(Ray)) == 0);
    }
  }
  // one context: the DIRECT plan (AUTO's choice for one device), while another thread runs batch chains on the
  // same context (every TiledChain member takes its contexts' locks, as the batch calls do)
  {
    bzr::Context sd(0);
    bzr::TiledChain one({{&sd}}, {&lens}, n, 512);
    CHECK(one.transport() == BZR_GATHER_DIRECT);
    one.setRays(rays.data());
    std::atomic<int> side_ok{0};
    std::thread side([&] {
      for (int k = 0; k < 3; ++k) {
        std::vector<Ray> o(n);
        std::vector<RefractionResult> so(n);
        std::vector<uint32_t> sg(n);
        bzr::traceChain({&lens}, rays.data(), n, o.data(), so.data(), sg.data(), &sd);
        side_ok += (so == status && sg == seg && std::memcmp(o.data(), out.data(), n * sizeof(Ray)) == 0) ? 1 : 0;
      }
    });
    for (int k = 0; k < 3; ++k) {
      std::vector<Ray> o(n);
      std::vector<RefractionResult> so(n);
      std::vector<uint32_t> sg(n);
      one.trace(o.data(), so.data(), sg.data());
      CHECK(so == status && sg == seg);
      CHECK(std::memcmp(o.data(), out.data(), out.size() * sizeof(Ray)) == 0);
    }
    side.join();
    CHECK(side_ok == 3);
  }
  // per-call latency of one ray: host single-ray methods vs the GPU batch of one (launch + PCIe + sync)
  const int calls = 200;
  BezierIntersection sink;
  double host_mesh = us_per_call([&](int k) { sink = bezier.intersect(rays[(k * 97) % n]); }, calls);
  double gpu_mesh = us_per_call([&](int k) { bezier.intersect(&rays[(k * 97) % n], 1, &sink); }, calls);
  double host_patch = us_per_call([&](int k) {
    sink = bezier[patch[(k * 97) % n] % bezier.size()].intersect(rays[(k * 97) % n], BezierTriangle::LimitPlaneIntersection::cThis);
  }, calls);
  std::pair<Ray, RefractionResult> rsink;
  double host_refr = us_per_call([&](int k) { rsink = lens.refract(rays[(k * 97) % n], RefractionResult::cInside); }, calls);
  RefractionResult e1 = RefractionResult::cInside, s1;
  Ray o1;
  double gpu_refr = us_per_call([&](int k) { lens.refract(&rays[(k * 97) % n], &e1, 1, &o1, &s1); }, calls);
  std::printf("latency us/call (cfg2 lens, %zu patches): BezierMesh::intersect host %.2f gpu-batch-of-1 %.2f; "
              "BezierTriangle::intersect host %.3f; BezierLens::refract host %.2f gpu-batch-of-1 %.2f\n",
              bezier.size(), host_mesh, gpu_mesh, host_patch, host_refr, gpu_refr);
  std::printf("hot path: %d hits, %d exits of %zu rays (GPU batch == host single ray)\n", hits, exits, n);
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
  single_ray(lens);
  if (devices > 0) hot_path(lens);
  else std::printf("no HIP device: hot-path part skipped\n");
  std::printf("%d checks, %d failed\n", g_checks, g_fail);
  return g_fail ? 1 : 0;
}
