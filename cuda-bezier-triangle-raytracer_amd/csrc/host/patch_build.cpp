// patch_build.cpp -- host construction of the cubic Bezier patches (Clough-Tocher
// split) and the BezierMesh tools that work on patch records.
//   BezierTriangle ctor / setMissingFields1-3 : reference/bezierTriangle.cpp:4-97
//   interpolate / interpolateLinear / getNormal: reference/bezierTriangle.cpp:99-121, 197-233
//   BezierMesh ctor, interpolate, dumpControlPoints, splitThickBezierTriangles:
//                                               reference/bezierMesh.cpp:4-204
// These run once per mesh on the host; the per-ray work is in csrc/device/.
#include <algorithm>

#include "bzr/bzr.hpp"

namespace {
// control point slots (reference/bezierTriangle.h:31-51): ijk = exponents of (b0, b1, b2)
enum : uint32_t { c300 = 0, c030 = 1, c003 = 2, c210 = 3, c120 = 4, c021 = 5, c012 = 6, c102 = 7, c201 = 8, c111 = 9 };

constexpr float kSideProportion = 0.291f;      // csProportionControlOnOriginalSide
constexpr float kCentroidProportion = 0.304f;  // csProportionControlOnOriginalVertexCentroid
constexpr float kMedianProportion = 0.2f;      // csProportionControlOnOriginalMedian
constexpr float kHeightSafety = 1.33333333f;   // csHeightSafetyFactor
constexpr int32_t kHeightSamples = 5;          // csHeightSampleDivisor
constexpr float kSplitBlend = 0.7f;            // BezierMesh::csSplitBezierInterpolateFactor
constexpr float kThickLimit = 0.03f;           // csBezierHeightPerPerimeterLimit

Triangle const kUnitBary{Vertex(1.0f, 0.0f, 0.0f), Vertex(0.0f, 1.0f, 0.0f), Vertex(0.0f, 0.0f, 1.0f)};
}  // namespace

BezierTriangle::BezierTriangle(Vertex const &v0, Vertex const &v1, Vertex const &centroid, Vector const &n0,
                               Vector const &n1, Plane const &between, std::array<uint32_t, 3u> const &neighbours)
    : mNeighbours(neighbours) {
  auto &cp = mControlPoints;
  cp[c300] = v0;
  cp[c030] = v1;
  // tangent planes at the two shared corners fix C1 continuity across the original edge
  Plane const tangent0{n0, v0.dot(n0)};
  Plane const tangent1{n1, v1.dot(n1)};
  cp[c210] = Plane::intersect(tangent0, between, Plane::createFrom1proportion2points(kSideProportion, v0, v1));
  cp[c120] = Plane::intersect(tangent1, between, Plane::createFrom1proportion2points(kSideProportion, v1, v0));

  Vector const faceNormal = util::getNormal(v0, v1, centroid);
  cp[c201] = Plane::intersect(tangent0, Plane::createFrom1vector2points(faceNormal, v0, centroid),
                              Plane::createFrom1proportion2points(kCentroidProportion, v0, centroid));
  cp[c021] = Plane::intersect(tangent1, Plane::createFrom1vector2points(faceNormal, v1, centroid),
                              Plane::createFrom1proportion2points(kCentroidProportion, v1, centroid));

  cp[c111] = Plane::intersect(Plane::createFrom1vector2points(between.mNormal, cp[c210], cp[c120]),
                              Plane::createFrom1proportion2points(0.5f, cp[c210], cp[c120]),
                              Plane::createFrom1proportion2points(kMedianProportion, (v0 + v1) / 2.0f, centroid));
  mNeighbourDividerPlanes[0] = between;
  mNeighbourDividerPlanes[0].makeDistancePositive(cp[c111]);
}

void BezierTriangle::setMissingFields1(Vertex const &centroid, BezierTriangle const &next, BezierTriangle const &previous) {
  auto &cp = mControlPoints;
  Vector const faceNormal = util::getNormal(cp[c300], cp[c030], centroid);
  Plane const across0 = Plane::createFrom3points(cp[c201], cp[c111], previous.mControlPoints[c111]);
  Plane const across1 = Plane::createFrom3points(cp[c021], next.mControlPoints[c111], cp[c111]);
  cp[c102] = Plane::intersect(across0, Plane::createFrom1vector2points(faceNormal, cp[c300], centroid),
                              Plane::createFrom1proportion2points(kCentroidProportion, centroid, cp[c300]));
  cp[c012] = Plane::intersect(across1, Plane::createFrom1vector2points(faceNormal, cp[c030], centroid),
                              Plane::createFrom1proportion2points(kCentroidProportion, centroid, cp[c030]));
}

void BezierTriangle::setMissingFields2(Vertex const &, BezierTriangle const &next, BezierTriangle const &) {
  auto &cp = mControlPoints;
  cp[c003] = (cp[c102] + cp[c012] + next.mControlPoints[c012]) / 3.0f;
  mUnderlyingPlane = Plane::createFrom3points(cp[c300], cp[c030], cp[c003]);
  mBarycentricInverse = util::getBarycentricInverse(cp[c300], cp[c030], cp[c003]);
  // dome heights sampled on a 5-division barycentric grid, then inflated
  float lowest = 0.0f, highest = 0.0f;
  util::divide(kUnitBary, kHeightSamples, [&](Triangle &&sample) {
    for (auto const &b : sample) {
      float h = mUnderlyingPlane.distance(interpolate(b));
      lowest = std::min(lowest, h);
      highest = std::max(highest, h);
    }
  });
  mHeightInside = lowest * kHeightSafety;
  mHeightOutside = highest * kHeightSafety;
  mBezierDerivativeDirectionVectorA = Vertex(1.0f, 0.0f, -1.0f);
  mBezierDerivativeDirectionVectorB = mBarycentricInverse * (cp[c003] - cp[c300]).cross(mUnderlyingPlane.mNormal);
}

void BezierTriangle::setMissingFields3(Vertex const &, BezierTriangle const &next, BezierTriangle const &previous) {
  auto const &cp = mControlPoints;
  mNeighbourDividerPlanes[1] = Plane::createFrom1vector2points(mUnderlyingPlane.mNormal + next.mUnderlyingPlane.mNormal,
                                                               cp[c030], cp[c003]);
  mNeighbourDividerPlanes[2] = Plane::createFrom1vector2points(mUnderlyingPlane.mNormal + previous.mUnderlyingPlane.mNormal,
                                                               cp[c300], cp[c003]);
  mNeighbourDividerPlanes[1].makeDistancePositive(cp[c111]);
  mNeighbourDividerPlanes[2].makeDistancePositive(cp[c111]);
}

Vertex BezierTriangle::interpolateLinear(float b0, float b1, float b2) const {
  return mControlPoints[c300] * b0 + mControlPoints[c030] * b1 + mControlPoints[c003] * b2;
}

Vertex BezierTriangle::interpolate(float b0, float b1, float b2) const {
  auto const &cp = mControlPoints;
  float const s0 = b0 * b0, s1 = b1 * b1, s2 = b2 * b2;
  Vertex const corners = cp[c300] * b0 * s0 + cp[c030] * b1 * s1 + cp[c003] * b2 * s2;
  Vertex const edges = cp[c210] * b1 * s0 + cp[c120] * b0 * s1 + cp[c021] * b2 * s1 + cp[c012] * b1 * s2 +
                       cp[c102] * b0 * s2 + cp[c201] * b2 * s0;
  return corners + 3.0f * edges + cp[c111] * b0 * b1 * b2 * 6.0f;
}

Vector BezierTriangle::getNormal(Vector const &b) const {
  auto const &cp = mControlPoints;
  float const s0 = b(0) * b(0), s1 = b(1) * b(1), s2 = b(2) * b(2);
  // the three quadratic partial-derivative nets
  Vector const d0 = cp[c300] * s0 + cp[c102] * s2 + cp[c120] * s1 +
                    2.0f * (cp[c201] * b(0) * b(2) + cp[c210] * b(0) * b(1) + cp[c111] * b(2) * b(1));
  Vector const d1 = cp[c030] * s1 + cp[c012] * s2 + cp[c210] * s0 +
                    2.0f * (cp[c111] * b(0) * b(2) + cp[c120] * b(0) * b(1) + cp[c021] * b(1) * b(2));
  Vector const d2 = cp[c003] * s2 + cp[c201] * s0 + cp[c021] * s1 +
                    2.0f * (cp[c102] * b(0) * b(2) + cp[c012] * b(1) * b(2) + cp[c111] * b(0) * b(1));
  Vector const &A = mBezierDerivativeDirectionVectorA;
  Vector const &B = mBezierDerivativeDirectionVectorB;
  Vector const alongA = A(0) * d0 + A(1) * d1 + A(2) * d2;
  Vector const alongB = B(0) * d0 + B(1) * d1 + B(2) * d2;
  return alongA.cross(alongB).normalized();
}

// ---------------------------------------------------------------- BezierMesh
BezierMesh::BezierMesh(std::vector<BezierTriangle> patches, Mesh::Face2neighbours originalNeighbours)
    : mMesh(std::move(patches)), mOriginalNeighbours(std::move(originalNeighbours)) {}

BezierMesh::BezierMesh(Mesh const &mesh) : mOriginalNeighbours(mesh.getFace2neighbours()) {
  if (mOriginalNeighbours.size() != mesh.size()) throw std::runtime_error("BezierMesh: mesh is not standardized");
  auto const &normals = mesh.getVertex2averageNormals();
  mMesh.reserve(mesh.size() * 3u);
  for (uint32_t f = 0; f < mesh.size(); ++f) {
    auto const &adj = mOriginalNeighbours[f];
    Triangle const &t = mesh[f];
    Vertex const centroid = (t[0] + t[1] + t[2]) / 3.0f;
    Vector const normal = util::getNormal(t).normalized();
    for (uint32_t k = 0; k < 3u; ++k) {  // Clough-Tocher: sub-triangle k spans edge (k, k+1) and the centroid
      Vertex const &a = t[k];
      Vertex const &b = t[(k + 1u) % 3u];
      Plane const between = Plane::createFrom1vector2points(
          normal + util::getNormal(mesh[adj.mFellowTriangles[k]]).normalized(), a, b);
      uint32_t const base = f * 3u;
      std::array<uint32_t, 3u> const links{3u * adj.mFellowTriangles[k] + adj.mFellowCommonSideStarts[k],
                                           base + (k + 1u) % 3u, base + (k + 2u) % 3u};
      mMesh.emplace_back(a, b, centroid, normals.at(a), normals.at(b), between, links);
    }
  }
  // three passes: each reads fields of the neighbouring sub-triangles set by the previous pass
  for (int pass = 1; pass <= 3; ++pass) {
    Vertex centroid = Vertex::Zero();
    for (uint32_t i = 0; i < mMesh.size(); ++i) {
      uint32_t const sub = i % 3u, base = i - sub;
      BezierTriangle const &next = mMesh[base + (sub + 1u) % 3u];
      BezierTriangle const &prev = mMesh[base + (sub + 2u) % 3u];
      if (sub == 0u) {
        Triangle const &t = mesh[base / 3u];
        centroid = (t[0] + t[1] + t[2]) / 3.0f;
      }
      if (pass == 1) mMesh[i].setMissingFields1(centroid, next, prev);
      else if (pass == 2) mMesh[i].setMissingFields2(centroid, next, prev);
      else mMesh[i].setMissingFields3(centroid, next, prev);
    }
  }
}

Mesh BezierMesh::interpolate(int32_t divisor) const {  // reference/bezierMesh.cpp:55-66
  Mesh out;
  util::divide(kUnitBary, divisor, [&](Triangle &&b) {
    for (auto const &p : mMesh) out.push_back({p.interpolate(b[0]), p.interpolate(b[1]), p.interpolate(b[2])});
  });
  return out;
}

std::vector<Vertex> BezierMesh::dumpControlPoints() const {  // reference/bezierMesh.cpp:68-77
  std::vector<Vertex> out;
  out.reserve(mMesh.size() * BezierTriangle::csControlPointsSize);
  for (auto const &p : mMesh)
    for (uint32_t i = 0; i < BezierTriangle::csControlPointsSize; ++i) out.push_back(p.getControlPoint(i));
  return out;
}

namespace {
// point on the original edge of sub-patch p: blend of the surface and the flat triangle
Vertex edgeSplitPoint(BezierTriangle const &p) {
  return p.interpolate(0.5f, 0.5f, 0.0f) * kSplitBlend + p.interpolateLinear(0.5f, 0.5f, 0.0f) * (1.0f - kSplitBlend);
}
}  // namespace

Mesh BezierMesh::splitThickBezierTriangles() const {  // reference/bezierMesh.cpp:79-198
  static constexpr uint8_t sideBit[3] = {1u, 2u, 4u};
  static constexpr uint8_t pieces[8] = {1u, 2u, 2u, 3u, 2u, 3u, 3u, 4u};
  static constexpr float samples[3] = {0.25f, 0.5f, 0.75f};
  uint32_t const faces = static_cast<uint32_t>(mOriginalNeighbours.size());
  std::vector<uint8_t> cut(faces, 0u);
  auto original = [this](uint32_t o) {
    return Triangle{mMesh[o * 3u].getControlPoint(0), mMesh[o * 3u + 1u].getControlPoint(0),
                    mMesh[o * 3u + 2u].getControlPoint(0)};
  };
  for (uint32_t o = 0; o < faces; ++o) {
    Triangle const t = original(o);
    Plane const flat = Plane::createFromTriangle(t);
    float bulge = std::fabs(flat.distance(mMesh[o * 3u].interpolateAboveOriginalCentroid()));
    for (uint32_t i = 0; i < 3u; ++i)
      for (float r : samples) bulge = std::max(bulge, std::fabs(flat.distance(mMesh[o * 3u + i].interpolate(r, 1.0f - r, 0.0f))));
    if (bulge / util::getPerimeter(t) > kThickLimit) {  // too thick: split every side, and the neighbours' shared side
      cut[o] = 7u;
      auto const &adj = mOriginalNeighbours[o];
      for (uint32_t s = 0; s < 3u; ++s) cut[adj.mFellowTriangles[s]] |= sideBit[adj.mFellowCommonSideStarts[s]];
    }
  }
  Mesh out;
  uint32_t total = 0;
  for (uint8_t c : cut) total += pieces[c];
  out.reserve(total);
  for (uint32_t o = 0; o < faces; ++o) {
    Triangle const t = original(o);
    uint8_t const c = cut[o];
    uint32_t const base = o * 3u;
    switch (pieces[c]) {
      case 1:
        out.push_back(t);
        break;
      case 2: {  // one side split: two triangles around the new point
        static constexpr uint8_t splitSide[8] = {3u, 0u, 1u, 3u, 2u, 3u, 3u, 3u};
        uint32_t const s = splitSide[c], after = (s + 1u) % 3u, before = (s + 2u) % 3u;
        Vertex const m = edgeSplitPoint(mMesh[base + s]);
        out.push_back({t[after], t[before], m});
        out.push_back({t[before], t[s], m});
        break;
      }
      case 3: {  // two sides split: corner triangle + the shorter diagonal of the rest
        static constexpr uint8_t keptCorner[8] = {3u, 3u, 3u, 2u, 3u, 1u, 0u, 3u};
        uint32_t const k = keptCorner[c], after = (k + 1u) % 3u, before = (k + 2u) % 3u;
        Vertex const mBefore = edgeSplitPoint(mMesh[base + before]);
        Vertex const mAfter = edgeSplitPoint(mMesh[base + after]);
        out.push_back({t[before], mBefore, mAfter});
        if ((t[after] - mBefore).norm() < (t[k] - mAfter).norm()) {
          out.push_back({t[after], mAfter, mBefore});
          out.push_back({t[k], t[after], mBefore});
        } else {
          out.push_back({t[after], mAfter, t[k]});
          out.push_back({t[k], mAfter, mBefore});
        }
        break;
      }
      default: {  // all three sides: central triangle + three corners
        Triangle mid;
        for (uint32_t i = 0; i < 3u; ++i) mid[i] = edgeSplitPoint(mMesh[base + i]);
        out.push_back(mid);
        for (uint32_t i = 0; i < 3u; ++i) out.push_back({t[i], mid[i], mid[(i + 2u) % 3u]});
      }
    }
  }
  return out;
}

// The barycentric sub-triangles of BezierMesh::interpolate (util::divide of the unit triangle, in the
// reference's order, reference/3dGeomUtil.h:99-122): divisor^2 triangles x 3 vertices x 3 floats
// into `out`.  The device tessellation (bzr_mesh_interpolate) evaluates the patches at these.
extern "C" uint32_t bzr_internal_unit_subtriangles(int32_t divisor, float *out) {
  uint32_t k = 0;
  util::divide(kUnitBary, divisor, [&](Triangle &&b) {
    for (uint32_t v = 0; v < 3u; ++v)
      for (int32_t c = 0; c < 3; ++c) out[(size_t)k * 9u + v * 3u + c] = b[v](c);
    ++k;
  });
  return k;
}
