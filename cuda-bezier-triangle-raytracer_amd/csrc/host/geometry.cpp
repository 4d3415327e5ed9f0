// geometry.cpp -- L1 geometry of the drop-in API (reference/3dGeomUtil.h:31-334).
// Host-only value maths used by preprocessing and by callers; none of it is on
// the GPU hot path (that lives in csrc/device/trace.hip).
#include "bzr/bzr.hpp"

Matrix util::getBarycentricInverse(Vertex const &v0, Vertex const &v1, Vertex const &v2) {
  // columns are the vertices (reference/3dGeomUtil.h:70-77)
  Matrix m;
  for (int i = 0; i < 3; ++i) {
    m(i, 0) = v0(i);
    m(i, 1) = v1(i);
    m(i, 2) = v2(i);
  }
  return m.inverse();
}

Vector util::getAperpendicular(Vector const &v) {  // reference/3dGeomUtil.h:80-95
  constexpr float eps = 1e-10f;
  Vector r;
  r(0) = 0.0f;
  if (std::fabs(v(1)) < eps && std::fabs(v(2)) < eps) {
    r(1) = 1.0f;
    r(2) = 0.0f;
  } else {
    float den = std::sqrt(v(1) * v(1) + v(2) * v(2));
    r(1) = -v(2) / den;
    r(2) = v(1) / den;
  }
  return r;
}

Vector util::getAltitude(Vertex const &common1, Vertex const &common2, Vertex const &independent) {  // :125-130
  Vector side = common2 - common1;
  Vector other = independent - common1;
  float foot = side.dot(other) / side.squaredNorm();
  return other - side * foot;
}

uint32_t util::toWhichSide(Vertex const &s, Vertex const &e) {  // :137-164
  uint32_t side = 3u;
  // edge k of the barycentric triangle runs between unit vertices k and k+1
  for (uint32_t k = 0; k < 3u; ++k) {
    uint32_t a = k, b = (k + 1u) % 3u;
    float den = s(a) - e(a) + s(b) - e(b);
    if (std::fabs(den) > cgGeneralEpsilon) {
      float ratio = ((s(a) - 1.0f) * e(b) - s(b) * (e(a) - 1.0f)) / den;
      float heading = (s(a) + s(b) - 1.0f) / den;
      if (ratio > -cgGeneralEpsilon && ratio < 1.0f + cgGeneralEpsilon && heading > 0.0f) side = k;
    }
  }
  return side;
}

float Ray::getAverageErrorSquared(std::vector<Vertex> const &points) const {  // :199-205
  float acc = 0.0f;
  for (auto const &p : points) acc += getDistance2(p);
  return points.empty() ? 0.0f : acc / static_cast<float>(points.size());
}

Plane Plane::createFrom1proportion2points(float proportion, Vertex const &p0, Vertex const &p1) {  // :233-238
  Plane pl;
  pl.mNormal = (p1 - p0).normalized();
  pl.mConstant = pl.mNormal.dot(p1 * proportion + p0 * (1.0f - proportion));
  return pl;
}

Plane Plane::createFrom3points(Vertex const &p0, Vertex const &p1, Vertex const &p2) {  // :241-246
  Plane pl;
  pl.mNormal = (p1 - p0).cross(p2 - p0).normalized();
  pl.mConstant = pl.mNormal.dot(p0);
  return pl;
}

Plane Plane::createFrom1vector2points(Vector const &direction, Vertex const &p0, Vertex const &p1) {  // :252-257
  Plane pl;
  pl.mNormal = direction.cross(p1 - p0).normalized();
  pl.mConstant = pl.mNormal.dot(p0);
  return pl;
}

Plane Plane::createFrom2vectors1point(Vertex const &d0, Vertex const &d1, Vertex const &p) {  // :260-265
  Plane pl;
  pl.mNormal = d0.cross(d1).normalized();
  pl.mConstant = pl.mNormal.dot(p);
  return pl;
}

Vertex Plane::intersect(Plane const &a, Plane const &b, Plane const &c) {  // :268-276
  Matrix rows;
  Plane const *pl[3] = {&a, &b, &c};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) rows(i, j) = pl[i]->mNormal(j);
  return rows.inverse() * Vector(a.mConstant, b.mConstant, c.mConstant);
}

Intersection Plane::intersect(Vertex const &start, Vector const direction) const {  // :279-296 + D1/D2
  Intersection r;
  r.mCosIncidence = direction.dot(mNormal);
  if (std::fabs(r.mCosIncidence) >= csRayPlaneIntersectionEpsilon) {
    r.mDistance = (mConstant - mNormal.dot(start)) / r.mCosIncidence;
    r.mValid = r.mDistance > 0.0f;
    r.mPoint = start + r.mDistance * direction;  // D1: written for negative distances too
  } else {
    r.mValid = false;
    r.mDistance = 0.0f;
    r.mPoint = start;  // D2
  }
  return r;
}

bool Plane::operator<(Plane const &o) const {  // :330-333 (lexicographic on normal, then constant)
  for (int i = 0; i < 3; ++i) {
    if (mNormal(i) < o.mNormal(i)) return true;
    if (!(mNormal(i) == o.mNormal(i))) return false;
  }
  return mConstant < o.mConstant;
}
