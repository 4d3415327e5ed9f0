// bzr.hpp -- C++17 drop-in for the reference's class API (balazs-bamer/cuda-bezier-triangle-raytracer @ v1).
//
// Same type and member names as reference/3dGeomUtil.h, mesh.h, bezierTriangle.h,
// bezierMesh.h and bezierLens.h, so reference callers (reference/test.cpp,
// the intended reference/rayTracer.cpp) compile unchanged against it; the
// forwarding headers next to this file carry the reference's file names.
//
// What differs underneath:
//   * no Eigen: Vector/Vertex/Matrix/Transform are bzr::Mat<R,C>, a small
//     column-major value type evaluating every operation in the order Eigen 3.3
//     uses for fixed-size float 3-vectors (redux a0 + (a1 + a2), cofactor inverse,
//     normalized() = v / sqrt(|v|^2) guarded by |v|^2 > 0);
//   * the ray-tracing hot path (BezierTriangle::intersect, BezierMesh::intersect,
//     BezierLens::refract): the batch overloads, bzr::traceChain and the multi-device
//     calls run on the GPU through libbzr's C ABI (include/bzr.h) -- the throughput
//     interface; the reference's single-ray methods run the same arithmetic on the
//     host (one ray: no launch, no PCIe round trip), bit-identical to the batch path;
//   * preprocessing (Mesh, BezierMesh construction) is host C++ as in the reference.
#ifndef BZR_BZR_HPP
#define BZR_BZR_HPP

#include <array>
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <initializer_list>
#include <limits>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "../bzr.h"

namespace bzr {

// ---------------------------------------------------------------- value type
template <int R, int C>
struct Mat {
  static constexpr int kRows = R, kCols = C, kSize = R * C;
  float a[R * C];  // column-major, like Eigen's default

  Mat() = default;
  template <int RR = R, int CC = C, typename = std::enable_if_t<RR * CC == 3>>
  Mat(float x, float y, float z) : a{x, y, z} {}
  // {{a,b,c}} (one row list) or {{a},{b},{c}} for vectors; row lists for matrices.
  Mat(std::initializer_list<std::initializer_list<float>> rows) {
    int nr = static_cast<int>(rows.size());
    int r = 0;
    for (auto const &row : rows) {
      int c = 0;
      for (float v : row) {
        if (nr == 1 && C == 1) a[c] = v;  // vector written as a single row
        else a[c * R + r] = v;
        ++c;
      }
      ++r;
    }
  }

  float &operator()(int i) { return a[i]; }
  float operator()(int i) const { return a[i]; }
  float &operator()(int i, int j) { return a[j * R + i]; }
  float operator()(int i, int j) const { return a[j * R + i]; }
  float &operator[](int i) { return a[i]; }
  float operator[](int i) const { return a[i]; }
  float *data() { return a; }
  float const *data() const { return a; }
  static constexpr int size() { return R * C; }
  static constexpr int rows() { return R; }
  static constexpr int cols() { return C; }

  static Mat Zero() { Mat m; for (auto &v : m.a) v = 0.0f; return m; }
  static Mat Constant(float s) { Mat m; for (auto &v : m.a) v = s; return m; }
  static Mat Identity() { Mat m = Zero(); for (int i = 0; i < (R < C ? R : C); ++i) m(i, i) = 1.0f; return m; }

  // comma initializer: v << x, y, z;  (row-major fill order, like Eigen)
  struct Comma {
    Mat &m; int k;
    Comma &operator,(float v) { m.a[(k % C) * R + k / C] = v; ++k; return *this; }
  };
  Comma operator<<(float v) { a[0] = v; return Comma{*this, 1}; }

  friend Mat operator+(Mat const &x, Mat const &y) { Mat r; for (int i = 0; i < R * C; ++i) r.a[i] = x.a[i] + y.a[i]; return r; }
  friend Mat operator-(Mat const &x, Mat const &y) { Mat r; for (int i = 0; i < R * C; ++i) r.a[i] = x.a[i] - y.a[i]; return r; }
  friend Mat operator-(Mat const &x) { Mat r; for (int i = 0; i < R * C; ++i) r.a[i] = -x.a[i]; return r; }
  template <typename S, typename = std::enable_if_t<std::is_arithmetic<S>::value>>
  friend Mat operator*(Mat const &x, S s) { float f = static_cast<float>(s); Mat r; for (int i = 0; i < R * C; ++i) r.a[i] = x.a[i] * f; return r; }
  template <typename S, typename = std::enable_if_t<std::is_arithmetic<S>::value>>
  friend Mat operator*(S s, Mat const &x) { float f = static_cast<float>(s); Mat r; for (int i = 0; i < R * C; ++i) r.a[i] = f * x.a[i]; return r; }
  template <typename S, typename = std::enable_if_t<std::is_arithmetic<S>::value>>
  friend Mat operator/(Mat const &x, S s) { float f = static_cast<float>(s); Mat r; for (int i = 0; i < R * C; ++i) r.a[i] = x.a[i] / f; return r; }
  Mat &operator+=(Mat const &y) { for (int i = 0; i < R * C; ++i) a[i] = a[i] + y.a[i]; return *this; }
  Mat &operator-=(Mat const &y) { for (int i = 0; i < R * C; ++i) a[i] = a[i] - y.a[i]; return *this; }
  template <typename S, typename = std::enable_if_t<std::is_arithmetic<S>::value>>
  Mat &operator*=(S s) { float f = static_cast<float>(s); for (auto &v : a) v = v * f; return *this; }
  template <typename S, typename = std::enable_if_t<std::is_arithmetic<S>::value>>
  Mat &operator/=(S s) { float f = static_cast<float>(s); for (auto &v : a) v = v / f; return *this; }
  friend bool operator==(Mat const &x, Mat const &y) { for (int i = 0; i < R * C; ++i) if (!(x.a[i] == y.a[i])) return false; return true; }
  friend bool operator!=(Mat const &x, Mat const &y) { return !(x == y); }

  // Eigen's unrolled redux: a0 + (a1 + a2) for three terms.
  float sum() const { static_assert(R * C == 3, "3-vector only"); return a[0] + (a[1] + a[2]); }
  float dot(Mat const &y) const { static_assert(R * C == 3, "3-vector only"); return a[0] * y.a[0] + (a[1] * y.a[1] + a[2] * y.a[2]); }
  float squaredNorm() const { return dot(*this); }
  float norm() const { return std::sqrt(squaredNorm()); }
  Mat normalized() const { float z = squaredNorm(); if (z > 0.0f) return *this / std::sqrt(z); return *this; }
  void normalize() { float z = squaredNorm(); if (z > 0.0f) *this /= std::sqrt(z); }
  Mat cross(Mat const &y) const {
    return Mat(a[1] * y.a[2] - a[2] * y.a[1], a[2] * y.a[0] - a[0] * y.a[2], a[0] * y.a[1] - a[1] * y.a[0]);
  }
  Mat<C, R> transpose() const { Mat<C, R> t; for (int i = 0; i < R; ++i) for (int j = 0; j < C; ++j) t(j, i) = (*this)(i, j); return t; }
  Mat inverse() const;  // 3x3 only
};

// matrix product, each entry the Eigen redux of the row-column products
template <int R, int K, int C>
inline Mat<R, C> operator*(Mat<R, K> const &x, Mat<K, C> const &y) {
  static_assert(K == 3, "inner dimension 3 only");
  Mat<R, C> r;
  for (int i = 0; i < R; ++i)
    for (int j = 0; j < C; ++j) r(i, j) = x(i, 0) * y(0, j) + (x(i, 1) * y(1, j) + x(i, 2) * y(2, j));
  return r;
}

template <int R, int C>
inline Mat<R, C> Mat<R, C>::inverse() const {
  static_assert(R == 3 && C == 3, "3x3 only");
  Mat const &m = *this;
  auto cof = [&m](int i, int j) {
    int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return m(i1, j1) * m(i2, j2) - m(i1, j2) * m(i2, j1);
  };
  float c0 = cof(0, 0), c1 = cof(1, 0), c2 = cof(2, 0);
  float det = c0 * m(0, 0) + (c1 * m(1, 0) + c2 * m(2, 0));
  float inv = 1.0f / det;
  Mat r;
  r(0, 0) = c0 * inv; r(0, 1) = c1 * inv; r(0, 2) = c2 * inv;
  r(1, 0) = cof(0, 1) * inv; r(1, 1) = cof(1, 1) * inv;
  r(2, 0) = cof(0, 2) * inv; r(2, 1) = cof(1, 2) * inv;
  r(1, 2) = cof(2, 1) * inv; r(2, 2) = cof(2, 2) * inv;
  return r;
}

class Context;  // a HIP device + stream (see bezierMesh section)
Context &defaultContext();

}  // namespace bzr

// ------------------------------------------------------------- 3dGeomUtil.h
constexpr float cgPi = 3.14159265358979323846;
constexpr float cgGeneralEpsilon = 1.0e-5;

using Vector = bzr::Mat<3, 1>;
using Vertex = bzr::Mat<3, 1>;
using Matrix = bzr::Mat<3, 3>;
using Transform = bzr::Mat<3, 3>;
using Triangle = std::array<Vertex, 3u>;

struct util {
  static Vector getNormal(Triangle const &f) { return (f[1] - f[0]).cross(f[2] - f[0]); }
  static Vector getNormal(Vertex const &a, Vertex const &b, Vertex const &c) { return (b - a).cross(c - a); }
  static float getPerimeter(Triangle const &t) { return (t[0] - t[1]).norm() + (t[1] - t[2]).norm() + (t[2] - t[0]).norm(); }
  static Vertex barycentric2cartesian(Triangle const &t, float b0, float b1, float b2) { return t[0] * b0 + t[1] * b1 + t[2] * b2; }
  static Vertex barycentric2cartesian(Triangle const &t, float b0, float b1) { return t[0] * b0 + t[1] * b1 + t[2] * (1.0f - b0 - b1); }
  static Vertex barycentric2cartesian(Vertex const &v0, Vertex const &v1, Vertex const &v2, float b0, float b1, float b2) {
    return v0 * b0 + v1 * b1 + v2 * b2;
  }
  static Vertex barycentric2cartesian(Vertex const &v0, Vertex const &v1, Vertex const &v2, float b0, float b1) {
    return v0 * b0 + v1 * b1 + v2 * (1.0f - b0 - b1);
  }
  static Matrix getBarycentricInverse(Vertex const &v0, Vertex const &v1, Vertex const &v2);
  static Vector getAperpendicular(Vector const &v);
  template <typename tLambda>
  static void divide(Triangle const &t, int32_t divisor, tLambda &&collector);
  static Vector getAltitude(Vertex const &common1, Vertex const &common2, Vertex const &independent);
  static uint32_t toWhichSide(Vertex const &start, Vertex const &end);
};

struct Ray final {
  Vertex mStart;
  Vector mDirection;  // normalized
  Ray() = default;
  Ray(Vertex const &start, Vector const &direction) : mStart(start), mDirection(direction.normalized()) {}
  Vector getPerpendicularTo(Vertex const &p) const { return p - mStart - (p - mStart).dot(mDirection) * mDirection; }
  float getDistance(Vertex const &p) const { return getPerpendicularTo(p).norm(); }
  float getDistance2(Vertex const &p) const { return getPerpendicularTo(p).squaredNorm(); }
  float getAverageErrorSquared(std::vector<Vertex> const &points) const;
};

struct Intersection final {
  bool mValid;
  Vertex mPoint;
  float mCosIncidence;
  float mDistance;
};

struct Plane final {
  static constexpr float csRayPlaneIntersectionEpsilon = 0.00001f;
  Vector mNormal;
  float mConstant;

  Plane() = default;
  Plane(Vector const &normal, float constant) : mNormal(normal), mConstant(constant) {}
  static Plane createFrom1proportion2points(float proportion, Vertex const &p0, Vertex const &p1);
  static Plane createFrom3points(Vertex const &p0, Vertex const &p1, Vertex const &p2);
  static Plane createFromTriangle(Triangle const &t) { return createFrom3points(t[0], t[1], t[2]); }
  static Plane createFrom1vector2points(Vector const &direction, Vertex const &p0, Vertex const &p1);
  static Plane createFrom2vectors1point(Vertex const &d0, Vertex const &d1, Vertex const &p);
  static Vertex intersect(Plane const &a, Plane const &b, Plane const &c);
  // Deviation D1/D2: mPoint is written for every |cos| >= eps (and = start otherwise).
  Intersection intersect(Vertex const &start, Vector const direction) const;
  Intersection intersect(Ray const &r) const { return intersect(r.mStart, r.mDirection); }
  Vector project(Vector const &p) const { return p - mNormal * (p.dot(mNormal) - mConstant); }
  float distance(Vector const &p) const { return p.dot(mNormal) - mConstant; }
  void makeDistancePositive(Vector const p) { if (distance(p) < 0.0f) { mNormal = -mNormal; mConstant = -mConstant; } }
  void makeDistanceNegative(Vector const p) { if (distance(p) > 0.0f) { mNormal = -mNormal; mConstant = -mConstant; } }
  bool operator<(Plane const &o) const;
};

struct Spherical final {
  float mR;
  float mAzimuth;
  float mInclination;
  Spherical(float x, float y, float z)
      : mR(std::sqrt(x * x + y * y + z * z)), mAzimuth(std::atan2(y, x)), mInclination(std::acos(z / mR)) {}
};

struct Sphere final {
  Vector mCenter;
  float mRadius;
  Sphere() = default;
  Sphere(Vector const &c, float r) : mCenter(c), mRadius(r) {}
};

template <typename tLambda>
void util::divide(Triangle const &t, int32_t divisor, tLambda &&collector) {
  Vector const v01 = (t[1] - t[0]) / divisor;
  Vector const v02 = (t[2] - t[0]) / divisor;
  Vertex line = t[0];
  Vertex b0 = line;
  Vertex b1 = divisor > 1 ? Vertex(b0 + v01) : t[1];
  Vertex b2 = divisor > 1 ? Vertex(b0 + v02) : t[2];
  for (int32_t i = 0; i + 1 < divisor; ++i) {
    for (int32_t j = 0; j < divisor - i - 1; ++j) {
      collector(Triangle{b0, b1, b2});
      Vertex b1n = b1 + v02;
      collector(Triangle{b1, b1n, b2});
      b1 = b1n;
      b0 = b2;
      b2 += v02;
    }
    collector(Triangle{b0, b1, b2});
    line += v01;
    b0 = line;
    b1 = b0 + v01;
    b2 = b0 + v02;
  }
  collector(Triangle{b0, t[1], b2});
}

// -------------------------------------------------------------------- mesh.h
class Mesh final {
 public:
  using TheMesh = std::vector<Triangle>;
  using value_type = Triangle;
  struct Neighbours final {
    std::array<uint32_t, 3u> mFellowTriangles;        // neighbour across edge (i, i+1)
    std::array<uint8_t, 3u> mFellowCommonSideStarts;  // that edge's start index in the neighbour
  };
  struct VertexHash {
    std::size_t operator()(Vertex const &v) const {
      return std::hash<float>{}(v[0]) ^ (std::hash<float>{}(v[1]) << 1u) ^ (std::hash<float>{}(v[2]) << 2u);
    }
  };
  using Face2neighbours = std::vector<Neighbours>;
  using Vertex2averageNormals = std::unordered_map<Vertex, Vector, VertexHash>;
  using Vertices = std::unordered_set<Vertex, VertexHash>;

  Mesh() = default;
  Mesh(Mesh &&) = default;
  Mesh(Mesh const &) = default;
  Mesh &operator=(Mesh &&) = default;
  Mesh &operator=(Mesh const &) = default;

  auto size() const { return mMesh.size(); }
  auto begin() const { return mMesh.begin(); }
  auto end() const { return mMesh.end(); }
  auto cbegin() const { return mMesh.cbegin(); }
  auto cend() const { return mMesh.cend(); }
  void reserve(uint32_t n) { mMesh.reserve(n); }
  void push_back(Triangle const &t) { mMesh.push_back(t); }
  void clear() { mMesh.clear(); }
  auto &operator[](uint32_t i) { return mMesh[i]; }
  auto const &operator[](uint32_t i) const { return mMesh[i]; }

  TheMesh const &getMesh() const { return mMesh; }
  Face2neighbours const &getFace2neighbours() const { return mFace2neighbours; }
  Vertex2averageNormals const &getVertex2averageNormals() const { return mVertex2averageNormals; }

  void standardizeVertices();
  Vertices getVertices() const;
  void standardizeNormals();  // throws char const* "Vertex on edge detected." like the reference
  void transform(Transform const &t, Vertex const displacement);
  Mesh &operator+=(Vector const d) { transform(Transform::Identity(), d); return *this; }
  Mesh &operator*=(Transform const &t) { transform(t, Vertex::Zero()); return *this; }
  Mesh &operator*=(float const &f) { transform(Transform::Identity() * f, Vertex::Zero()); return *this; }
  void splitTriangles(float maxTriangleSide);
  void splitTriangles(int32_t divisor);
  void readMesh(std::string const &filename);
  void writeMesh(std::string const &filename) const;
  void makeSolidOfRevolution(int32_t sectors, int32_t belts, std::function<float(float)> envelope, Vector const &size);
  void makeEllipsoid(int32_t sectors, int32_t belts, Vector const &size) {
    makeSolidOfRevolution(sectors, belts, [](float x) { return std::sqrt(1 - x * x); }, size);
  }
  void makeUnitSphere(int32_t sectors, int32_t belts) { makeEllipsoid(sectors, belts, Vector(1.0f, 1.0f, 1.0f)); }

 private:
  TheMesh mMesh;
  Face2neighbours mFace2neighbours;
  Vertex2averageNormals mVertex2averageNormals;
};

// ---------------------------------------------------------- bezierTriangle.h
struct BezierIntersection final {
  enum class What : uint32_t { cFollowSide0 = 0u, cFollowSide1 = 1u, cFollowSide2 = 2u, cNone = 3u, cIntersect = 4u };
  Intersection mIntersection;
  Vertex mBarycentric;
  Vector mNormal;
  What mWhat;
};

class BezierTriangle final {  // cubic Bezier triangle; layout == bzr_patch (264 B)
 public:
  enum class LimitPlaneIntersection : uint32_t { cThis = 0u, cNone = 1u };
  static constexpr uint32_t csControlPointsSize = 10u;

  BezierTriangle() = default;
  BezierTriangle(Vertex const &originalCommonVertex0, Vertex const &originalCommonVertex1, Vertex const &originalCentroid,
                 Vector const &averageNormal0, Vector const &averageNormal1, Plane const &planeBetweenOriginalNeighbours,
                 std::array<uint32_t, 3u> const &neighbourIndices);
  void setMissingFields1(Vertex const &originalCentroid, BezierTriangle const &next, BezierTriangle const &previous);
  void setMissingFields2(Vertex const &, BezierTriangle const &next, BezierTriangle const &);
  void setMissingFields3(Vertex const &, BezierTriangle const &next, BezierTriangle const &previous);

  Vertex getControlPoint(uint32_t i) const { return mControlPoints[i]; }
  std::array<uint32_t, 3u> getNeighbours() const { return mNeighbours; }
  Vertex interpolateLinear(float b0, float b1, float b2) const;
  Vertex interpolateLinear(float b0, float b1) const { return interpolateLinear(b0, b1, 1.0f - b0 - b1); }
  Vertex interpolateLinear(Vertex const &b) const { return interpolateLinear(b(0), b(1), b(2)); }
  Vertex interpolate(float b0, float b1, float b2) const;
  Vertex interpolate(float b0, float b1) const { return interpolate(b0, b1, 1.0f - b0 - b1); }
  Vertex interpolate(Vertex const &b) const { return interpolate(b(0), b(1), b(2)); }
  Vertex interpolateAboveOriginalCentroid() const { return mControlPoints[2]; }
  Vector getNormal(Vector const &barycentric) const;
  // Host, bit-identical to the GPU (bzr_patch_intersect); see BezierMesh::intersect for the batch interface.
  BezierIntersection intersect(Ray const &ray, LimitPlaneIntersection limit) const;

  Plane mUnderlyingPlane;
  std::array<Plane, 3u> mNeighbourDividerPlanes;
  std::array<uint32_t, 3u> mNeighbours;
  std::array<Vertex, csControlPointsSize> mControlPoints;
  Matrix mBarycentricInverse;
  float mHeightInside;
  float mHeightOutside;
  Vector mBezierDerivativeDirectionVectorA;
  Vector mBezierDerivativeDirectionVectorB;
};

// -------------------------------------------------------------- bezierMesh.h
namespace bzr {
// Owns one bzr_ctx (a HIP device and stream).
class Context {
 public:
  explicit Context(int device = 0);
  ~Context();
  Context(Context const &) = delete;
  Context &operator=(Context const &) = delete;
  bzr_ctx *get() const { return mCtx; }
  // Process-unique, never reused (a new Context may get a destroyed one's bzr_ctx address).
  uint64_t id() const { return mId; }
  void sync() const;
  // Held by the batch calls for their whole (synchronous) use of the context: several host threads may share
  // one context -- e.g. defaultContext() -- and call the batch overloads concurrently, as the reference's hot
  // methods may be; the calls then run one after another.
  std::mutex &lock() const { return mLock; }

 private:
  bzr_ctx *mCtx = nullptr;
  uint64_t mId = 0;
  mutable std::mutex mLock;
};
void check(bzr_status s);  // throws std::runtime_error with bzr_last_error() text
struct DeviceMesh;         // device copy of a patch array (bzr_mesh)
}  // namespace bzr

class BezierMesh final {
 public:
  explicit BezierMesh(Mesh const &mesh);
  BezierMesh(std::vector<BezierTriangle> patches, Mesh::Face2neighbours originalNeighbours);

  auto size() const { return mMesh.size(); }
  auto cbegin() const { return mMesh.cbegin(); }
  auto cend() const { return mMesh.cend(); }
  auto const &operator[](uint32_t i) const { return mMesh[i]; }

  Mesh interpolate(int32_t divisor) const;
  std::vector<Vertex> dumpControlPoints() const;
  Mesh splitThickBezierTriangles() const;
  BezierIntersection intersect(Ray const &ray) const;  // host (brute force, index order), bit-identical to the GPU
  BezierIntersection intersect(Ray const &ray, uint32_t *patchIndex) const;  // the same + the patch hit (~0u: miss)
  // Batch interface (GPU).  patchIndex (optional) receives the index of the patch hit, ~0u on a miss.
  void intersect(Ray const *rays, std::size_t n, BezierIntersection *out, uint32_t *patchIndex = nullptr,
                 bzr::Context *ctx = nullptr) const;
  // Device handle of this mesh on ctx (uploaded on first use and cached per context; thread-safe).
  bzr_mesh *device(bzr::Context &ctx) const;

 private:
  std::vector<BezierTriangle> mMesh;
  Mesh::Face2neighbours mOriginalNeighbours;
  mutable std::vector<std::shared_ptr<bzr::DeviceMesh>> mDevices;
};

// -------------------------------------------------------------- bezierLens.h
enum class RefractionResult : uint32_t { cNone = 0u, cInside = 1u, cOutside = 2u };

class BezierLens final {
 public:
  BezierLens(float ri, BezierMesh const &mesh) : mRefractiveIndex(ri), mMesh(mesh) {}
  BezierLens(float ri, BezierMesh &&mesh) : mRefractiveIndex(ri), mMesh(std::move(mesh)) {}
  std::pair<Ray, RefractionResult> refract(Ray const &ray, RefractionResult expected) const;  // host, as intersect(Ray)
  void refract(Ray const *rays, RefractionResult const *expected, std::size_t n, Ray *outRays,
               RefractionResult *outStatus, bzr::Context *ctx = nullptr) const;
  float getRefractiveIndex() const { return mRefractiveIndex; }
  BezierMesh const &getMesh() const { return mMesh; }

 private:
  float mRefractiveIndex;
  BezierMesh mMesh;
};

namespace bzr {
// Whole refraction chain through `lenses` in one GPU launch (reference/test.cpp:376-401 semantics).
void traceChain(std::vector<BezierLens const *> const &lenses, Ray const *rays, std::size_t n, Ray *outRays,
                RefractionResult *outStatus, uint32_t *outSegments = nullptr, Context *ctx = nullptr);
// The same chain over several devices from one process (bzr_trace_tiled): tiles of tileRays
// consecutive rays dealt round-robin to `ctxs` (one per device, distinct), results in input order.
void traceChainTiled(std::vector<Context *> const &ctxs, std::vector<BezierLens const *> const &lenses,
                     Ray const *rays, std::size_t n, Ray *outRays, RefractionResult *outStatus,
                     uint32_t *outSegments = nullptr, uint32_t tileRays = 4096);
// Frame after frame over several devices from one process (bzr_tiled): slots[s][d] is frame slot s's
// context on device d; a frame's n tile-major rays are dealt in tiles of tileRays to the devices and the
// results gathered to device 0 on the device side (RCCL over xGMI between distinct devices, peer copies
// otherwise).  The device-pointer trace() is asynchronous (frames on different slots overlap; keep one set
// of outputs per frame in flight, sync() before reading them); the host-pointer trace() is synchronous.
// Every member takes its contexts' locks (in context id order, as traceChainTiled does), so the contexts may
// also serve batch calls from other threads.
class TiledChain {
 public:
  TiledChain(std::vector<std::vector<Context *>> const &slots, std::vector<BezierLens const *> const &lenses,
             std::size_t n, uint32_t tileRays = 4096, int transport = BZR_GATHER_AUTO);
  ~TiledChain();
  TiledChain(TiledChain const &) = delete;
  TiledChain &operator=(TiledChain const &) = delete;
  int transport() const;  // BZR_GATHER_RCCL, BZR_GATHER_PEER, or BZR_GATHER_DIRECT (AUTO's choice for one device)
  void setRays(Ray const *rays);  // n host rays, tile-major; copied before it returns, then resident
  // [6][n] SoA on slot 0 device 0: the copy is only queued (on device 0's stream); the source must stay unchanged
  // and allocated until the next sync()
  void setRaysDevice(float const *raysSoaOnDevice0);
  void trace(float *outRaysSoa, uint32_t *outStatus, uint32_t *outSegments = nullptr, uint32_t flags = 0);  // device 0
  void trace(Ray *outRays, RefractionResult *outStatus, uint32_t *outSegments = nullptr, uint32_t flags = 0);  // host
  // Compact gather (bzr_tiled_calibrate): one counted frame, then only the refracted rays cross to device 0
  // (needs setRays); returns the capacity.  sync() throws if a later frame exceeds it.
  uint32_t calibrate(uint32_t flags = 0);
  void sync();

 private:
  bzr_tiled *mPlan = nullptr;
  std::size_t mDevices = 0, mN = 0;
  std::vector<bzr_mesh const *> mMeshes;  // [device][lens]
  std::vector<Context *> mContexts;      // every slot's contexts (their locks)
  std::vector<float> mRi;
};
}  // namespace bzr

static_assert(sizeof(BezierTriangle) == sizeof(bzr_patch), "BezierTriangle must match the 264-byte record");
static_assert(sizeof(Vector) == 12 && sizeof(Matrix) == 36 && sizeof(Plane) == 16, "Eigen-compatible layout");
static_assert(sizeof(BezierIntersection) == sizeof(bzr_hit_record) &&
                  offsetof(BezierIntersection, mIntersection.mPoint) == offsetof(bzr_hit_record, point) &&
                  offsetof(BezierIntersection, mIntersection.mCosIncidence) == offsetof(bzr_hit_record, cos_incidence) &&
                  offsetof(BezierIntersection, mIntersection.mDistance) == offsetof(bzr_hit_record, distance) &&
                  offsetof(BezierIntersection, mBarycentric) == offsetof(bzr_hit_record, bary) &&
                  offsetof(BezierIntersection, mNormal) == offsetof(bzr_hit_record, normal) &&
                  offsetof(BezierIntersection, mWhat) == offsetof(bzr_hit_record, what),
              "BezierIntersection must match the 52-byte bzr_hit_record (bzr_intersect_records)");

#endif
