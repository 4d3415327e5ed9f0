// trimesh.cpp -- Mesh of the drop-in API: triangle soup -> welded, consistently
// oriented, neighbour-annotated mesh (reference/mesh.h, reference/mesh.cpp).
//
// Where the reference's result depends on container iteration order, the same
// libstdc++ container (or an order-equivalent one) is used so the patch records
// built from this mesh are bit-identical to the oracle's (tests/test_host_parity.py):
//   * projected coordinates: stable sort == std::multimap<float,...> order;
//   * edge -> faces: std::unordered_multimap (equal_range newest-first);
//   * faces around the smallest-x vertex: std::unordered_set<uint32_t> order;
//   * per-vertex normal sums: faces in decreasing index order (newest-first equal_range).
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>

#include "bzr/bzr.hpp"

namespace {

struct Projected {
  float key;
  uint32_t face;
  uint32_t corner;
};

bool lexLess(Vertex const &a, Vertex const &b) {
  return a(0) < b(0) || (a(0) == b(0) && a(1) < b(1)) || (a(0) == b(0) && a(1) == b(1) && a(2) < b(2));
}

// A face's index triple plus the edge table, rebuilt after every re-orientation.
struct Topology {
  std::vector<std::array<uint32_t, 3>> faceVertex;
  std::unordered_map<Vertex, uint32_t, Mesh::VertexHash> vertexIndex;
  std::unordered_multimap<uint64_t, uint32_t> edgeFaces;

  static uint64_t edgeKey(uint32_t a, uint32_t b) {
    if (a > b) std::swap(a, b);
    return (static_cast<uint64_t>(a) << 32) | b;
  }

  explicit Topology(Mesh::TheMesh const &mesh) {  // reference/mesh.cpp:118-153
    faceVertex.reserve(mesh.size());
    for (uint32_t f = 0; f < mesh.size(); ++f) {
      std::array<uint32_t, 3> ids;
      for (uint32_t k = 0; k < 3; ++k) {
        auto it = vertexIndex.find(mesh[f][k]);
        if (it == vertexIndex.end()) it = vertexIndex.emplace(mesh[f][k], static_cast<uint32_t>(vertexIndex.size())).first;
        ids[k] = it->second;
      }
      faceVertex.push_back(ids);
      for (uint32_t k = 0; k < 3; ++k) edgeFaces.emplace(edgeKey(ids[k], ids[(k + 1) % 3]), f);
    }
  }

  // reference/mesh.cpp:185-222
  Mesh::Face2neighbours neighbours() const {
    static constexpr uint8_t sideOf[3][3] = {{3, 0, 2}, {0, 3, 1}, {2, 1, 3}};
    Mesh::Face2neighbours out(faceVertex.size());
    for (uint32_t f = 0; f < faceVertex.size(); ++f) {
      for (uint32_t k = 0; k < 3; ++k) {
        uint32_t a = faceVertex[f][k], b = faceVertex[f][(k + 1) % 3];
        auto range = edgeFaces.equal_range(edgeKey(a, b));
        auto it = range.first;
        if (it == range.second) throw "Vertex on edge detected.";
        if (it->second == f && ++it == range.second) throw "Vertex on edge detected.";
        uint32_t other = it->second;
        auto const &of = faceVertex[other];
        auto ia = std::find(of.begin(), of.end(), a) - of.begin();
        auto ib = std::find(of.begin(), of.end(), b) - of.begin();
        out[f].mFellowTriangles[k] = other;
        out[f].mFellowCommonSideStarts[k] = (ia < 3 && ib < 3) ? sideOf[ia][ib] : 3u;
      }
    }
    return out;
  }
};

uint32_t firstCornerNotIn(Triangle const &target, Triangle const &other) {  // reference/mesh.cpp:107-116
  for (uint32_t i = 0; i < 3; ++i)
    if (std::find(other.begin(), other.end(), target[i]) == other.end()) return i;
  return 3u;
}

// Orient `face` so its normal has a non-negative component along `outward` (reference/mesh.cpp:241-248).
void orientAlong(Triangle &face, Vertex const &outward) {
  if (outward.dot(util::getNormal(face)) < 0.0f) std::swap(face[0], face[1]);
}

// Orient `unknown` consistently with its edge-neighbour `known` (reference/mesh.cpp:250-282).
void orientLike(Triangle const &known, Triangle &unknown) {
  uint32_t ik = firstCornerNotIn(known, unknown);
  uint32_t iu = firstCornerNotIn(unknown, known);
  if (ik > 2 || iu > 2) return;  // identical faces: out-of-range in the reference, unreachable on valid meshes
  uint32_t k1 = (ik + 1) % 3, k2 = (ik + 2) % 3, u1 = (iu + 1) % 3, u2 = (iu + 2) % 3;
  Vector altKnown = util::getAltitude(known[k1], known[k2], known[ik]);
  Vector altUnknown = util::getAltitude(unknown[u1], unknown[u2], unknown[iu]);
  float altDot = altKnown.dot(altUnknown);
  Vector nKnown = util::getNormal(known);
  Vector nUnknown = util::getNormal(unknown);
  float normalDot = nKnown.dot(nUnknown);
  if (std::fabs(normalDot / (nKnown.norm() * nUnknown.norm())) < 0.01f) {
    // nearly perpendicular faces: judge with the free corner pushed along the known face
    Vertex moved = unknown[iu] + 0.2f * (known[ik] - (known[k1] + known[k2]) / 2.0f);
    Triangle probe = unknown;
    probe[iu] = moved;
    altUnknown = util::getAltitude(unknown[u1], unknown[u2], moved);
    altDot = altKnown.dot(altUnknown);
    nUnknown = util::getNormal(probe);
    normalDot = nKnown.dot(nUnknown);
  }
  if (altDot * normalDot > 0.0f) std::swap(unknown[u1], unknown[u2]);
}

}  // namespace

// ------------------------------------------------------------ vertex welding
void Mesh::standardizeVertices() {  // reference/mesh.cpp:72-91 (+ helpers :4-70)
  if (mMesh.empty()) return;
  float shortest = std::numeric_limits<float>::max();
  for (auto const &t : mMesh)
    for (uint32_t i = 0; i < 3; ++i) shortest = std::min(shortest, (t[i] - t[(i + 1) % 3]).norm());
  float const eps = shortest * 0.2f;

  std::array<std::vector<Projected>, 3> sorted;
  std::array<std::vector<uint32_t>, 3> bounds;  // interval starts + end sentinel
  std::array<uint32_t, 3> widest{};
  for (int d = 0; d < 3; ++d) {
    auto &s = sorted[d];
    s.reserve(mMesh.size() * 3);
    for (uint32_t f = 0; f < mMesh.size(); ++f)
      for (uint32_t k = 0; k < 3; ++k) s.push_back({mMesh[f][k](d), f, k});
    std::stable_sort(s.begin(), s.end(), [](Projected const &x, Projected const &y) { return x.key < y.key; });
    // group entries closer than eps to the group's first entry
    uint32_t groupStart = 0, count = 1, most = 0;
    float startKey = s[0].key;
    bounds[d].push_back(0);
    for (uint32_t i = 1; i < s.size(); ++i) {
      if (s[i].key - startKey >= eps) {
        bounds[d].push_back(i);
        startKey = s[i].key;
        groupStart = i;
        most = std::max(most, count);
        count = 1;
      } else {
        ++count;
      }
    }
    (void)groupStart;
    most = std::max(most, count);
    bounds[d].push_back(static_cast<uint32_t>(s.size()));
    widest[d] = most;
  }
  int const d = static_cast<int>(std::min_element(widest.begin(), widest.end()) - widest.begin());
  float const eps2 = eps * eps;
  auto const &s = sorted[d];
  auto const &b = bounds[d];
  for (std::size_t g = 0; g + 1 < b.size(); ++g) {
    for (uint32_t i = b[g]; i < b[g + 1]; ++i) {
      Vertex &v1 = mMesh[s[i].face][s[i].corner];
      for (uint32_t j = b[g]; j < b[g + 1]; ++j) {
        Vertex const &v2 = mMesh[s[j].face][s[j].corner];
        if ((v1 - v2).squaredNorm() < eps2 && lexLess(v1, v2)) v1 = v2;  // snap to the lexicographically larger one
      }
    }
  }
}

Mesh::Vertices Mesh::getVertices() const {  // reference/mesh.cpp:95-103
  Vertices out;
  for (auto const &t : mMesh)
    for (auto const &v : t) out.insert(v);
  return out;
}

// -------------------------------------------------------- orientation & adjacency
void Mesh::standardizeNormals() {  // reference/mesh.cpp:310-357
  mFace2neighbours.clear();
  mVertex2averageNormals.clear();
  if (mMesh.empty()) return;
  {
    Topology topo(mMesh);
    // vertex with the smallest x (first one on ties), reference/mesh.cpp:155-170
    float smallestX = std::numeric_limits<float>::max();
    uint32_t smallestIndex = 0;
    for (uint32_t f = 0; f < mMesh.size(); ++f)
      for (uint32_t k = 0; k < 3; ++k)
        if (mMesh[f][k](0) < smallestX) {
          smallestX = mMesh[f][k](0);
          smallestIndex = topo.faceVertex[f][k];
        }
    std::unordered_set<uint32_t> around;
    for (uint32_t f = 0; f < mMesh.size(); ++f)
      for (uint32_t k = 0; k < 3; ++k)
        if (topo.faceVertex[f][k] == smallestIndex) around.insert(f);
    mFace2neighbours = topo.neighbours();

    Vertex const outward(-1.0f, 0.0f, 0.0f);
    float bestDot = -std::numeric_limits<float>::max();
    uint32_t seed = 0;
    for (uint32_t f : around) {  // reference/mesh.cpp:224-239
      float d = std::fabs(outward.dot(util::getNormal(mMesh[f]).normalized()));
      if (d > bestDot) {
        bestDot = d;
        seed = f;
      }
    }
    orientAlong(mMesh[seed], outward);
    std::vector<bool> pending(mMesh.size(), true);
    std::vector<std::pair<uint32_t, uint32_t>> stack;  // (known, unknown), LIFO
    for (uint32_t f : mFace2neighbours[seed].mFellowTriangles) stack.emplace_back(seed, f);
    pending[seed] = false;
    while (!stack.empty()) {
      auto [known, unknown] = stack.back();
      stack.pop_back();
      if (pending[unknown]) orientLike(mMesh[known], mMesh[unknown]);
      pending[unknown] = false;
      for (uint32_t f : mFace2neighbours[unknown].mFellowTriangles)
        if (pending[f] && unknown != f) stack.emplace_back(unknown, f);
    }
  }
  mFace2neighbours = Topology(mMesh).neighbours();  // corners may have been swapped

  // angle-weighted vertex normals, reference/mesh.cpp:284-308
  std::unordered_map<Vertex, std::vector<uint32_t>, VertexHash> facesOf;
  for (uint32_t f = 0; f < mMesh.size(); ++f)
    for (uint32_t k = 0; k < 3; ++k) facesOf[mMesh[f][k]].push_back(f);
  for (auto const &entry : facesOf) {
    Vertex const &v = entry.first;
    Vector sum = Vector::Zero();
    for (auto it = entry.second.rbegin(); it != entry.second.rend(); ++it) {
      Triangle const &t = mMesh[*it];
      uint32_t w = static_cast<uint32_t>(std::find(t.begin(), t.end(), v) - t.begin());
      Vector sideA = t[(w + 1) % 3] - t[w];
      Vector sideB = t[(w + 2) % 3] - t[w];
      float cosAngle = sideA.dot(sideB) / (sideA.norm() * sideB.norm());
      sum += util::getNormal(t).normalized() * std::acos(cosAngle);
    }
    sum.normalize();
    mVertex2averageNormals.emplace(v, sum);
  }
}

// -------------------------------------------------------------- transforms
void Mesh::transform(Transform const &t, Vertex const displacement) {  // reference/mesh.cpp:361-367
  for (auto &tri : mMesh)
    for (auto &v : tri) v = t * v + displacement;
}

void Mesh::splitTriangles(float maxTriangleSide) {  // reference/mesh.cpp:375-385
  TheMesh out;
  for (auto const &t : mMesh) {
    float side = (t[0] - t[1]).norm();
    side = std::max(side, (t[0] - t[2]).norm());
    side = std::max(side, (t[1] - t[2]).norm());
    util::divide(t, static_cast<int32_t>(std::ceil(side / maxTriangleSide)), [&out](Triangle &&n) { out.push_back(n); });
  }
  mMesh = std::move(out);
}

void Mesh::splitTriangles(int32_t divisor) {  // reference/mesh.cpp:389-395
  TheMesh out;
  for (auto const &t : mMesh) util::divide(t, divisor, [&out](Triangle &&n) { out.push_back(n); });
  mMesh = std::move(out);
}

// ----------------------------------------------------------------- STL I/O
void Mesh::readMesh(std::string const &filename) {  // reference/mesh.cpp:399-415 (binary or ASCII STL)
  mMesh.clear();
  mFace2neighbours.clear();
  std::ifstream in(filename, std::ios::binary);
  if (!in) throw std::runtime_error("cannot open " + filename);
  std::string bytes((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  uint32_t declared = 0;
  if (bytes.size() >= 84) std::memcpy(&declared, bytes.data() + 80, 4);
  if (bytes.size() >= 84 && bytes.size() == 84ull + 50ull * declared) {
    for (uint32_t i = 0; i < declared; ++i) {
      float c[9];
      std::memcpy(c, bytes.data() + 84 + 50ull * i + 12, sizeof c);
      mMesh.push_back({Vertex(c[0], c[1], c[2]), Vertex(c[3], c[4], c[5]), Vertex(c[6], c[7], c[8])});
    }
    return;
  }
  char const *p = bytes.c_str();
  Triangle t;
  int corner = 0;
  while ((p = std::strstr(p, "vertex")) != nullptr) {
    p += 6;
    char *e;
    float x = std::strtof(p, &e);
    float y = std::strtof(e, &e);
    float z = std::strtof(e, &e);
    p = e;
    t[corner++] = Vertex(x, y, z);
    if (corner == 3) {
      mMesh.push_back(t);
      corner = 0;
    }
  }
}

void Mesh::writeMesh(std::string const &filename) const {  // reference/mesh.cpp:419-430
  std::ofstream out(filename);
  out << "solid Exported from Blender-2.82 (sub 7)\n";
  for (auto const &t : mMesh) {
    out << "facet normal 0.000000 0.000000 0.000000\nouter loop\n";
    for (auto const &v : t) out << "vertex " << v(0) << ' ' << v(1) << ' ' << v(2) << '\n';
    out << "endloop\nendfacet\n";
  }
  out << "endsolid Exported from Blender-2.82 (sub 7)\n";
}

// --------------------------------------------------------------- generators
void Mesh::makeSolidOfRevolution(int32_t sectors, int32_t belts, std::function<float(float)> envelope,
                                 Vector const &size) {  // reference/mesh.cpp:434-477
  mMesh.clear();
  mMesh.reserve(static_cast<uint32_t>(2 * sectors * belts));
  mFace2neighbours.clear();
  float const halfSector = cgPi / sectors;
  float const fullSector = halfSector * 2.0f;
  float const beltStep = cgPi / (belts + 1.0f);
  // three consecutive latitude rings: upper, middle, lower
  float angleMid = beltStep, angleLow = 2.0f * beltStep;
  float radiusUp = 0.0f;
  float radiusMid = size(0) * envelope(std::cos(angleMid));
  float radiusLow = size(0) * envelope(std::cos(angleLow));
  float zUp = size(2), zMid = size(2) * std::cos(angleMid), zLow = size(2) * std::cos(angleLow);
  float twist = 0.0f;
  for (int32_t belt = 0; belt < belts; ++belt) {
    float apex = twist + halfSector, left = twist + 0.0f, right = twist + fullSector;
    for (int32_t sector = 0; sector < sectors; ++sector) {
      Vertex up(radiusUp * std::sin(apex), size(1) * radiusUp * std::cos(apex), zUp);
      Vertex midL(radiusMid * std::sin(left), size(1) * radiusMid * std::cos(left), zMid);
      Vertex midR(radiusMid * std::sin(right), size(1) * radiusMid * std::cos(right), zMid);
      mMesh.push_back({up, midL, midR});
      // the lower corner applies size(0) a second time, as the reference does (mesh.cpp:460)
      Vertex low(size(0) * radiusLow * std::sin(apex), size(1) * radiusLow * std::cos(apex), zLow);
      mMesh.push_back({midL, midR, low});
      apex += fullSector;
      left = right;
      right += fullSector;
    }
    angleMid = angleLow;
    angleLow += beltStep;
    radiusUp = radiusMid;
    radiusMid = radiusLow;
    radiusLow = size(0) * envelope(std::cos(angleLow));
    zUp = zMid;
    zMid = zLow;
    zLow = size(2) * std::cos(angleLow);
    twist += halfSector;
  }
}
