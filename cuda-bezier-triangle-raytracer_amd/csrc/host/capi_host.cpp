// capi_host.cpp -- C ABI over the host preprocessing (Mesh, BezierMesh construction).
// Every entry point catches what the drop-in classes throw (the reference throws
// char const* and std::out_of_range, reference/mesh.cpp:204, bezierMesh.cpp:17-18)
// and reports it as a status code + bzr_last_error() text.
#include <cstring>
#include <new>
#include <string>

#include "bzr/bzr.hpp"

extern "C" void bzr_internal_set_error(const char *msg);

struct bzr_trimesh {
  Mesh mesh;
};

namespace {
template <typename F>
bzr_status guarded(F &&f) {
  try {
    f();
    return BZR_OK;
  } catch (char const *what) {
    bzr_internal_set_error(what);
    return BZR_ERR_PREPROCESS;
  } catch (std::bad_alloc const &) {
    bzr_internal_set_error("out of memory");
    return BZR_ERR_OUT_OF_MEMORY;
  } catch (std::out_of_range const &e) {
    bzr_internal_set_error((std::string("std::out_of_range: ") + e.what()).c_str());
    return BZR_ERR_PREPROCESS;
  } catch (std::exception const &e) {
    bzr_internal_set_error(e.what());
    return BZR_ERR_PREPROCESS;
  }
}
bzr_status bad(const char *msg) {
  bzr_internal_set_error(msg);
  return BZR_ERR_INVALID_ARGUMENT;
}
}  // namespace

extern "C" {

bzr_status bzr_trimesh_create(bzr_trimesh **out) {
  if (!out) return bad("null out");
  *out = new (std::nothrow) bzr_trimesh();
  return *out ? BZR_OK : BZR_ERR_OUT_OF_MEMORY;
}

bzr_status bzr_trimesh_destroy(bzr_trimesh *m) {
  delete m;
  return BZR_OK;
}

bzr_status bzr_trimesh_copy(const bzr_trimesh *src, bzr_trimesh **out) {
  if (!src || !out) return bad("null argument");
  return guarded([&] { *out = new bzr_trimesh(*src); });
}

bzr_status bzr_trimesh_size(const bzr_trimesh *m, uint32_t *n) {
  if (!m || !n) return bad("null argument");
  *n = static_cast<uint32_t>(m->mesh.size());
  return BZR_OK;
}

bzr_status bzr_trimesh_get(const bzr_trimesh *m, float *xyz) {
  if (!m || (!xyz && m->mesh.size())) return bad("null argument");
  for (uint32_t f = 0; f < m->mesh.size(); ++f)
    for (uint32_t k = 0; k < 3; ++k) std::memcpy(xyz + 9 * f + 3 * k, m->mesh[f][k].data(), 12);
  return BZR_OK;
}

bzr_status bzr_trimesh_set(bzr_trimesh *m, const float *xyz, uint32_t n) {
  if (!m || (!xyz && n)) return bad("null argument");
  return guarded([&] {
    Mesh fresh;
    fresh.reserve(n);
    for (uint32_t f = 0; f < n; ++f) {
      Triangle t;
      for (uint32_t k = 0; k < 3; ++k) t[k] = Vertex(xyz[9 * f + 3 * k], xyz[9 * f + 3 * k + 1], xyz[9 * f + 3 * k + 2]);
      fresh.push_back(t);
    }
    m->mesh = std::move(fresh);
  });
}

bzr_status bzr_trimesh_make_solid_of_revolution(bzr_trimesh *m, int32_t sectors, int32_t belts, int32_t envelope,
                                                float sx, float sy, float sz) {
  if (!m) return bad("null mesh");
  if (sectors < 1 || belts < 1) return bad("sectors and belts must be positive");
  std::function<float(float)> env;
  if (envelope == BZR_ENVELOPE_ELLIPSOID) {
    env = [](float x) { return std::sqrt(1 - x * x); };  // reference/mesh.h:99
  } else if (envelope == BZR_ENVELOPE_TESTLENS) {
    env = [](float x) {  // reference/test.cpp:242-245, 336-339
      float x2 = x * x;
      return std::sqrt(1.0f - x2) + 0.7f * (std::exp(-4.0f) - std::exp(-4.0f * x2));
    };
  } else {
    return bad("unknown envelope");
  }
  return guarded([&] { m->mesh.makeSolidOfRevolution(sectors, belts, env, Vector(sx, sy, sz)); });
}

bzr_status bzr_trimesh_make_ellipsoid(bzr_trimesh *m, int32_t sectors, int32_t belts, float sx, float sy, float sz) {
  if (!m) return bad("null mesh");
  if (sectors < 1 || belts < 1) return bad("sectors and belts must be positive");
  return guarded([&] { m->mesh.makeEllipsoid(sectors, belts, Vector(sx, sy, sz)); });
}

bzr_status bzr_trimesh_read_stl(bzr_trimesh *m, const char *path) {
  if (!m || !path) return bad("null argument");
  return guarded([&] { m->mesh.readMesh(path); });
}

bzr_status bzr_trimesh_write_stl(const bzr_trimesh *m, const char *path) {
  if (!m || !path) return bad("null argument");
  return guarded([&] { m->mesh.writeMesh(path); });
}

bzr_status bzr_trimesh_transform(bzr_trimesh *m, const float t[9], const float d[3]) {
  if (!m || !t || !d) return bad("null argument");
  Transform tr;
  std::memcpy(tr.data(), t, 36);
  return guarded([&] { m->mesh.transform(tr, Vertex(d[0], d[1], d[2])); });
}

bzr_status bzr_trimesh_split(bzr_trimesh *m, int32_t divisor) {
  if (!m) return bad("null mesh");
  if (divisor < 1) return bad("divisor must be >= 1");
  return guarded([&] { m->mesh.splitTriangles(divisor); });
}

bzr_status bzr_trimesh_split_maxside(bzr_trimesh *m, float max_side) {
  if (!m) return bad("null mesh");
  if (!(max_side > 0.0f)) return bad("max_side must be > 0");
  return guarded([&] { m->mesh.splitTriangles(max_side); });
}

bzr_status bzr_trimesh_standardize_vertices(bzr_trimesh *m) {
  if (!m) return bad("null mesh");
  return guarded([&] { m->mesh.standardizeVertices(); });
}

bzr_status bzr_trimesh_standardize_normals(bzr_trimesh *m) {
  if (!m) return bad("null mesh");
  return guarded([&] { m->mesh.standardizeNormals(); });
}

bzr_status bzr_trimesh_neighbours(const bzr_trimesh *m, uint32_t *fellow, uint8_t *start) {
  if (!m || !fellow || !start) return bad("null argument");
  auto const &f2n = m->mesh.getFace2neighbours();
  if (f2n.size() != m->mesh.size()) return bad("mesh is not standardized");
  for (std::size_t f = 0; f < f2n.size(); ++f)
    for (int k = 0; k < 3; ++k) {
      fellow[3 * f + k] = f2n[f].mFellowTriangles[k];
      start[3 * f + k] = f2n[f].mFellowCommonSideStarts[k];
    }
  return BZR_OK;
}

bzr_status bzr_bezier_build(const bzr_trimesh *m, bzr_patch *out) {
  if (!m || (!out && m->mesh.size())) return bad("null argument");
  return guarded([&] {
    BezierMesh bm(m->mesh);
    if (bm.size()) std::memcpy(static_cast<void *>(out), &bm[0], sizeof(bzr_patch) * bm.size());
  });
}

bzr_status bzr_bezier_split_thick(const bzr_trimesh *m, bzr_trimesh *out) {
  if (!m || !out) return bad("null argument");
  return guarded([&] { out->mesh = BezierMesh(m->mesh).splitThickBezierTriangles(); });
}

bzr_status bzr_bezier_interpolate(const bzr_trimesh *m, int32_t divisor, bzr_trimesh *out) {
  if (!m || !out) return bad("null argument");
  if (divisor < 1) return bad("divisor must be >= 1");
  return guarded([&] { out->mesh = BezierMesh(m->mesh).interpolate(divisor); });
}

}  // extern "C"
