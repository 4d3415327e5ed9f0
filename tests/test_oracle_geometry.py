"""The reference's unit tests (reference/googleTest.cpp, 12 gtest cases on the L1 geometry of
reference/3dGeomUtil.h) restated against the oracle, with the reference's tolerance cgEpsilon = 1e-4
(googleTest.cpp:10).  planeIntersection.Ray's second case is restated with the oracle's documented
semantics (deviation D1: mValid stays false for t < 0, mPoint is written) -- the reference's own
expectation there (googleTest.cpp:248) fails against reference/3dGeomUtil.h:284-290.
The same cases run against the product's C++ drop-in API in tests/test_cpp_dropin.py."""
import ctypes

import numpy as np
import pytest

EPS = 1e-4


def V(o, *a):
    return o.v(*a)


def T(x):
    return np.array([x.x, x.y, x.z], dtype=np.float64)


def close(a, b, eps=EPS):
    return np.linalg.norm(np.asarray(a, np.float64) - np.asarray(b, np.float64)) < eps


def test_get_aperpendicular(orc):  # googleTest.cpp:46-67
    for d in [(1, 0, 0), (1, 1, 0), (1, 0, 1), (1, -1, -1)]:
        v = np.asarray(d, np.float32)
        v = v / np.linalg.norm(v)
        p = orc.lib().orc_get_aperpendicular(V(orc, v))
        assert abs(float(np.dot(T(p), v))) < 1e-6


def _ray_err(orc, points, d=(1, 0, 0)):
    r = orc.lib().orc_ray_make(V(orc, 0, 0, 0), V(orc, d))
    pts = np.ascontiguousarray(points, np.float32).reshape(-1, 3)
    return orc.lib().orc_ray_average_error_squared(ctypes.byref(r), pts.ctypes.data if len(pts) else None, len(pts))


def test_ray_average_error_squared(orc):  # googleTest.cpp:69-85
    assert _ray_err(orc, np.zeros((0, 3))) == 0.0
    assert _ray_err(orc, [(2, 0, 0), (-3, 0, 0)]) == 0.0
    assert _ray_err(orc, [(2, 1, 0), (-3, 0, 1)]) > 0.0


def _plane_pt_normal(orc, point, d):
    n = np.asarray(d, np.float32)
    n = n / np.sqrt(np.float32((n * n).sum()))
    return orc.oplane(V(orc, n), float(np.dot(n.astype(np.float32), np.asarray(point, np.float32))))


@pytest.mark.parametrize("common,d1,d2,d3", [
    ((1, 2, 3), (1, 2, 3), (3, 1, 2), (3, 2, 1)),
    ((3, -2, 1), (1, 0, 0), (0, 1, 0), (0, 0, 1)),
    ((3, -2, -1), (1, -2, 3), (-1, 2, 3), (1, 2, -3)),
])
def test_plane_intersection_normals(orc, common, d1, d2, d3):  # googleTest.cpp:87-103
    planes = [_plane_pt_normal(orc, common, d) for d in (d1, d2, d3)]
    assert close(T(orc.lib().orc_plane_intersect3(*planes)), common)


@pytest.mark.parametrize("common,pairs", [
    ((0, 0, 0), [(0.5, (1, 0, 0)), (0.5, (0, 1, 0)), (0.5, (0, 0, 1))]),
    ((0, 0, 0), [(0.5, (1, 0, 0)), (0.2, (0, 1, 0)), (0.1, (0, 0, 1))]),
    ((-1, 2, 3), [(0.1, (10, 10, 0)), (0.2, (0, 10, 10)), (0.3, (10, 0, 10))]),
    ((-1, 2, 3), [(0.1, (-10, 10, 0)), (0.2, (0, -10, 10)), (0.3, (10, 0, 10))]),
    ((-1, 2, 3), [(0.1, (10, 10, 0)), (0.2, (0, -10, 10)), (0.3, (-10, 0, 10))]),
])
def test_plane_intersection_proportion(orc, common, pairs):  # googleTest.cpp:105-141
    c = np.asarray(common, np.float32)
    planes = []
    for prop, one in pairs:
        o = np.asarray(one, np.float32)
        other = o + np.float32(1.0 / np.float32(prop)) * (c - o)
        planes.append(orc.lib().orc_plane_from_1proportion_2points(prop, V(orc, o), V(orc, other)))
    assert close(T(orc.lib().orc_plane_intersect3(*planes)), common)


@pytest.mark.parametrize("o1,o2,o3", [
    ((10, 0, 0), (0, 10, 0), (0, 0, 10)),
    ((-10, 0, 0), (0, 10, 0), (0, 0, 10)),
    ((-10, 0, 0), (0, -10, 0), (0, 0, 10)),
    ((-10, 0, 0), (0, -10, 0), (0, 0, -10)),
])
def test_plane_intersection_vertices(orc, o1, o2, o3):  # googleTest.cpp:143-174
    c = (1, 2, 3)
    L = orc.lib()
    p1 = L.orc_plane_from_3points(V(orc, o1), V(orc, o2), V(orc, c))
    p2 = L.orc_plane_from_3points(V(orc, o2), V(orc, o3), V(orc, c))
    p3 = L.orc_plane_from_3points(V(orc, o1), V(orc, o3), V(orc, c))
    assert close(T(L.orc_plane_intersect3(p1, p2, p3)), c)


@pytest.mark.parametrize("spec", [
    [((10, 0, 0), (0, 1, 0)), ((0, 10, 0), (0, 0, 1)), ((0, 0, 10), (1, 0, 0))],
    [((10, 0, 0), (0, 1, 1)), ((0, 10, 0), (1, 0, -1)), ((0, 0, 10), (1, 1, 0))],
    [((10, 0, 0), (-4, 1, 1)), ((0, 10, 0), (1, -4, -1)), ((0, 0, 10), (1, 1, -4))],
    # planeIntersection.VectorsPoint (googleTest.cpp:220-235) calls the same 1vector2points helper
    [((10, 1, 0), (1, 10, 0)), ((0, 10, 1), (0, 1, 10)), ((1, 0, 10), (10, 0, 1))],
])
def test_plane_intersection_vector_points(orc, spec):  # googleTest.cpp:176-235
    c = (1, 2, -3)
    L = orc.lib()
    planes = [L.orc_plane_from_1vector_2points(V(orc, d), V(orc, one), V(orc, c)) for one, d in spec]
    assert close(T(L.orc_plane_intersect3(*planes)), c)


def test_plane_from_2vectors_1point(orc):  # the helper googleTest.cpp:210-218 defines but never runs
    L = orc.lib()
    c = (1, 2, -3)
    planes = [L.orc_plane_from_2vectors_1point(V(orc, a), V(orc, b), V(orc, c))
              for a, b in [((1, 0, 0), (0, 1, 0)), ((0, 1, 0), (0, 0, 1)), ((1, 0, 0), (0, 0, 1))]]
    assert close(T(L.orc_plane_intersect3(*planes)), c)


def _ray_plane(orc, start, d, p0, p1, p2):
    L = orc.lib()
    r = L.orc_ray_make(V(orc, start), V(orc, d))
    pl = L.orc_plane_from_3points(V(orc, p0), V(orc, p1), V(orc, p2))
    pt, cs, t = orc.ov3(), ctypes.c_float(), ctypes.c_float()
    valid = L.orc_plane_intersect_ray(pl, r.start, r.dir, ctypes.byref(pt), ctypes.byref(cs), ctypes.byref(t))
    return valid, T(pt), cs.value, t.value


def test_plane_intersection_ray(orc):  # googleTest.cpp:237-265
    valid, _, _, _ = _ray_plane(orc, (1, 2, -3), (1, 1, 1), (10, 1, 2), (11, 11.1, 2), (12, 1.1, 4.4))
    assert valid
    # reference expects mValid with a negative distance here; the reference code (and D1) gives
    # mValid == false with the negative distance still reported
    valid, _, _, t = _ray_plane(orc, (1, 2, -3), (-1, 2, 3), (10, 1, 2), (11, 11.1, 2), (12, 1.1, 4.4))
    assert not valid and t < 0.0
    valid, _, _, _ = _ray_plane(orc, (1, 2, -3), (0, 2, 0), (10, 1, 2), (10, 11.1, 2), (10, 1.1, 4.4))
    assert not valid
    valid, pt, cs, _ = _ray_plane(orc, (1, 2, -3), (0, 2, 0), (10, 10, 2), (0, 10, 2), (10, 10, 10.4))
    assert valid and np.linalg.norm(pt - (1, 10, -3)) < 1e-5 and abs(cs) > 0.9999


@pytest.mark.parametrize("point,tri,expected", [
    ((0, 0, 0), ((2, 0, 0), (0, 2, 0), (0, 0, 2)), (0.666666, 0.666666, 0.666666)),
    ((0, 0, 0), ((2, 0, 0), (2, 1, 0), (2, 0, 1)), (2, 0, 0)),
    ((1, 2, 3), ((3, 2, 3), (1, 4, 3), (1, 2, 5)), (1.666666, 2.666666, 3.666666)),
    ((-1, -2, 3), ((1, -2, 3), (1, -3, 3), (1, -2, 4)), (1, -2, 3)),
    ((1.666666, 2.666666, 3.666666), ((3, 2, 3), (1, 4, 3), (1, 2, 5)), (1.666666, 2.666666, 3.666666)),
])
def test_plane_projection(orc, point, tri, expected):  # googleTest.cpp:267-298
    L = orc.lib()
    pl = L.orc_plane_from_3points(*[V(orc, p) for p in tri])
    assert close(T(L.orc_plane_project(pl, V(orc, point))), expected)


@pytest.mark.parametrize("point,tri,expected", [
    ((0, 0, 0), ((2, 0, 0), (0, 2, 0), (0, 0, 2)), 1.15468),
    ((0, 0, 0), ((2, 0, 0), (2, 1, 0), (2, 0, 1)), 2.0),
    ((1, 2, 3), ((3, 2, 3), (1, 4, 3), (1, 2, 5)), 1.15468),
    ((-1, -2, 3), ((1, -2, 3), (1, -3, 3), (1, -2, 4)), 2.0),
    ((1.666666, 2.666666, 3.666666), ((3, 2, 3), (1, 4, 3), (1, 2, 5)), 0.0),
])
def test_plane_distance(orc, point, tri, expected):  # googleTest.cpp:300-331
    L = orc.lib()
    pl = L.orc_plane_from_3points(*[V(orc, p) for p in tri])
    assert abs(abs(L.orc_plane_distance(pl, V(orc, point))) - expected) < EPS


@pytest.mark.parametrize("step,expected", [((1, 0, 0), 2), ((0, 1, 0), 1), ((-1, -1, 0), 0)])
def test_to_which_side(orc, step, expected):  # googleTest.cpp:333-353
    L = orc.lib()
    t0, t1, t2 = np.float32([3, 2, 5]), np.float32([1, 4, 5]), np.float32([6, 5, 5])
    start = (t0 + t1 + t2) / np.float32(3)
    end = start + np.float32(step)
    m = np.empty(9, np.float32)
    L.orc_barycentric_inverse(V(orc, t0), V(orc, t1), V(orc, t2), m.ctypes.data)
    bs = L.orc_matvec(m.ctypes.data, V(orc, start))
    be = L.orc_matvec(m.ctypes.data, V(orc, end))
    assert L.orc_to_which_side(bs, be) == expected
