"""The product's host preprocessing (libbzr's C++ Mesh / BezierMesh, reached through the C ABI)
against the oracle's restatement: triangles, neighbour tables and the 264-byte patch records must be
bit-identical after every step of every recipe the configs and the reference's harnesses use.
(a self-contained drop-in needs the meshes built on the GPU box.)"""
import numpy as np
import pytest

from bzr_amd.configs import CONFIGS, build_lens


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def same(a, b):
    return a.shape == b.shape and np.array_equal(bits(a), bits(b))


@pytest.mark.parametrize("name", ["cfg1", "cfg2", "cfg3", "cfg4"])
def test_config_patches_bit_identical(bzr, orc, name):
    for lens in CONFIGS[name].lenses:
        a = build_lens(bzr.TriMesh, lens)
        b = build_lens(orc.OMesh, lens)
        assert same(a.triangles, b.triangles)
        fa, sa = a.neighbours()
        fb, sb = b.neighbours()
        assert np.array_equal(fa, fb) and np.array_equal(sa, sb)
        assert same(a.bezier_patches(), b.bezier_patches())


@pytest.mark.slow
def test_cfg5_patches_bit_identical(bzr, orc):
    lens = CONFIGS["cfg5"].lenses[0]
    a = build_lens(bzr.TriMesh, lens).bezier_patches()
    b = build_lens(orc.OMesh, lens).bezier_patches()
    assert a.shape == (301056, 66) and same(a, b)


@pytest.mark.parametrize("sectors,belts,size", [(3, 1, (1, 1, 1)), (7, 3, (1, 4, 2)), (15, 5, (1, 4, 2)),
                                                (21, 15, (1, 4, 2)), (5, 3, (1, 0.5, 0.25))])
def test_ellipsoid_pipeline(bzr, orc, sectors, belts, size):
    a = bzr.TriMesh().make_ellipsoid(sectors, belts, size)
    b = orc.OMesh().make_ellipsoid(sectors, belts, size)
    assert same(a.triangles, b.triangles)
    a.standardize_vertices()
    b.standardize_vertices()
    assert same(a.triangles, b.triangles)
    a.standardize_normals()
    b.standardize_normals()
    assert same(a.triangles, b.triangles)
    assert same(a.bezier_patches(), b.bezier_patches())


def test_split_thick_and_interpolate(bzr, orc):
    """measureApproximation's loop (reference/test.cpp:429-445) step by step."""
    a = bzr.TriMesh().make_ellipsoid(7, 3, (1, 4, 2)).standardize()
    b = orc.OMesh().make_ellipsoid(7, 3, (1, 4, 2)).standardize()
    for _ in range(2):
        a = a.bezier_split_thick()
        b = b.bezier_split_thick()
        assert same(a.triangles, b.triangles)
        a.standardize()
        b.standardize()
        assert same(a.triangles, b.triangles)
    assert same(a.bezier_interpolate(3).triangles, b.bezier_interpolate(3).triangles)


def test_test_lens_envelope_and_transforms(bzr, orc):
    """testBezierRefraction's solid of revolution (reference/test.cpp:336-339), moved and scaled."""
    a = bzr.TriMesh().make_solid_of_revolution(21, 15, bzr.ENVELOPE_TESTLENS, (1, 4, 2))
    b = orc.OMesh().make_solid_of_revolution(21, 15, 1, (1, 4, 2))
    assert same(a.triangles, b.triangles)
    m = np.diag([1.5, 0.5, 2.0]).astype(np.float32)
    m[0, 1] = 0.25
    a.transform(m, (10, -1, 0.5)).standardize()
    b.transform(m, (10, -1, 0.5)).standardize()
    assert same(a.triangles, b.triangles)
    assert same(a.bezier_patches(), b.bezier_patches())


def test_split_maxside(bzr, orc):
    a = bzr.TriMesh().make_unit_sphere(4, 2).transform(np.eye(3) * 13).split_maxside(11.0)
    b = orc.OMesh().make_unit_sphere(4, 2).transform(np.eye(3) * 13).split_maxside(11.0)
    assert len(a) > 16 and same(a.triangles, b.triangles)


def test_stl_roundtrip_and_robot(bzr, orc, tmp_path):
    """Mesh::readMesh on the reference's binary robot.stl and on an ASCII file written by writeMesh."""
    from bzr_amd.configs import ROBOT_STL
    a = bzr.TriMesh().read_stl(ROBOT_STL)
    b = orc.OMesh().read_stl(ROBOT_STL)
    assert len(a) == 150 and same(a.triangles, b.triangles)
    sphere = bzr.TriMesh().make_unit_sphere(7, 7)
    path = tmp_path / "sphere.stl"
    sphere.write_stl(path)
    text = path.read_text()
    assert text.startswith("solid Exported from Blender-2.82 (sub 7)\nfacet normal 0.000000 0.000000 0.000000")
    back = bzr.TriMesh().read_stl(path)
    obak = orc.OMesh().read_stl(path)
    assert len(back) == len(sphere) and same(back.triangles, obak.triangles)
    assert np.allclose(back.triangles, sphere.triangles, atol=1e-5)  # 6 significant digits, like the reference


def test_vertex_on_edge_is_reported(bzr, orc):
    """reference/mesh.cpp:204 throws "Vertex on edge detected." for an open mesh: the C ABI reports it."""
    t = np.array([[[0, 0, 0], [1, 0, 0], [0, 1, 0]]], np.float32)
    a = bzr.TriMesh()
    a.triangles = t
    with pytest.raises(bzr.BzrError, match="Vertex on edge detected"):
        a.standardize_normals()
    b = orc.OMesh()
    b.triangles = t
    with pytest.raises(RuntimeError, match="Vertex on edge detected"):
        b.standardize_normals()


def test_makeEllipsoid_nonunit_x_is_not_watertight(bzr):
    """makeEllipsoid double-applies aSize(0) (reference/mesh.cpp:456-460), so a size with
    x != 1 leaves cracks and standardizeNormals throws -- reproduced, not "fixed"."""
    with pytest.raises(bzr.BzrError, match="Vertex on edge"):
        bzr.TriMesh().make_ellipsoid(8, 4, (2, 1, 1)).standardize()


@pytest.mark.parametrize("seed", list(range(12)))
def test_random_recipes_bit_identical(bzr, orc, seed):
    """The fuzz lenses' recipe (tests/test_gpu_fuzz.py: random sectors, belts and sizes -- x sizes other than 1
    too, which the reference refuses -- the test-lens envelope, a random stretch, rotation and displacement):
    product and oracle agree on refusing, and otherwise on every triangle, neighbour and patch word."""
    rng = np.random.default_rng(7000 + seed)
    sectors, belts = int(rng.integers(3, 41)), int(rng.integers(2, 25))
    size = (1.0 if seed % 4 else float(rng.integers(2, 4)), float(rng.integers(1, 6)), float(rng.integers(1, 6)))
    q = rng.normal(size=4)
    w, x, y, z = q / np.linalg.norm(q)
    rot = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                    [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                    [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]], np.float32)
    rot *= np.float32(rng.uniform(0.5, 3.0))
    disp = rng.uniform(-20, 20, 3)
    out = []
    for cls in (bzr.TriMesh, orc.OMesh):
        m = cls()
        if seed % 3 == 2:
            m.make_solid_of_revolution(sectors, belts, bzr.ENVELOPE_TESTLENS, size)
        else:
            m.make_ellipsoid(sectors, belts, size)
        m.transform(rot, disp)
        try:
            m.standardize()
            out.append((m.triangles, m.neighbours(), m.bezier_patches()))
        except (bzr.BzrError, RuntimeError) as e:
            assert "Vertex on edge" in str(e)
            out.append(None)
    a, b = out
    assert (a is None) == (b is None)
    if a is not None:
        assert same(a[0], b[0]) and np.array_equal(a[1][0], b[1][0]) and np.array_equal(a[1][1], b[1][1])
        assert same(a[2], b[2])
