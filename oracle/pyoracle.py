"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper of oracle/liboracle.so.

The CPU restatement of the reference (see bzr_oracle.h for its contract and
pinning status).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg use it, always as the checker or the CPU baseline, never as
the thing measured or shipped.
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
LIB_PATH = ORACLE_DIR / "liboracle.so"
PATCH_WORDS = 66


class ov3(ctypes.Structure):
    _fields_ = [("x", ctypes.c_float), ("y", ctypes.c_float), ("z", ctypes.c_float)]


class omesh(ctypes.Structure):
    _fields_ = [
        ("tri", ctypes.c_void_p), ("n", ctypes.c_uint32), ("cap", ctypes.c_uint32),
        ("f2n", ctypes.c_void_p), ("nf2n", ctypes.c_uint32),
        ("nrm_key", ctypes.c_void_p), ("nrm_val", ctypes.c_void_p), ("nnrm", ctypes.c_uint32),
    ]


class oplane(ctypes.Structure):
    _fields_ = [("n", ov3), ("c", ctypes.c_float)]


class ohit(ctypes.Structure):
    _fields_ = [("t", ctypes.c_float), ("point", ov3), ("cos_inc", ctypes.c_float), ("bary", ov3),
                ("normal", ov3), ("what", ctypes.c_uint32), ("patch", ctypes.c_uint32)]


class oray(ctypes.Structure):
    _fields_ = [("start", ov3), ("dir", ov3)]


_lib = None
_P = ctypes.c_void_p
_MP = ctypes.POINTER(omesh)


def build(force: bool = False) -> Path:
    newest = max((ORACLE_DIR / f).stat().st_mtime for f in ("bzr_oracle.c", "illum_oracle.c", "bzr_oracle.h"))
    if force or not LIB_PATH.exists() or LIB_PATH.stat().st_mtime < newest:
        subprocess.run(["make", "-C", str(ORACLE_DIR)], check=True, capture_output=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = _configure(ctypes.CDLL(str(LIB_PATH)))
    return _lib


def load_variant(cflags: str, tag: str):
    """The oracle compiled with other flags (e.g. "-O3 -march=native" for bench.py's CPU baseline) into
    a private temporary library; returns its configured handle.  Compiled where it runs (-march=native
    must describe the host that times it)."""
    import os
    import tempfile

    out = Path(tempfile.gettempdir()) / f"bzr_oracle_{tag}_{os.getuid()}_{os.getpid()}.so"
    cmd = ["gcc", *cflags.split(), "-std=c11", "-fPIC", "-ffp-contract=off", "-fopenmp", "-shared", "-o", str(out),
           str(ORACLE_DIR / "bzr_oracle.c"), str(ORACLE_DIR / "illum_oracle.c"), "-lm"]
    subprocess.run(cmd, check=True, capture_output=True)
    try:
        return _configure(ctypes.CDLL(str(out)))
    finally:
        out.unlink(missing_ok=True)  # the mapping stays valid


def _configure(L):
    if True:
        sig = {
            "orc_last_error": ([], ctypes.c_char_p),
            "orc_mesh_init": ([_MP], None),
            "orc_mesh_free": ([_MP], None),
            "orc_mesh_copy": ([_MP, _MP], ctypes.c_int),
            "orc_mesh_push": ([_MP, _P], ctypes.c_int),
            "orc_mesh_make_solid_of_revolution": ([_MP, ctypes.c_int32, ctypes.c_int32, ctypes.c_int, ov3], ctypes.c_int),
            "orc_mesh_make_ellipsoid": ([_MP, ctypes.c_int32, ctypes.c_int32, ov3], ctypes.c_int),
            "orc_mesh_standardize_vertices": ([_MP], ctypes.c_int),
            "orc_mesh_standardize_normals": ([_MP], ctypes.c_int),
            "orc_mesh_transform": ([_MP, _P, ov3], None),
            "orc_mesh_split_divisor": ([_MP, ctypes.c_int32], ctypes.c_int),
            "orc_mesh_split_maxside": ([_MP, ctypes.c_float], ctypes.c_int),
            "orc_mesh_read_stl": ([_MP, ctypes.c_char_p], ctypes.c_int),
            "orc_mesh_write_stl": ([_MP, ctypes.c_char_p], ctypes.c_int),
            "orc_mesh_unique_vertices": ([_MP, _P], ctypes.c_uint32),
            "orc_bezier_build": ([_MP, _P], ctypes.c_int),
            "orc_bezier_interpolate_mesh": ([_P, ctypes.c_uint32, ctypes.c_int32, _MP], ctypes.c_int),
            "orc_bezier_split_thick": ([_P, ctypes.c_uint32, _MP, _MP], ctypes.c_int),
            "orc_patch_intersect": ([_P, ctypes.POINTER(oray), ctypes.c_int], ohit),
            "orc_mesh_intersect": ([_P, ctypes.c_uint32, ctypes.POINTER(oray)], ohit),
            "orc_intersect_batch": ([_P, ctypes.c_uint32, _P, ctypes.c_uint32, _P, ctypes.c_int], None),
            "orc_refract_batch": ([_P, ctypes.c_uint32, ctypes.c_float, _P, _P, ctypes.c_uint32, _P, _P, ctypes.c_int], None),
            "orc_trace_chain_batch": ([_P, _P, _P, ctypes.c_uint32, _P, ctypes.c_uint32, _P, _P, _P, ctypes.c_int], None),
            "orc_measure_approximation": ([ctypes.c_uint32, ctypes.c_int32, ctypes.c_int32, ov3, ctypes.c_int32,
                                           ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
            "orc_debug_uset_order": ([_P, ctypes.c_uint32, _P], ctypes.c_uint32),
            "orc_counters": ([_P], None),
            "orc_planar_gate_batch": ([_P, ctypes.c_uint32, _P, ctypes.c_uint32, _P, ctypes.c_int], None),
            "orc_counters_reset": ([], None),
            "orc_hemisphere_create": ([ctypes.c_uint32], _P),
            "orc_hemisphere_free": ([_P], None),
            "orc_hemisphere_patch_count": ([_P], ctypes.c_uint32),
            "orc_hemisphere_random": ([_P, _P], ctypes.c_uint32),
            "orc_emit": ([_P, ctypes.c_uint64, ctypes.c_uint32, _P, _P], ctypes.c_int),
            "orc_land": ([_P, _P, _P, ctypes.c_uint32, _P, _P, _P], None),
            "orc_plane_from_1proportion_2points": ([ctypes.c_float, ov3, ov3], oplane),
            "orc_plane_from_3points": ([ov3, ov3, ov3], oplane),
            "orc_plane_from_1vector_2points": ([ov3, ov3, ov3], oplane),
            "orc_plane_from_2vectors_1point": ([ov3, ov3, ov3], oplane),
            "orc_plane_intersect3": ([oplane, oplane, oplane], ov3),
            "orc_plane_intersect_ray": ([oplane, ov3, ov3, ctypes.POINTER(ov3), ctypes.POINTER(ctypes.c_float),
                                         ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
            "orc_plane_project": ([oplane, ov3], ov3),
            "orc_plane_distance": ([oplane, ov3], ctypes.c_float),
            "orc_barycentric_inverse": ([ov3, ov3, ov3, _P], None),
            "orc_matvec": ([_P, ov3], ov3),
            "orc_to_which_side": ([ov3, ov3], ctypes.c_uint32),
            "orc_get_aperpendicular": ([ov3], ov3),
            "orc_ray_make": ([ov3, ov3], oray),
            "orc_ray_average_error_squared": ([ctypes.POINTER(oray), _P, ctypes.c_uint32], ctypes.c_float),
        }
        for name, (args, ret) in sig.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = ret
    return L


def v(x, y=None, z=None) -> ov3:
    if y is None:
        x, y, z = x
    return ov3(float(x), float(y), float(z))


def tup(a: ov3):
    return (a.x, a.y, a.z)


def _err():
    return lib().orc_last_error().decode()


class OMesh:
    """Oracle triangle mesh (the reference's Mesh)."""

    def __init__(self):
        self.m = omesh()
        lib().orc_mesh_init(ctypes.byref(self.m))

    def __del__(self):
        try:
            lib().orc_mesh_free(ctypes.byref(self.m))
        except Exception:
            pass

    def __len__(self):
        return self.m.n

    @property
    def triangles(self) -> np.ndarray:
        if self.m.n == 0:
            return np.zeros((0, 3, 3), np.float32)
        buf = (ctypes.c_float * (9 * self.m.n)).from_address(self.m.tri)
        return np.frombuffer(buf, dtype=np.float32).reshape(-1, 3, 3).copy()

    @triangles.setter
    def triangles(self, tris):
        t = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 3, 3)
        lib().orc_mesh_free(ctypes.byref(self.m))
        lib().orc_mesh_init(ctypes.byref(self.m))
        for k in range(len(t)):
            lib().orc_mesh_push(ctypes.byref(self.m), t[k].ctypes.data)

    def neighbours(self):
        n = self.m.nf2n
        raw = np.frombuffer((ctypes.c_uint8 * (16 * n)).from_address(self.m.f2n), dtype=np.uint8).reshape(n, 16)
        fellow = raw[:, :12].copy().view(np.uint32).reshape(n, 3)
        start = raw[:, 12:15].copy()
        return fellow, start

    def _rc(self, rc):
        if rc != 0:
            raise RuntimeError(_err())
        return self

    def make_ellipsoid(self, sectors, belts, size=(1, 1, 1)):
        return self._rc(lib().orc_mesh_make_ellipsoid(ctypes.byref(self.m), sectors, belts, v(size)))

    def make_unit_sphere(self, sectors, belts):
        return self.make_ellipsoid(sectors, belts, (1, 1, 1))

    def make_solid_of_revolution(self, sectors, belts, envelope, size):
        return self._rc(lib().orc_mesh_make_solid_of_revolution(ctypes.byref(self.m), sectors, belts, envelope, v(size)))

    def read_stl(self, path):
        return self._rc(lib().orc_mesh_read_stl(ctypes.byref(self.m), str(path).encode()))

    def write_stl(self, path):
        return self._rc(lib().orc_mesh_write_stl(ctypes.byref(self.m), str(path).encode()))

    def transform(self, matrix=None, displacement=(0, 0, 0)):
        m = np.eye(3, dtype=np.float32) if matrix is None else np.asarray(matrix, dtype=np.float32)
        cm = np.ascontiguousarray(m.T.reshape(-1))
        lib().orc_mesh_transform(ctypes.byref(self.m), cm.ctypes.data, v(displacement))
        return self

    def translate(self, d):
        return self.transform(None, d)

    def split(self, divisor):
        return self._rc(lib().orc_mesh_split_divisor(ctypes.byref(self.m), divisor))

    def split_maxside(self, s):
        return self._rc(lib().orc_mesh_split_maxside(ctypes.byref(self.m), float(s)))

    def standardize_vertices(self):
        return self._rc(lib().orc_mesh_standardize_vertices(ctypes.byref(self.m)))

    def standardize_normals(self):
        return self._rc(lib().orc_mesh_standardize_normals(ctypes.byref(self.m)))

    def standardize(self):
        return self.standardize_vertices().standardize_normals()

    def unique_vertices(self) -> np.ndarray:
        n = lib().orc_mesh_unique_vertices(ctypes.byref(self.m), None)
        out = np.empty((n, 3), np.float32)
        lib().orc_mesh_unique_vertices(ctypes.byref(self.m), out.ctypes.data)
        return out

    def bezier_patches(self) -> np.ndarray:
        out = np.empty((3 * self.m.n, PATCH_WORDS), dtype=np.float32)
        self._rc(lib().orc_bezier_build(ctypes.byref(self.m), out.ctypes.data))
        return out

    def bezier_split_thick(self) -> "OMesh":
        p = self.bezier_patches()
        out = OMesh()
        lib().orc_mesh_free(ctypes.byref(out.m))
        if lib().orc_bezier_split_thick(p.ctypes.data, len(p), ctypes.byref(self.m), ctypes.byref(out.m)):
            raise RuntimeError(_err())
        return out

    def bezier_interpolate(self, divisor) -> "OMesh":
        p = self.bezier_patches()
        out = OMesh()
        lib().orc_mesh_free(ctypes.byref(out.m))
        lib().orc_bezier_interpolate_mesh(p.ctypes.data, len(p), divisor, ctypes.byref(out.m))
        return out


# ------------------------------------------------------------------ hot path
def intersect(patches: np.ndarray, rays: np.ndarray, threads: int = 0, L=None) -> np.ndarray:
    p = np.ascontiguousarray(patches, dtype=np.float32)
    r = np.ascontiguousarray(rays, dtype=np.float32)
    n = r.shape[1]
    out = np.empty((13, n), np.float32)
    (L or lib()).orc_intersect_batch(p.ctypes.data, len(p), r.ctypes.data, n, out.ctypes.data, threads)
    return out


def patch_intersect(patches: np.ndarray, idx, limit, rays: np.ndarray) -> np.ndarray:
    """BezierTriangle::intersect per (patch, ray, limit); returns hits [13, n] with every field as computed."""
    p = np.ascontiguousarray(patches, dtype=np.float32)
    r = np.ascontiguousarray(rays, dtype=np.float32)
    n = r.shape[1]
    out = np.empty((13, n), np.float32)
    u = out.view(np.uint32)
    for i in range(n):
        ray = oray(v(r[0, i], r[1, i], r[2, i]), v(r[3, i], r[4, i], r[5, i]))
        h = lib().orc_patch_intersect(p[int(idx[i])].ctypes.data, ctypes.byref(ray), int(limit[i]))
        out[:11, i] = (h.t, h.point.x, h.point.y, h.point.z, h.cos_inc, h.bary.x, h.bary.y, h.bary.z,
                       h.normal.x, h.normal.y, h.normal.z)
        u[11, i] = h.what
        u[12, i] = int(idx[i])
    return out


def refract(patches, ri, rays, expected, threads=0):
    p = np.ascontiguousarray(patches, dtype=np.float32)
    r = np.ascontiguousarray(rays, dtype=np.float32)
    e = np.ascontiguousarray(expected, dtype=np.uint32)
    n = r.shape[1]
    o = np.empty((6, n), np.float32)
    s = np.empty(n, np.uint32)
    lib().orc_refract_batch(p.ctypes.data, len(p), float(ri), r.ctypes.data, e.ctypes.data, n, o.ctypes.data,
                            s.ctypes.data, threads)
    return o, s


def trace_chain(lenses, ri, rays, threads=0, L=None):
    ps = [np.ascontiguousarray(p, dtype=np.float32) for p in lenses]
    ptrs = (ctypes.c_void_p * len(ps))(*[p.ctypes.data for p in ps])
    nps = (ctypes.c_uint32 * len(ps))(*[len(p) for p in ps])
    ris = (ctypes.c_float * len(ps))(*[float(x) for x in ri])
    r = np.ascontiguousarray(rays, dtype=np.float32)
    n = r.shape[1]
    o = np.empty((6, n), np.float32)
    s = np.empty(n, np.uint32)
    g = np.empty(n, np.uint32)
    (L or lib()).orc_trace_chain_batch(ctypes.cast(ptrs, ctypes.c_void_p), ctypes.cast(nps, ctypes.c_void_p),
                                ctypes.cast(ris, ctypes.c_void_p), len(ps), r.ctypes.data, n, o.ctypes.data,
                                s.ctypes.data, g.ctypes.data, threads)
    return o, s, g


def planar_gate(patches, rays, threads=0) -> np.ndarray:
    """bool [n_rays, n_patches]: the planar gate of BezierTriangle::intersect (reference/bezierTriangle.cpp:124-131)."""
    p = np.ascontiguousarray(patches, dtype=np.float32)
    r = np.ascontiguousarray(rays, dtype=np.float32)
    out = np.zeros((r.shape[1], len(p)), np.uint8)
    lib().orc_planar_gate_batch(p.ctypes.data, len(p), r.ctypes.data, r.shape[1], out.ctypes.data, threads)
    return out.astype(bool)


def counters_reset():
    lib().orc_counters_reset()


def counters() -> dict:
    """Work done since counters_reset(): planar tests, Newton runs, follow-side retries, intersect calls."""
    out = np.zeros(4, np.uint64)
    lib().orc_counters(out.ctypes.data)
    return dict(zip(("tests", "newton", "follow", "segments"), map(int, out)))


def measure_approximation(split_steps, sectors, belts, size, divisor) -> float:
    e = ctypes.c_float(0)
    rc = lib().orc_measure_approximation(split_steps, sectors, belts, v(size), divisor, ctypes.byref(e))
    if rc:
        raise RuntimeError(_err())
    return e.value


# ------------------------------------------------------------------ illumination ends (illum_oracle.c)
class Emitter(ctypes.Structure):
    """orc_emitter (same layout as libbzr's bzr_emitter)."""
    _fields_ = [("origin", ctypes.c_float * 3), ("edge_u", ctypes.c_float * 3), ("edge_v", ctypes.c_float * 3),
                ("parts_u", ctypes.c_uint32), ("parts_v", ctypes.c_uint32), ("points_per_part", ctypes.c_uint32),
                ("rays_per_point", ctypes.c_uint32), ("belts", ctypes.c_uint32), ("seed", ctypes.c_uint64)]


class Target(ctypes.Structure):
    """orc_target (same layout as libbzr's bzr_target)."""
    _fields_ = [("origin", ctypes.c_float * 3), ("axis_u", ctypes.c_float * 3), ("axis_v", ctypes.c_float * 3),
                ("size_u", ctypes.c_float), ("size_v", ctypes.c_float), ("bins_u", ctypes.c_uint32),
                ("bins_v", ctypes.c_uint32)]


def emit(em: Emitter, first: int, n: int):
    """Rays first .. first+n-1 of the counter-based emitter -> (rays [6, n], hemisphere patch [n])."""
    rays = np.empty((6, n), np.float32)
    patch = np.empty(n, np.uint32)
    if lib().orc_emit(ctypes.byref(em), first, n, rays.ctypes.data, patch.ctypes.data):
        raise RuntimeError("orc_emit: bad emitter")
    return rays, patch


def land(tg: Target, rays: np.ndarray, status: np.ndarray, hist: np.ndarray | None = None):
    """Bin the rays with status OUTSIDE on the target -> (hist [bins_v, bins_u] uint32, exited, landed)."""
    r = np.ascontiguousarray(rays, np.float32)
    s = np.ascontiguousarray(status, np.uint32)
    h = np.zeros((tg.bins_v, tg.bins_u), np.uint32) if hist is None else hist
    ex, la = ctypes.c_uint64(0), ctypes.c_uint64(0)
    lib().orc_land(ctypes.byref(tg), r.ctypes.data, s.ctypes.data, r.shape[1], h.ctypes.data, ctypes.byref(ex),
                   ctypes.byref(la))
    return h, ex.value, la.value


class Hemisphere:
    """UniformHemisphere (reference/hostUtil.cpp) with the reference's std::ranlux24_base stream."""

    def __init__(self, belts: int):
        self.h = lib().orc_hemisphere_create(belts)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_hemisphere_free(self.h)
            self.h = None

    @property
    def patch_count(self) -> int:
        return lib().orc_hemisphere_patch_count(self.h)

    def random(self, n: int):
        """n draws of getRandom() -> (directions [n, 3] float32, patch indices [n])."""
        d = np.empty((n, 3), np.float32)
        idx = np.empty(n, np.uint32)
        for k in range(n):
            idx[k] = lib().orc_hemisphere_random(self.h, d[k].ctypes.data)
        return d, idx
