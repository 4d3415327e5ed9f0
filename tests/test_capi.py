"""The C-ABI library: it loads without a GPU, exports every symbol include/*.h declares, reports
errors as status codes + text, and refuses to run the hot path without a HIP device (no CPU fallback)."""
import ctypes
import re
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]


def declared(header):
    text = (REPO / "include" / header).read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(bzr_[a-z0-9_]+)\s*\(", text)))


@pytest.mark.parametrize("header", ["bzr.h", "bzr_debug.h"])
def test_every_declared_symbol_is_exported(bzr, header):
    lib = ctypes.CDLL(str(bzr.LIB_PATH))
    names = declared(header)
    assert len(names) > (30 if header == "bzr.h" else 0)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_the_header(bzr):
    assert set(declared("bzr.h")) <= set(bzr.exported_symbols())


def test_abi_version_and_patch_layout(bzr):
    assert bzr.lib().bzr_abi_version() == 2
    # bzr_patch is the reference's 264-byte BezierTriangle (reference/bezierTriangle.h:64-80)
    assert bzr.PATCH_WORDS * 4 == 264


def test_hot_path_needs_a_device(bzr):
    if bzr.device_count() > 0:
        pytest.skip("a GPU is visible here")
    with pytest.raises(bzr.BzrError, match="no HIP device"):
        bzr.Context(0)


def test_errors_are_status_codes(bzr):
    L = bzr.lib()
    assert L.bzr_trimesh_split(None, 2) == 1
    assert b"null" in L.bzr_last_error()
    m = bzr.TriMesh()
    with pytest.raises(bzr.BzrError, match="divisor"):
        m.split(0)
    with pytest.raises(bzr.BzrError, match="cannot open"):
        m.read_stl("/nonexistent/file.stl")
    with pytest.raises(bzr.BzrError, match="not standardized"):
        bzr.TriMesh().make_ellipsoid(4, 2).bezier_patches()


def test_flags_are_validated_first(bzr):
    """Unknown flag bits and both pipeline bits together are rejected before anything else (no device
    needed): a caller's mistake fails loudly instead of silently picking one pipeline."""
    L = bzr.lib()
    bad = {bzr.PIPELINE_STAGED | bzr.PIPELINE_FUSED: b"exclusive", 1 << 7: b"unknown flag", 1 << 31: b"unknown flag",
           bzr.MODE_FAST | bzr.ACCEL_NONE: b"culled path"}
    f = (ctypes.c_float * 1)(1.3)
    for flags, msg in bad.items():
        assert L.bzr_intersect(None, None, None, 0, None, flags) == 1
        assert msg in L.bzr_last_error(), (flags, L.bzr_last_error())
        assert L.bzr_refract(None, None, ctypes.c_float(1.3), None, None, 0, 0, None, None, flags) == 1
        assert msg in L.bzr_last_error()
        assert L.bzr_trace_chain(None, None, f, 1, None, 0, None, None, None, flags) == 1
        assert msg in L.bzr_last_error()
    # every documented combination passes the flag check (and then fails on the null context)
    for flags in (0, bzr.DEVICE_PTRS, bzr.MODE_FAST, bzr.ACCEL_NONE, bzr.PIPELINE_STAGED, bzr.PIPELINE_FUSED,
                  bzr.DEVICE_PTRS | bzr.MODE_FAST | bzr.PIPELINE_FUSED, bzr.RAYS_AOS, bzr.RAYS_AOS | bzr.DEVICE_PTRS):
        assert L.bzr_intersect(None, None, None, 0, None, flags) == 1
        assert b"null context" in L.bzr_last_error()
    # the ray-record layout: taken by the ray-batch calls, refused by the others
    assert L.bzr_trace_chain(None, None, f, 1, None, 0, None, None, None, bzr.RAYS_AOS) == 1
    assert b"null context" in L.bzr_last_error()
    assert L.bzr_refract(None, None, ctypes.c_float(1.3), None, None, 0, 0, None, None, bzr.RAYS_AOS) == 1
    assert b"null context" in L.bzr_last_error()
    assert L.bzr_patch_intersect(None, None, None, None, None, 0, None, bzr.RAYS_AOS) == 1
    assert b"BZR_RAYS_AOS" in L.bzr_last_error()
    # and the Python helpers check the [n, 6] shape before any call
    with pytest.raises(bzr.BzrError, match=r"\[n, 6\]"):
        bzr.intersect(None, None, np.zeros((6, 10), np.float32), mode=bzr.RAYS_AOS)


def test_trace_tiled_validates_before_touching_a_device(bzr):
    import ctypes
    L = bzr.lib()
    f = (ctypes.c_float * 1)(1.3)
    assert L.bzr_trace_tiled(None, 0, None, f, 1, None, 0, 4096, None, None, None, 0) == 1
    assert b"no contexts" in L.bzr_last_error()
    fake = (ctypes.c_void_p * 2)(1, 1)  # the same context twice: rejected (one host thread per context)
    assert L.bzr_trace_tiled(fake, 2, fake, f, 1, None, 0, 4096, None, None, None, 0) == 1
    assert b"repeated context" in L.bzr_last_error()
    one = (ctypes.c_void_p * 1)(1)
    assert L.bzr_trace_tiled(one, 1, one, f, 1, None, 0, 0, None, None, None, 0) == 1
    assert b"tile_rays" in L.bzr_last_error()
    assert L.bzr_trace_tiled(one, 1, one, f, 1, None, 64, 64, None, None, None, bzr.DEVICE_PTRS) == 1
    assert b"null buffer" in L.bzr_last_error()


def test_tiled_plan_validates_before_touching_a_device(bzr):
    """bzr_tiled_create / _trace / _info reject bad arguments without a device (include/bzr.h)."""
    import ctypes
    L = bzr.lib()
    out = ctypes.c_void_p()
    one = (ctypes.c_void_p * 1)(1)
    assert L.bzr_tiled_create(None, 0, 1, 64, 64, 0, ctypes.byref(out)) == 1 and b"no contexts" in L.bzr_last_error()
    assert L.bzr_tiled_create(one, 1, 1, 64, 0, 0, ctypes.byref(out)) == 1 and b"tile_rays" in L.bzr_last_error()
    assert L.bzr_tiled_create(one, 1, 1, 0, 64, 0, ctypes.byref(out)) == 1 and b"empty frame" in L.bzr_last_error()
    assert L.bzr_tiled_create(one, 1, 1, 64, 64, 7, ctypes.byref(out)) == 1 and b"transport" in L.bzr_last_error()
    two = (ctypes.c_void_p * 2)(1, 1)
    assert L.bzr_tiled_create(two, 1, 2, 64, 64, 0, ctypes.byref(out)) == 1 and b"repeated" in L.bzr_last_error()
    assert out.value is None
    assert L.bzr_tiled_trace(None, None, None, 0, None, None, None, 0) == 1
    assert L.bzr_tiled_info(None, None, None, None) == 1
    assert L.bzr_tiled_destroy(None) == 0


def test_patch_records_view_as_reference_struct(bzr):
    """The 66-word records reinterpret as the bzr_patch / BezierTriangle layout: neighbours are u32 indices
    into the patch array, the direction vector A is (1, 0, -1) (reference/bezierTriangle.cpp:83)."""
    p = bzr.TriMesh().make_unit_sphere(3, 7).standardize().bezier_patches()
    neigh = p[:, 16:19].view(np.uint32)
    assert neigh.max() < len(p)
    assert np.array_equal(p[:, 60:63], np.tile([1.0, 0.0, -1.0], (len(p), 1)).astype(np.float32))
    assert (p[:, 58] <= 0).all() and (p[:, 59] >= 0).all()  # mHeightInside <= 0 <= mHeightOutside


def test_pack_frame_validates_before_touching_a_device(bzr):
    """bzr_pack_frame (the gather-buffer packer, include/bzr.h) rejects bad layouts and sizes before it
    looks at the context."""
    L = bzr.lib()
    p = ctypes.c_void_p(16)  # never dereferenced: every call below fails validation first
    cases = [((7, p, p, p, 10, 16, 0, p), b"unknown pack layout"),
             ((bzr.PACK_IMAGE, None, p, p, 17, 16, 0, p), b"n > npad"),
             ((bzr.PACK_COMPACT, p, p, p, 10, 18, 4, p), b"multiple of 4"),
             ((bzr.PACK_COMPACT, p, p, p, 10, 16, 0, p), b"0 < cap"),
             ((bzr.PACK_COMPACT, p, p, p, 10, 16, 17, p), b"0 < cap"),
             ((bzr.PACK_RAYS, None, p, p, 10, 16, 0, p), b"null rays"),
             ((bzr.PACK_IMAGE, None, None, p, 10, 16, 0, p), b"null status"),
             ((bzr.PACK_IMAGE, None, p, p, 10, 16, 0, None), b"null status"),
             ((bzr.PACK_COMPACT, None, None, None, 0, 16, 4, p), b"null context"),  # n = 0: empty inputs
             ((bzr.PACK_IMAGE, None, p, p, 10, 16, 0, p), b"null context")]
    for args, msg in cases:
        assert L.bzr_pack_frame(None, *args) == 1, args
        assert msg in L.bzr_last_error(), (args, L.bzr_last_error())


def test_pack_frame_python_checks_buffer_sizes(bzr):
    """bzr_amd.pack_frame checks the gather buffer against the layout's size and the rays' shape before the
    device would write past it."""
    torch = pytest.importorskip("torch")
    n, npad, cap = 100, 4096, 64
    st, sg = torch.zeros(n, dtype=torch.int32), torch.zeros(n, dtype=torch.int32)
    rays = torch.zeros((6, n))
    cases = [("rays", rays, torch.zeros(7 * npad - 1), "needs"),
             ("image", None, torch.zeros(npad - 1), "needs"),
             ("compact", rays, torch.zeros(npad // 4 + 1 + 6 * cap), "needs"),
             ("rays", torch.zeros((7, n)), torch.zeros(7 * npad), r"\[6, 100\]"),
             ("image", None, torch.zeros(npad), None)]
    for layout, r, packed, msg in cases:
        if msg is None:  # sizes fine: the call gets as far as the residency check (host tensors)
            with pytest.raises(bzr.BzrError, match="device tensors"):
                bzr.pack_frame(None, layout, r, st, sg, packed, npad, cap)
        else:
            with pytest.raises(bzr.BzrError, match=msg):
                bzr.pack_frame(None, layout, r, st, sg, packed, npad, cap)
