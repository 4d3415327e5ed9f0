"""Python binding of libbzr.so (the MI355X-native Bezier-triangle ray tracer).

Thin ctypes layer over the C ABI in include/bzr.h.  The hot path
(BezierMesh::intersect, BezierTriangle::intersect, BezierLens::refract and the
refraction chain; reference/bezierMesh.cpp:206-227, bezierTriangle.cpp:123-195,
bezierLens.cpp:4-34, test.cpp:376-401) only exists as HIP kernels inside
libbzr.so: there is no Python or CPU fallback, and importing this package
raises if the library has not been built.

Arrays: rays are float32 SoA [6, n] (ox, oy, oz, dx, dy, dz); hits are
float32 [13, n] with rows t, px, py, pz, cos, b0, b1, b2, nx, ny, nz and the
uint32 bit patterns of `what` and `patch` in rows 11 and 12.  Host numpy
arrays or CUDA (HIP) torch tensors are accepted; tensors stay on the device
and the call returns before the kernels finish.  Stream: a context bound with
Context.set_stream / use_torch_stream launches there; an unbound context
launches tensor calls on torch's current stream (so the inputs torch produced
are ready and torch's caching allocator sees the outputs used in stream
order), then hands its own stream an event to wait on.
"""
from __future__ import annotations

import ctypes
import os
from contextlib import contextmanager
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent.parent
# BZR_LIBRARY: an alternative build of libbzr.so (A/B experiments); default: the in-tree build
LIB_PATH = Path(os.environ.get("BZR_LIBRARY", PKG_DIR / "lib" / "libbzr.so"))

OK = 0
HOST_PTRS, DEVICE_PTRS = 0, 1
MODE_PARITY, MODE_FAST = 0, 2
ACCEL_NONE = 4  # brute-force scan (A/B against the default BVH-culled path)
PIPELINE_STAGED = 8  # the culled path as separate kernels (traverse, bucket, Newton, resolve, finish)
PIPELINE_FUSED = 16  # the culled path as one k_trace kernel (default for dense batches; see include/bzr.h)
RAYS_AOS = 32  # rays / out_rays as [n, 6] records (the reference's Ray layout), transposed on the device
WHAT_FOLLOW0, WHAT_FOLLOW1, WHAT_FOLLOW2, WHAT_NONE, WHAT_INTERSECT = 0, 1, 2, 3, 4
LIMIT_THIS, LIMIT_NONE = 0, 1
RR_NONE, RR_INSIDE, RR_OUTSIDE = 0, 1, 2
ENVELOPE_ELLIPSOID, ENVELOPE_TESTLENS = 0, 1
PATCH_WORDS = 66  # sizeof(bzr_patch) / 4
KERNELS = ("k_traverse", "bucket", "k_newton", "k_follow", "k_finish", "k_overflow", "k_intersect_scan",
           "k_refract_scan", "k_chain_scan", "k_patch", "k_newton_lane", "k_trace")  # BZR_KERNEL_* ids
COUNTERS = ("segments", "pairs", "follows", "overflow_rays", "lane_chunks", "node_visits", "leaf_fetches",
            "gate_tests", "newton_rounds", "rounds_odd", "runs_odd", "dirty_rows")  # BZR_COUNTER_* ids
HIT_FIELDS = 13

_P = ctypes.c_void_p
_U32 = ctypes.c_uint32
_I32 = ctypes.c_int32
_F = ctypes.c_float

# name -> argtypes (all return bzr_status = int32 unless listed in _RET)
_SIGS = {
    "bzr_abi_version": [],
    "bzr_last_error": [],
    "bzr_device_count": [ctypes.POINTER(_I32)],
    "bzr_ctx_create": [_I32, ctypes.POINTER(_P)],
    "bzr_ctx_destroy": [_P],
    "bzr_ctx_set_stream": [_P, _P],
    "bzr_ctx_use_own_stream": [_P],
    "bzr_ctx_get_stream": [_P, ctypes.POINTER(_P)],
    "bzr_sync": [_P],
    "bzr_ctx_timing": [_P, _I32],
    "bzr_ctx_timing_report": [_P, _P, _P],
    "bzr_ctx_counters": [_P, _I32],
    "bzr_ctx_counters_report": [_P, _P],
    "bzr_mesh_create": [_P, _P, _U32, _U32, ctypes.POINTER(_P)],
    "bzr_mesh_destroy": [_P],
    "bzr_mesh_size": [_P, ctypes.POINTER(_U32)],
    "bzr_intersect": [_P, _P, _P, _U32, _P, _U32],
    "bzr_intersect_records": [_P, _P, _P, _U32, _P, _P, _U32],
    "bzr_patch_intersect": [_P, _P, _P, _P, _P, _U32, _P, _U32],
    "bzr_refract": [_P, _P, _F, _P, _P, _U32, _U32, _P, _P, _U32],
    "bzr_trace_chain": [_P, _P, _P, _U32, _P, _U32, _P, _P, _P, _U32],
    "bzr_trace_tiled": [_P, _U32, _P, _P, _U32, _P, _U32, _U32, _P, _P, _P, _U32],
    "bzr_tiled_create": [_P, _U32, _U32, _U32, _U32, _I32, ctypes.POINTER(_P)],
    "bzr_tiled_destroy": [_P],
    "bzr_tiled_info": [_P, _P, _P, _P],
    "bzr_tiled_set_rays": [_P, _P, _U32],
    "bzr_tiled_share_rays": [_P, _U32, ctypes.POINTER(_P)],
    "bzr_tiled_trace": [_P, _P, _P, _U32, _P, _P, _P, _U32],
    "bzr_tiled_stream": [_P, ctypes.POINTER(_P)],
    "bzr_tiled_sync": [_P],
    "bzr_tiled_set_layout": [_P, _I32, _U32],
    "bzr_tiled_calibrate": [_P, _P, _P, _U32, _U32, ctypes.POINTER(_U32)],
    "bzr_mesh_interpolate": [_P, _P, _I32, _P, _U32],
    "bzr_emit": [_P, _P, ctypes.c_uint64, _U32, _P, _P, _U32],
    "bzr_illuminate": [_P, _P, _P, _U32, _P, ctypes.c_uint64, _P, _P, _P, _U32],
    "bzr_mesh_bounding_sphere": [_P, _P],
    "bzr_trimesh_create": [ctypes.POINTER(_P)],
    "bzr_trimesh_destroy": [_P],
    "bzr_trimesh_copy": [_P, ctypes.POINTER(_P)],
    "bzr_trimesh_size": [_P, ctypes.POINTER(_U32)],
    "bzr_trimesh_get": [_P, _P],
    "bzr_trimesh_set": [_P, _P, _U32],
    "bzr_trimesh_make_solid_of_revolution": [_P, _I32, _I32, _I32, _F, _F, _F],
    "bzr_trimesh_make_ellipsoid": [_P, _I32, _I32, _F, _F, _F],
    "bzr_trimesh_read_stl": [_P, ctypes.c_char_p],
    "bzr_trimesh_write_stl": [_P, ctypes.c_char_p],
    "bzr_trimesh_transform": [_P, _P, _P],
    "bzr_trimesh_split": [_P, _I32],
    "bzr_trimesh_split_maxside": [_P, _F],
    "bzr_trimesh_standardize_vertices": [_P],
    "bzr_trimesh_standardize_normals": [_P],
    "bzr_trimesh_neighbours": [_P, _P, _P],
    "bzr_bezier_build": [_P, _P],
    "bzr_bezier_split_thick": [_P, _P],
    "bzr_bezier_interpolate": [_P, _I32, _P],
    "bzr_pack_frame": [_P, _I32, _P, _P, _P, _U32, _U32, _U32, _P],
    "bzr_debug_unit": [_P, _P, _U32, _P],
    "bzr_debug_div_heights": [_P, _P, _U32, _P],
    "bzr_debug_wave_clock": [_P, _P, _U32],
    "bzr_debug_wave_clock_rate": [_P, _P, _U32],
}
_RET = {"bzr_last_error": ctypes.c_char_p, "bzr_abi_version": _I32}

_lib = None


class BzrError(RuntimeError):
    pass


def lib():
    """Load libbzr.so (raises BzrError if it has not been built).

    PyTorch-ROCm ships its own libamdhip64 / libhsa-runtime64.  If libbzr were loaded first it
    would bind /opt/rocm's copies and torch would then load a second HIP runtime into the process
    (torch reports "No HIP GPUs are available").  Importing torch first (when installed) makes
    libbzr bind the runtime torch already loaded: one HIP runtime per process."""
    global _lib
    if _lib is None:
        if os.environ.get("BZR_NO_TORCH_PRELOAD") != "1":
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
        if not LIB_PATH.exists():
            raise BzrError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        handle = ctypes.CDLL(str(LIB_PATH))
        for name, args in _SIGS.items():
            if os.environ.get("BZR_LIBRARY") and name.startswith("bzr_debug_") and not hasattr(handle, name):
                continue  # an explicitly chosen other build (A/B against an earlier round): its debug hooks may differ
            fn = getattr(handle, name)
            fn.argtypes = args
            fn.restype = _RET.get(name, _I32)
        _lib = handle
    return _lib


def exported_symbols():
    return list(_SIGS)


def _check(status: int):
    if status != OK:
        msg = lib().bzr_last_error().decode(errors="replace")
        raise BzrError(f"libbzr status {status}: {msg}")


def device_count() -> int:
    c = _I32(0)
    _check(lib().bzr_device_count(ctypes.byref(c)))
    return c.value


# --------------------------------------------------------------- buffers
def _is_tensor(x) -> bool:
    return hasattr(x, "data_ptr") and hasattr(x, "is_cuda")


class _Buf:
    """Pointer + residency of a numpy array or a torch tensor."""

    def __init__(self, x, dtype, writable=False):
        if x is None:
            self.ptr, self.device, self.keep = None, None, None
            return
        if _is_tensor(x):
            if not x.is_contiguous():
                raise BzrError("tensor arguments must be contiguous")
            want = {np.float32: "torch.float32", np.uint32: "torch.uint32", np.int32: "torch.int32"}
            if str(x.dtype) not in (want[dtype], "torch.int32" if dtype == np.uint32 else want[dtype]):
                raise BzrError(f"tensor dtype {x.dtype} where {want[dtype]} is expected")
            self.ptr, self.device, self.keep = x.data_ptr(), bool(x.is_cuda), x
        else:
            a = np.asarray(x)
            if a.dtype != dtype or not a.flags["C_CONTIGUOUS"]:
                if writable:
                    raise BzrError(f"output array must be C-contiguous {np.dtype(dtype).name}")
                a = np.ascontiguousarray(a, dtype=dtype)
            self.ptr, self.device, self.keep = a.ctypes.data, False, a


def _residency(*bufs) -> int:
    flags = {b.device for b in bufs if b.device is not None}
    if len(flags) != 1:
        raise BzrError("mix of host and device buffers in one call")
    return DEVICE_PTRS if flags.pop() else HOST_PTRS


@contextmanager
def _stream_for(ctx: "Context", residency: int):
    """Device-buffer calls on an unbound context run on torch's current stream: the torch-made inputs are
    ready there and the outputs are used in that stream's order (torch's caching allocator relies on
    it).  The context's own stream is then ordered after them (event hand-off, no host wait)."""
    if residency == DEVICE_PTRS and not ctx.bound:
        import torch

        _check(lib().bzr_ctx_set_stream(ctx.handle, torch.cuda.current_stream(ctx.device).cuda_stream or None))
        try:
            yield
        finally:
            _check(lib().bzr_ctx_use_own_stream(ctx.handle))
    else:
        yield


# --------------------------------------------------------------- context
class Context:
    """A HIP device + stream (bzr_ctx)."""

    def __init__(self, device: int = 0):
        h = _P()
        _check(lib().bzr_ctx_create(device, ctypes.byref(h)))
        self.handle = h
        self.device = device
        self.bound = False  # launching on a caller stream (set_stream / use_torch_stream)

    def set_stream(self, stream_ptr: int | None):
        """Launch on this hipStream_t (0 / None = the HIP null stream); None-safe.  The stream must stay
        alive while bound (include/bzr.h bzr_ctx_set_stream)."""
        _check(lib().bzr_ctx_set_stream(self.handle, stream_ptr or None))
        self.bound = True

    def use_own_stream(self):
        _check(lib().bzr_ctx_use_own_stream(self.handle))
        self.bound = False

    def use_torch_stream(self, stream=None):
        """Launch on a torch stream (default: torch's current stream, which may be the null stream),
        so torch ops and torch.cuda.Event timing order with the kernels."""
        import torch

        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        self.set_stream(s.cuda_stream)

    def sync(self):
        _check(lib().bzr_sync(self.handle))

    def timing(self, enable: bool = True):
        """Bracket every launch with hipEvents on this context's stream (bzr_ctx_timing)."""
        _check(lib().bzr_ctx_timing(self.handle, int(bool(enable))))

    def timing_report(self) -> dict:
        """{kernel name: (total ms, launches)} since the last report (synchronises)."""
        ms = np.zeros(len(KERNELS), np.float32)
        calls = np.zeros(len(KERNELS), np.uint32)
        _check(lib().bzr_ctx_timing_report(self.handle, ms.ctypes.data, calls.ctypes.data))
        return {k: (float(ms[i]), int(calls[i])) for i, k in enumerate(KERNELS) if calls[i]}

    def counters(self, enable: bool = True):
        """Enable/disable the culled path's device work counters (see counters_report)."""
        _check(lib().bzr_ctx_counters(self.handle, 1 if enable else 0))

    def counters_report(self) -> dict:
        """{segments, pairs, follows, overflow_rays} accumulated since the last report (synchronises)."""
        out = np.zeros(len(COUNTERS), np.uint64)
        _check(lib().bzr_ctx_counters_report(self.handle, out.ctypes.data))
        return {k: int(out[i]) for i, k in enumerate(COUNTERS)}

    def close(self):
        if getattr(self, "handle", None):
            lib().bzr_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceMesh:
    """Immutable device copy of a patch array (bzr_mesh): float32 [n, 66] records."""

    def __init__(self, ctx: Context, patches: np.ndarray):
        p = np.ascontiguousarray(patches, dtype=np.float32).reshape(-1, PATCH_WORDS)
        h = _P()
        _check(lib().bzr_mesh_create(ctx.handle, p.ctypes.data if len(p) else None, len(p), PATCH_WORDS * 4,
                                     ctypes.byref(h)))
        self.handle, self.ctx, self.n = h, ctx, len(p)

    def close(self):
        if getattr(self, "handle", None):
            lib().bzr_mesh_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _n_of(rays, mode=0) -> int:
    """Rays in a batch: [6, n] rows, or [n, 6] records when mode has RAYS_AOS."""
    shape = tuple(rays.shape)
    if mode & RAYS_AOS:
        if len(shape) != 2 or shape[1] != 6:
            raise BzrError(f"RAYS_AOS rays must be [n, 6], got {shape}")
        return int(shape[0])
    if len(shape) != 2 or shape[0] != 6:
        raise BzrError(f"rays must be [6, n], got {shape}")
    return int(shape[1])


def _empty_like(rays, rows, dtype, mode=0):
    n = _n_of(rays, mode)
    shape = ((n, 6) if mode & RAYS_AOS else (6, n)) if rows == 6 else ((rows, n) if rows else (n,))
    if _is_tensor(rays):
        import torch

        tdt = {np.float32: torch.float32, np.uint32: torch.int32}[dtype]
        return torch.empty(shape, dtype=tdt, device=rays.device)
    return np.empty(shape, dtype=dtype)


def intersect(ctx: Context, mesh: DeviceMesh, rays, out=None, mode=MODE_PARITY):
    """BezierMesh::intersect over a batch -> hits [13, n].  mode |= ACCEL_NONE for the brute-force scan; mode |=
    RAYS_AOS for [n, 6] ray records."""
    n = _n_of(rays, mode)
    out = _empty_like(rays, HIT_FIELDS, np.float32, mode) if out is None else out
    r, o = _Buf(rays, np.float32), _Buf(out, np.float32, True)
    res = _residency(r, o)
    with _stream_for(ctx, res):
        _check(lib().bzr_intersect(ctx.handle, mesh.handle, r.ptr, n, o.ptr, res | mode))
    return out


HIT_RECORD_WORDS = 13  # bzr_hit_record: valid, point xyz, cos, distance, bary xyz, normal xyz, what


def intersect_records(ctx: Context, mesh: DeviceMesh, rays, records=None, patch=None, mode=MODE_PARITY):
    """bzr_intersect_records: the hits as the reference's BezierIntersection records -> (records uint32 [n, 13]
    (view float words with .view(float32)), patch [n]).  Same values as intersect()'s rows."""
    n = _n_of(rays, mode)
    if records is None and _is_tensor(rays):
        import torch

        records = torch.empty((n, HIT_RECORD_WORDS), dtype=torch.int32, device=rays.device)
    elif records is None:
        records = np.empty((n, HIT_RECORD_WORDS), np.uint32)
    patch = _empty_like(rays, 0, np.uint32, mode) if patch is None else patch
    r, o, p_ = _Buf(rays, np.float32), _Buf(records, np.uint32, True), _Buf(patch, np.uint32, True)
    res = _residency(r, o, p_)
    with _stream_for(ctx, res):
        _check(lib().bzr_intersect_records(ctx.handle, mesh.handle, r.ptr, n, o.ptr, p_.ptr, res | mode))
    return records, patch


def patch_intersect(ctx: Context, mesh: DeviceMesh, patch_index, limit, rays, out=None):
    """BezierTriangle::intersect for (patch, ray, limit) triples -> hits [13, n]."""
    n = _n_of(rays)
    out = _empty_like(rays, HIT_FIELDS, np.float32) if out is None else out
    i, l_ = _Buf(patch_index, np.uint32), _Buf(limit, np.uint32)
    r, o = _Buf(rays, np.float32), _Buf(out, np.float32, True)
    res = _residency(i, l_, r, o)
    with _stream_for(ctx, res):
        _check(lib().bzr_patch_intersect(ctx.handle, mesh.handle, i.ptr, l_.ptr, r.ptr, n, o.ptr, res))
    return out


def refract(ctx: Context, mesh: DeviceMesh, ri: float, rays, expected=None, expected_all=RR_INSIDE,
            out_rays=None, out_status=None, mode=MODE_PARITY):
    """BezierLens::refract over a batch -> (rays [6, n], status [n]); RAYS_AOS in mode: rays [n, 6] both ways."""
    n = _n_of(rays, mode)
    out_rays = _empty_like(rays, 6, np.float32, mode) if out_rays is None else out_rays
    out_status = _empty_like(rays, 0, np.uint32, mode) if out_status is None else out_status
    r, e = _Buf(rays, np.float32), _Buf(expected, np.uint32)
    o, s = _Buf(out_rays, np.float32, True), _Buf(out_status, np.uint32, True)
    res = _residency(r, o, s, *([e] if expected is not None else []))
    with _stream_for(ctx, res):
        _check(lib().bzr_refract(ctx.handle, mesh.handle, float(ri), r.ptr, e.ptr, int(expected_all), n, o.ptr, s.ptr,
                                 res | mode))
    return out_rays, out_status


def trace_chain(ctx: Context, lenses, ri, rays, out_rays=None, out_status=None, out_segments=None, mode=MODE_PARITY):
    """Refraction chain through `lenses` (list of DeviceMesh) -> (rays [6, n], status [n], segments [n]);
    RAYS_AOS in mode: rays [n, 6] both ways."""
    n = _n_of(rays, mode)
    nl = len(lenses)
    handles = (_P * nl)(*[m.handle for m in lenses])
    ris = (_F * nl)(*[float(x) for x in ri])
    out_rays = _empty_like(rays, 6, np.float32, mode) if out_rays is None else out_rays
    out_status = _empty_like(rays, 0, np.uint32, mode) if out_status is None else out_status
    out_segments = _empty_like(rays, 0, np.uint32, mode) if out_segments is None else out_segments
    r = _Buf(rays, np.float32)
    o, s, g = _Buf(out_rays, np.float32, True), _Buf(out_status, np.uint32, True), _Buf(out_segments, np.uint32, True)
    res = _residency(r, o, s, g)
    with _stream_for(ctx, res):
        _check(lib().bzr_trace_chain(ctx.handle, ctypes.cast(handles, _P), ctypes.cast(ris, _P), nl, r.ptr, n, o.ptr,
                                     s.ptr, g.ptr, res | mode))
    return out_rays, out_status, out_segments


PACK_IMAGE, PACK_RAYS, PACK_COMPACT = 0, 1, 2  # BZR_PACK_*
PACK_LAYOUTS = {"image": PACK_IMAGE, "rays": PACK_RAYS, "compact": PACK_COMPACT}


def pack_frame(ctx: Context, layout: str, rays, status, segments, packed, npad: int, cap: int = 0):
    """bzr_pack_frame: one chain frame's device outputs (rays [6, n], status [n], segments [n]) into the
    gather buffer `packed` (a CUDA tensor laid out as bzr_amd.frame's `layout`: image, rays or compact)
    on the device, no host sync.  Same bits as frame.pack / frame.pack_compact in the columns they read."""
    if layout not in PACK_LAYOUTS:
        raise ValueError(f"layout {layout!r}")
    n = int(status.shape[0])
    if int(segments.shape[0]) != n:
        raise BzrError(f"pack_frame: segments [{int(segments.shape[0])}] for status [{n}]")
    if rays is not None and tuple(rays.shape) != (6, n):
        raise BzrError(f"pack_frame: rays must be [6, {n}], got {tuple(rays.shape)}")
    # the device writes this many floats into `packed` (include/bzr.h bzr_pack_frame)
    need = {"image": npad, "rays": 7 * npad, "compact": npad // 4 + 1 + 6 * (cap + 1)}[layout]
    if int(packed.numel()) < need:
        raise BzrError(f"pack_frame: {layout} layout needs {need} floats (npad {npad}, cap {cap}), packed has "
                       f"{int(packed.numel())}")
    bufs = [_Buf(status, np.uint32), _Buf(segments, np.uint32), _Buf(packed, np.float32, True)]
    r = _Buf(rays, np.float32) if rays is not None else _Buf(None, np.float32)
    if r.ptr is not None:
        bufs.append(r)
    if _residency(*bufs) != DEVICE_PTRS:
        raise BzrError("pack_frame takes device tensors")
    with _stream_for(ctx, DEVICE_PTRS):
        _check(lib().bzr_pack_frame(ctx.handle, PACK_LAYOUTS[layout], r.ptr, bufs[0].ptr, bufs[1].ptr, n, int(npad),
                                    int(cap), bufs[2].ptr))
    return packed


def trace_tiled(ctxs, lenses, ri, rays, tile_rays=4096, mode=MODE_PARITY, out=None):
    """bzr_trace_tiled: the chain over several contexts (one per device) from one process, gathered to
    ctxs[0]'s device on the device side.  `lenses[d]` is the list of DeviceMesh living on ctxs[d]; rays
    [6, n] ordered tile-major, a host array or a tensor on ctxs[0]'s device (then the outputs are tensors
    there).  -> (rays [6, n], status [n], segments [n]) in input order (RAYS_AOS in mode: rays [n, 6] both ways)."""
    nc, nl = len(ctxs), len(ri)
    if len(lenses) != nc or any(len(ls) != nl for ls in lenses):
        raise ValueError("lenses must hold one list of len(ri) meshes per context")
    r = _Buf(rays, np.float32)
    n = _n_of(rays, mode)
    if out is None:
        out = (_empty_like(rays, 6, np.float32, mode), _empty_like(rays, 0, np.uint32, mode),
               _empty_like(rays, 0, np.uint32, mode))
    o, s_, g = _Buf(out[0], np.float32, True), _Buf(out[1], np.uint32, True), _Buf(out[2], np.uint32, True)
    res = _residency(r, o, s_, g)
    cs = (_P * nc)(*[c.handle for c in ctxs])
    hs = (_P * (nc * nl))(*[m.handle for ls in lenses for m in ls])
    ris = (_F * nl)(*[float(x) for x in ri])
    if res == DEVICE_PTRS:
        import torch

        torch.cuda.current_stream(ctxs[0].device).synchronize()  # torch-made inputs are complete
    _check(lib().bzr_trace_tiled(ctypes.cast(cs, _P), nc, ctypes.cast(hs, _P), ctypes.cast(ris, _P), nl,
                                 r.ptr, n, tile_rays, o.ptr, s_.ptr, g.ptr, mode | res))
    return out


GATHER_AUTO, GATHER_RCCL, GATHER_PEER, GATHER_DIRECT = 0, 1, 2, 3  # BZR_GATHER_*


class TiledPlan:
    """bzr_tiled: multi-device frames from one process, gathered to device 0 on the device side (RCCL over
    xGMI between distinct devices, peer copies otherwise; one device: traced straight into the outputs).  ctxs: nslot lists of ndev contexts (slot s, device
    d); the frame is n tile-major rays."""

    def __init__(self, ctxs, n: int, tile_rays: int = 4096, transport: int = GATHER_AUTO):
        slots = [list(s) for s in ctxs]
        self.ndev, self.nslot = len(slots[0]), len(slots)
        if any(len(s) != self.ndev for s in slots):
            raise ValueError("every slot lists the same number of devices")
        self.ctxs = slots
        flat = (_P * (self.ndev * self.nslot))(*[c.handle for s in slots for c in s])
        h = _P()
        _check(lib().bzr_tiled_create(ctypes.cast(flat, _P), self.ndev, self.nslot, n, tile_rays, transport,
                                      ctypes.byref(h)))
        self.handle, self.n, self.tile_rays = h, n, tile_rays

    def info(self):
        """(transport, rays per device share, npad)"""
        t, npad = _I32(0), _U32(0)
        share = np.zeros(self.ndev, np.uint32)
        _check(lib().bzr_tiled_info(self.handle, ctypes.byref(t), share.ctypes.data, ctypes.byref(npad)))
        return int(t.value), share, int(npad.value)

    def set_rays(self, rays, mode=0):
        """The frame's rays [6, n] (or [n, 6] records with mode RAYS_AOS), host array or tensor on device 0."""
        if _n_of(rays, mode) != self.n:
            raise BzrError(f"set_rays: {_n_of(rays, mode)} rays for a plan of {self.n}")
        r = _Buf(rays, np.float32)
        if r.device:
            import torch

            torch.cuda.current_stream(self.ctxs[0][0].device).synchronize()
        _check(lib().bzr_tiled_set_rays(self.handle, r.ptr, (DEVICE_PTRS if r.device else HOST_PTRS) | (mode & RAYS_AOS)))
        # a device source is only queued for copying (bzr_tiled_set_rays): keep it -- and any contiguous / float32
        # copy _Buf made of it -- alive until the copy has run, i.e. until the next sync() or set_rays(), so torch's
        # caching allocator cannot hand its memory to a kernel that overwrites it first
        self._pending_src = (rays, r) if r.device else None

    def trace(self, lenses, ri, out_rays, out_status, out_segments=None, mode=MODE_PARITY):
        """One frame; lenses[d] = device d's DeviceMesh list.  Device tensors (on device 0): queued, ready on
        stream() / after sync(); host arrays: synchronous."""
        nl = len(ri)
        hs = (_P * (self.ndev * nl))(*[m.handle for ls in lenses for m in ls])
        ris = (_F * nl)(*[float(x) for x in ri])
        o, s_ = _Buf(out_rays, np.float32, True), _Buf(out_status, np.uint32, True)
        g = _Buf(out_segments, np.uint32, True)
        res = _residency(o, s_, *([g] if out_segments is not None else []))
        _check(lib().bzr_tiled_trace(self.handle, ctypes.cast(hs, _P), ctypes.cast(ris, _P), nl, o.ptr, s_.ptr, g.ptr,
                                     res | mode))

    def stream(self) -> int:
        p = _P()
        _check(lib().bzr_tiled_stream(self.handle, ctypes.byref(p)))
        return int(p.value or 0)

    def sync(self):
        _check(lib().bzr_tiled_sync(self.handle))
        self._pending_src = None  # the queued ray copy has run

    def set_layout(self, layout: str, cap: int = 0):
        """"rays" (28 B per ray) or "compact" (survivors only, up to `cap` per device share)."""
        _check(lib().bzr_tiled_set_layout(self.handle, PACK_LAYOUTS[layout], cap))

    def calibrate(self, lenses, ri, mode=MODE_PARITY) -> int:
        """One synchronous frame, then the compact layout sized from its survivors; returns the capacity."""
        nl = len(ri)
        hs = (_P * (self.ndev * nl))(*[m.handle for ls in lenses for m in ls])
        ris = (_F * nl)(*[float(x) for x in ri])
        cap = _U32(0)
        _check(lib().bzr_tiled_calibrate(self.handle, ctypes.cast(hs, _P), ctypes.cast(ris, _P), nl, mode,
                                          ctypes.byref(cap)))
        return int(cap.value)

    def close(self):
        if getattr(self, "handle", None):
            lib().bzr_tiled_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def interpolate(ctx: Context, mesh: DeviceMesh, divisor: int, out=None):
    """BezierMesh::interpolate(divisor) on the device -> triangles [divisor^2 * n_patches, 3, 3] float32
    (reference order: sub-triangle outer, patch inner).  `out` may be a CUDA tensor (stays on the device)."""
    count = int(divisor) * int(divisor) * mesh.n
    if out is None:
        out = np.empty((count, 3, 3), np.float32)
    o = _Buf(out, np.float32, True)
    res = _residency(o)
    with _stream_for(ctx, res):
        _check(lib().bzr_mesh_interpolate(ctx.handle, mesh.handle, int(divisor), o.ptr, res))
    return out


# ------------------------------------------------------------ illumination
class Emitter(ctypes.Structure):
    """bzr_emitter: rectangle origin + a*edge_u + b*edge_v, parts_u x parts_v parts, points_per_part
    points per part, rays_per_point rays per point, hemisphere around +x numbered by `belts`."""
    _fields_ = [("origin", _F * 3), ("edge_u", _F * 3), ("edge_v", _F * 3), ("parts_u", _U32), ("parts_v", _U32),
                ("points_per_part", _U32), ("rays_per_point", _U32), ("belts", _U32), ("seed", ctypes.c_uint64)]


class Target(ctypes.Structure):
    """bzr_target: origin + a*axis_u + b*axis_v, a < size_u, b < size_v, bins_u x bins_v cells."""
    _fields_ = [("origin", _F * 3), ("axis_u", _F * 3), ("axis_v", _F * 3), ("size_u", _F), ("size_v", _F),
                ("bins_u", _U32), ("bins_v", _U32)]


ILLUM_STATS = ("emitted", "culled", "exited", "landed")  # BZR_ILLUM_* ids


def emit(ctx: Context, em: Emitter, first: int, n: int, rays=None, patch=None):
    """Rays first .. first+n-1 of the emitter -> (rays [6, n], hemisphere patch index [n])."""
    rays = np.empty((6, n), np.float32) if rays is None else rays
    patch = np.empty(n, np.uint32) if patch is None else patch
    r, p = _Buf(rays, np.float32, True), _Buf(patch, np.uint32, True)
    res = _residency(r, p)
    with _stream_for(ctx, res):
        _check(lib().bzr_emit(ctx.handle, ctypes.byref(em), int(first), int(n), r.ptr, p.ptr, res))
    return rays, patch


def illuminate(ctx: Context, lenses, ri, em: Emitter, total_rays: int, target: Target, hist=None):
    """Emitter -> bounding-sphere cull -> refraction chain -> target counts.  Returns (hist [bins_v, bins_u]
    uint32, accumulated into `hist` if given, stats dict)."""
    nl = len(lenses)
    handles = (_P * nl)(*[m.handle for m in lenses])
    ris = (_F * nl)(*[float(x) for x in ri])
    hist = np.zeros((target.bins_v, target.bins_u), np.uint32) if hist is None else hist
    h = _Buf(hist, np.uint32, True)
    stats = (ctypes.c_uint64 * 4)()
    res = _residency(h)
    with _stream_for(ctx, res):
        _check(lib().bzr_illuminate(ctx.handle, handles, ris, nl, ctypes.byref(em), int(total_rays),
                                    ctypes.byref(target), h.ptr, stats, res))
    return hist, dict(zip(ILLUM_STATS, [int(x) for x in stats]))


def bounding_sphere(mesh: DeviceMesh) -> np.ndarray:
    """The lens's Ritter sphere over its gate-region boxes: [cx, cy, cz, r]."""
    out = (_F * 4)()
    _check(lib().bzr_mesh_bounding_sphere(mesh.handle, out))
    return np.array(list(out), np.float32)


# ------------------------------------------------------------ host preprocessing
class TriMesh:
    """The reference's Mesh (host C++ in libbzr): generators, welding, orientation, Bezier build."""

    def __init__(self, _handle=None):
        if _handle is None:
            h = _P()
            _check(lib().bzr_trimesh_create(ctypes.byref(h)))
            _handle = h
        self.handle = _handle

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                lib().bzr_trimesh_destroy(self.handle)
                self.handle = None
        except Exception:
            pass

    def copy(self) -> "TriMesh":
        h = _P()
        _check(lib().bzr_trimesh_copy(self.handle, ctypes.byref(h)))
        return TriMesh(h)

    def __len__(self):
        n = _U32(0)
        _check(lib().bzr_trimesh_size(self.handle, ctypes.byref(n)))
        return n.value

    @property
    def triangles(self) -> np.ndarray:
        t = np.empty((len(self), 3, 3), dtype=np.float32)
        _check(lib().bzr_trimesh_get(self.handle, t.ctypes.data))
        return t

    @triangles.setter
    def triangles(self, tris):
        t = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 3, 3)
        _check(lib().bzr_trimesh_set(self.handle, t.ctypes.data, len(t)))

    def make_ellipsoid(self, sectors, belts, size=(1.0, 1.0, 1.0)):
        _check(lib().bzr_trimesh_make_ellipsoid(self.handle, sectors, belts, *map(float, size)))
        return self

    def make_unit_sphere(self, sectors, belts):
        return self.make_ellipsoid(sectors, belts, (1.0, 1.0, 1.0))

    def make_solid_of_revolution(self, sectors, belts, envelope, size):
        _check(lib().bzr_trimesh_make_solid_of_revolution(self.handle, sectors, belts, envelope, *map(float, size)))
        return self

    def read_stl(self, path):
        _check(lib().bzr_trimesh_read_stl(self.handle, str(path).encode()))
        return self

    def write_stl(self, path):
        _check(lib().bzr_trimesh_write_stl(self.handle, str(path).encode()))
        return self

    def transform(self, matrix=None, displacement=(0.0, 0.0, 0.0)):
        m = np.eye(3, dtype=np.float32) if matrix is None else np.asarray(matrix, dtype=np.float32)
        colmajor = np.ascontiguousarray(m.T.reshape(-1))
        d = np.ascontiguousarray(displacement, dtype=np.float32)
        _check(lib().bzr_trimesh_transform(self.handle, colmajor.ctypes.data, d.ctypes.data))
        return self

    def translate(self, d):
        return self.transform(None, d)

    def split(self, divisor: int):
        _check(lib().bzr_trimesh_split(self.handle, divisor))
        return self

    def split_maxside(self, max_side: float):
        _check(lib().bzr_trimesh_split_maxside(self.handle, float(max_side)))
        return self

    def standardize_vertices(self):
        _check(lib().bzr_trimesh_standardize_vertices(self.handle))
        return self

    def standardize_normals(self):
        _check(lib().bzr_trimesh_standardize_normals(self.handle))
        return self

    def standardize(self):
        return self.standardize_vertices().standardize_normals()

    def neighbours(self):
        n = len(self)
        fellow = np.empty((n, 3), dtype=np.uint32)
        start = np.empty((n, 3), dtype=np.uint8)
        _check(lib().bzr_trimesh_neighbours(self.handle, fellow.ctypes.data, start.ctypes.data))
        return fellow, start

    def bezier_patches(self) -> np.ndarray:
        """BezierMesh(Mesh) -> float32 [3n, 66] patch records (bzr_patch layout)."""
        out = np.empty((3 * len(self), PATCH_WORDS), dtype=np.float32)
        _check(lib().bzr_bezier_build(self.handle, out.ctypes.data))
        return out

    def bezier_split_thick(self) -> "TriMesh":
        out = TriMesh()
        _check(lib().bzr_bezier_split_thick(self.handle, out.handle))
        return out

    def bezier_interpolate(self, divisor: int) -> "TriMesh":
        out = TriMesh()
        _check(lib().bzr_bezier_interpolate(self.handle, divisor, out.handle))
        return out


__all__ = [
    "BzrError", "Context", "DeviceMesh", "TriMesh", "intersect", "patch_intersect", "refract", "trace_chain", "interpolate",
    "Emitter", "Target", "emit", "illuminate", "bounding_sphere",
    "device_count", "lib", "exported_symbols", "LIB_PATH",
]
