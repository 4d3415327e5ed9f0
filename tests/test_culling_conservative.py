"""The BVH culling is exact-preserving: every (ray, patch) pair that passes the reference's planar gate
(reference/bezierTriangle.cpp:124-131, computed by the oracle) must also pass the float32 slab test
the traversal kernel runs against that patch's gate-region box (csrc/host/bvh.cpp,
csrc/device/trace.hip `slab`).  A pair that passes the gate but misses its box would silently change
the result; this checks it on CPU for grazing, far, random and config rays -- including the
ill-conditioned patches whose plane passes near the origin.  Both BVH tiers are checked:
the far tier (origins up to 100x the mesh span) and the near tier (tighter boxes, origins up to 8x)."""
import ctypes

import numpy as np
import pytest

from bzr_amd.configs import CONFIGS, build_lens, grid_rays


TIERS = [0, 1]  # bvh.hpp kTierFar, kTierNear


def gate_boxes(bzr, patches, tier=0):
    L = bzr.lib()
    fn = L.bzr_debug_gate_boxes_tier
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]
    fn.restype = ctypes.c_int32
    p = np.ascontiguousarray(patches, np.float32)
    boxes = np.zeros((len(p), 6), np.float32)
    smax = np.zeros(1, np.float32)
    assert fn(p.ctypes.data, len(p), 264, tier, boxes.ctypes.data, smax.ctypes.data) == 0
    return boxes, float(smax[0])


def slab_f32(boxes, rays):
    """float32 replica of the kernel's slab(): hit[r, i]."""
    f = np.float32
    s = rays[:3].T.astype(f)[:, None, :]  # [R,1,3]
    d = rays[3:].T.astype(f)
    d = np.where(np.abs(d) < f(1e-20), np.copysign(f(1e-20), d), d).astype(f)
    inv = (f(1.0) / d)[:, None, :]
    lo, hi = boxes[None, :, :3], boxes[None, :, 3:]
    with np.errstate(invalid="ignore", over="ignore"):
        a = ((lo - s) * inv).astype(f)
        b = ((hi - s) * inv).astype(f)
    tnear = np.fmax(np.fmax(np.fmin(a[..., 0], b[..., 0]), np.fmin(a[..., 1], b[..., 1])), np.fmin(a[..., 2], b[..., 2]))
    tfar = np.fmin(np.fmin(np.fmax(a[..., 0], b[..., 0]), np.fmax(a[..., 1], b[..., 1])), np.fmax(a[..., 2], b[..., 2]))
    return (tnear <= tfar) & (tfar >= 0)


def random_rays(rng, n, centre, spread, far=False):
    c = np.asarray(centre, np.float64)
    o = c + rng.uniform(-spread, spread, (n, 3)) * (8.0 if far else 1.5)
    tgt = c + rng.uniform(-spread, spread, (n, 3))
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    # a quarter of the rays get a zeroed direction component (axis-parallel cases)
    z = rng.random(n) < 0.25
    d[z, rng.integers(0, 3, z.sum())] = 0.0
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return np.concatenate([o.T, d.T]).astype(np.float32)


def check(bzr, orc, patches, rays, tier=0):
    boxes, smax = gate_boxes(bzr, patches, tier)
    gate = orc.planar_gate(patches, rays)
    near = np.abs(rays[:3]).max(axis=0) <= smax
    assert near.mean() > 0.5, "most test rays must start within this tier's radius"
    hit = slab_f32(boxes, rays)
    missed = gate & ~hit & near[:, None]
    assert gate.sum() > 0
    assert not missed.any(), f"{int(missed.sum())} gate-passing pairs culled, e.g. {np.argwhere(missed)[:5]}"
    return gate.sum(), hit.sum()


@pytest.mark.parametrize("tier", TIERS)
@pytest.mark.parametrize("name", ["cfg1", "cfg2", "cfg3"])
def test_config_rays_never_culled(bzr, orc, name, tier):
    cfg = CONFIGS[name]
    patches = build_lens(bzr.TriMesh, cfg.lenses[0]).bezier_patches()
    rays = grid_rays(cfg, side=48)
    check(bzr, orc, patches, rays, tier)


@pytest.mark.parametrize("tier", TIERS)
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_and_grazing_rays_never_culled(bzr, orc, seed, tier):
    rng = np.random.default_rng(seed)
    patches = build_lens(bzr.TriMesh, CONFIGS["cfg2"].lenses[0]).bezier_patches()
    rays = np.concatenate([random_rays(rng, 1500, (10, 0, 0), 3.0), random_rays(rng, 500, (10, 0, 0), 3.0, far=True)], 1)
    # refracted-ray-like origins: points on the lens surface heading inward
    cp = patches[:, 19:22]
    pick = rng.integers(0, len(patches), 500)
    o = cp[pick] + rng.normal(0, 1e-3, (500, 3)).astype(np.float32)
    d = np.array([10, 0, 0], np.float32) - o + rng.normal(0, 0.5, (500, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([rays, np.concatenate([o.T, d.T]).astype(np.float32)], 1)
    gate, hit = check(bzr, orc, patches, rays, tier)
    assert hit < 0.2 * rays.shape[1] * len(patches)  # and the boxes do cull


@pytest.mark.parametrize("tier", TIERS)
def test_ill_conditioned_patches(bzr, orc, tier):
    """Lens placed so that many patch planes pass close to the origin: the gate region is far larger than
    the flat triangle there, and the boxes must cover it."""
    m = bzr.TriMesh().make_ellipsoid(16, 8, (1.0, 4.0, 2.0)).translate((1.3, 0.5, 0.0)).standardize()
    patches = m.bezier_patches()
    c = np.abs(patches[:, 3])
    assert (c < 3e-3).sum() >= 2  # planes through (nearly) the origin
    rng = np.random.default_rng(7)
    rays = random_rays(rng, 3000, (1.3, 0.5, 0.0), 3.0)
    # plus rays aimed at the ill-conditioned patches themselves
    worst = np.argsort(c)[:8]
    cp = patches[worst][:, 19:28].reshape(-1, 3, 3)
    tgt = cp.mean(axis=1).repeat(125, 0) + rng.normal(0, 0.05, (1000, 3))
    o = tgt + rng.normal(0, 2.0, (1000, 3))
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([rays, np.concatenate([o.T, d.T]).astype(np.float32)], 1)
    check(bzr, orc, patches, rays, tier)


@pytest.mark.parametrize("cfg_name", ["cfg1", "cfg2", "cfg3"])
def test_bounding_sphere_encloses_gate_boxes(bzr, cfg_name):
    """bzr_illuminate's pre-cull is exact only if the sphere holds every gate-region box: check all
    eight corners of every non-empty box (in double, against the float centre and radius)."""
    patches = build_lens(bzr.TriMesh, CONFIGS[cfg_name].lenses[0]).bezier_patches()
    boxes, _ = gate_boxes(bzr, patches)
    L = bzr.lib()
    fn = L.bzr_debug_bounding_sphere
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    fn.restype = ctypes.c_int32
    sph = np.zeros(4, np.float32)
    p = np.ascontiguousarray(patches, np.float32)
    assert fn(p.ctypes.data, len(p), 264, sph.ctypes.data) == 0
    lo, hi = boxes[:, :3].astype(np.float64), boxes[:, 3:].astype(np.float64)
    keep = (lo <= hi).all(axis=1)
    assert keep.sum() > 0 and np.isfinite(sph).all()
    corners = np.stack([np.where([(c >> a) & 1 for a in range(3)], hi[keep], lo[keep]) for c in range(8)])
    dist = np.linalg.norm(corners - sph[:3].astype(np.float64), axis=2)
    assert dist.max() <= float(sph[3])
    # and it is a useful cull: not much larger than the boxes' own extent
    assert float(sph[3]) < 1.5 * 0.5 * np.linalg.norm(hi[keep].max(0) - lo[keep].min(0)) + 1e-3


def test_near_tier_is_tighter(bzr):
    """The near tier exists to shrink the boxes: on cfg2 its boxes are never larger than the far
    tier's, and smaller in total."""
    patches = build_lens(bzr.TriMesh, CONFIGS["cfg2"].lenses[0]).bezier_patches()
    far, s_far = gate_boxes(bzr, patches, 0)
    near, s_near = gate_boxes(bzr, patches, 1)
    assert s_near < s_far
    ok = np.isfinite(far).all(axis=1) & (far[:, :3] <= far[:, 3:]).all(axis=1)
    assert (near[ok, :3] >= far[ok, :3]).all() and (near[ok, 3:] <= far[ok, 3:]).all()
    assert (near[ok, 3:] - near[ok, :3]).sum() < 0.99 * (far[ok, 3:] - far[ok, :3]).sum()


# ------------------------------------------------------------------ oriented boxes (wide patches)
def gate_obbs(bzr, patches, tier):
    L = bzr.lib()
    fn = L.bzr_debug_gate_obbs
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int32, ctypes.c_void_p]
    fn.restype = ctypes.c_int32
    p = np.ascontiguousarray(patches, np.float32)
    out = np.zeros((len(p), 16), np.float32)
    assert fn(p.ctypes.data, len(p), 264, tier, out.ctypes.data) == 0
    return out


def obb_f32(obbs, rays):
    """float32 replica of the kernel's obb_hit (1/x for v_rcp_f32): hit[r, i]."""
    f = np.float32
    s = rays[:3].T.astype(f)[:, None, :]
    d = rays[3:].T.astype(f)[:, None, :]
    r = (s - obbs[None, :, 0:3]).astype(f)
    tn = np.full(r.shape[:2], -np.finfo(f).max, f)
    tf = np.full(r.shape[:2], np.finfo(f).max, f)
    with np.errstate(all="ignore"):
        for a in range(3):
            u = obbs[None, :, 3 + 3 * a:6 + 3 * a]
            o = (r * u).sum(-1).astype(f)
            dd = (d * u).sum(-1).astype(f)
            dd = np.where(np.abs(dd) < f(1e-20), np.copysign(f(1e-20), dd), dd).astype(f)
            inv = (f(1) / dd).astype(f)
            h = obbs[None, :, 12 + a]
            t1, t2 = ((-h - o) * inv).astype(f), ((h - o) * inv).astype(f)
            tn, tf = np.fmax(tn, np.fmin(t1, t2)), np.fmin(tf, np.fmax(t1, t2))
    return (tn <= tf) & (tf >= 0)


def ill_conditioned(patches):
    """gamma_3 max_k l1_k sum_k |q_k| >= 1/2 (l1_k = |M_k|_1, q_k = column k of M^-1): the ill-conditioned
    patches (planes through ~the origin).  Most still have proven boxes (bvh.cpp); the rest are
    rounding_dominated()."""
    M = patches[:, 49:58].astype(np.float64).reshape(-1, 3, 3).transpose(0, 2, 1)
    fin = np.isfinite(M).all(axis=(1, 2))
    Mf = np.where(fin[:, None, None], M, np.eye(3))
    kappa = 3.0000002 * 2.0 ** -24 * np.abs(Mf).sum(axis=2).max(axis=1) * np.abs(np.linalg.inv(Mf)).max(axis=1).sum(axis=1)
    return np.nonzero(fin & (kappa >= 0.5))[0]


def rounding_dominated(patches):
    """bvh.cpp's criterion, mirrored: I - gamma_3 |M^-1| |M| is not a nonsingular M-matrix (a leading
    principal minor <= 1e-9), so no bound on where the float gate can pass; boxes use round 1's allowance."""
    M = patches[:, 49:58].astype(np.float64).reshape(-1, 3, 3).transpose(0, 2, 1)
    fin = np.isfinite(M).all(axis=(1, 2))
    Mf = np.where(fin[:, None, None], M, np.eye(3))
    A = np.eye(3)[None] - 3.0000002 * 2.0 ** -24 * np.einsum("nik,nkj->nij", np.abs(np.linalg.inv(Mf)), np.abs(Mf))
    m1, m2, m3 = A[:, 0, 0], A[:, 0, 0] * A[:, 1, 1] - A[:, 0, 1] * A[:, 1, 0], np.linalg.det(A)
    return np.nonzero(fin & ~((m1 > 1e-9) & (m2 > 1e-9) & (m3 > 1e-9)))[0]


@pytest.mark.slow
@pytest.mark.parametrize("tier", TIERS)
def test_ill_conditioned_patches_never_culled(bzr, orc, tier):
    """cfg5's ~1200 ill-conditioned patches (planes through ~the origin), 126 of them
    rounding-dominated: every gate pass of config rays and of rays aimed at those patches from near the origin
    must hit both the patch's AABB and, for wide patches, its oriented box.  (Before the untruncated region
    clip, hundreds were missed.)  The rounding-dominated ones -- whose boxes are not proven -- must be among
    the passes checked."""
    cfg = CONFIGS["cfg5"]
    patches = build_lens(bzr.TriMesh, cfg.lenses[0]).bezier_patches()
    ill = ill_conditioned(patches)
    assert len(ill) > 1000
    dominated = np.isin(ill, rounding_dominated(patches))
    assert 100 < dominated.sum() < len(ill)
    dominated_passes = 0
    boxes, smax = gate_boxes(bzr, patches, tier)
    obbs = gate_obbs(bzr, patches, tier)[ill]
    pi, bi = patches[ill], boxes[ill]
    rng = np.random.default_rng(17 + tier)
    from bzr_amd.configs import pixel_coords, rays_for
    r, c = pixel_coords(cfg, side=8192, order="rows")
    pick = rng.choice(len(r), 20000, replace=False)
    n = 20000
    aimed = []
    # all of them, then the unproven ones (aimed closer: their triangles are ~0.05 across)
    for targets, m, jitter in ((np.arange(len(ill)), n, 0.5), (np.nonzero(dominated)[0], 2 * n, 0.05)):
        o = rng.uniform(-6, 6, (m, 3))
        o[:, 0] = rng.uniform(-2, 2, m)
        tgt = pi[targets[rng.integers(0, len(targets), m)], 19:22] + rng.normal(size=(m, 3)) * jitter
        d = tgt - o
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        aimed.append(np.concatenate([o.T, d.T]).astype(np.float32))
    passes = 0
    for rays in [rays_for(cfg, r[pick], c[pick], side=8192)] + aimed:
        near = np.abs(rays[:3]).max(axis=0) <= smax
        gate = orc.planar_gate(pi, rays, threads=8) & near[:, None]
        ri, pj = np.nonzero(gate)
        passes += len(ri)
        dominated_passes += int(dominated[pj].sum())
        ur = np.unique(ri)
        k = np.searchsorted(ur, ri)
        assert slab_f32(bi, rays[:, ur])[k, pj].all()
        wide = obbs[:, 15] > 0
        assert (obb_f32(obbs, rays[:, ur])[k, pj] | ~wide[pj]).all()
    assert passes > 200 and dominated_passes > 150


def always_list(bzr, patches, tier):
    L = bzr.lib()
    fn = L.bzr_debug_always_list
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]
    fn.restype = ctypes.c_int32
    p = np.ascontiguousarray(patches, np.float32)
    cnt = np.zeros(1, np.uint32)
    assert fn(p.ctypes.data, len(p), 264, tier, None, cnt.ctypes.data) == 0
    out = np.zeros(int(cnt[0]), np.uint32)
    assert fn(p.ctypes.data, len(p), 264, tier, out.ctypes.data, cnt.ctypes.data) == 0
    return out


# A small lens with one rounding-dominated patch and no non-finite record: ellipsoid(16, 8, (1, 2, 2)) moved
# so that patch 0's plane passes within 3e-6 of the origin (its always-hit box used to make the
# illumination sphere infinite).
DOMINATED_LENS_SHIFT = (3.099341, -0.02972891, -0.16860084)


def dominated_lens(bzr):
    m = bzr.TriMesh().make_ellipsoid(16, 8, (1.0, 2.0, 2.0))
    m.translate(DOMINATED_LENS_SHIFT)
    return m.standardize().bezier_patches()


def test_bounding_sphere_survives_an_always_listed_patch(bzr):
    """The illumination sphere is built over the proven (tree) boxes only: a lens with a rounding-dominated
    patch keeps a finite sphere holding every proven box (bzr_illuminate tests the always list per ray)."""
    patches = dominated_lens(bzr)
    alw = always_list(bzr, patches, 0)
    assert len(alw) == 1 and np.isfinite(patches[:, 49:58]).all()
    boxes, _ = gate_boxes(bzr, patches)
    L = bzr.lib()
    fn = L.bzr_debug_bounding_sphere
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    fn.restype = ctypes.c_int32
    sph = np.zeros(4, np.float32)
    p = np.ascontiguousarray(patches, np.float32)
    assert fn(p.ctypes.data, len(p), 264, sph.ctypes.data) == 0
    assert np.isfinite(sph).all()
    keep = np.ones(len(p), bool)
    keep[alw] = False
    lo, hi = boxes[keep, :3].astype(np.float64), boxes[keep, 3:].astype(np.float64)
    corners = np.stack([np.where([(c >> a) & 1 for a in range(3)], hi, lo) for c in range(8)])
    assert np.linalg.norm(corners - sph[:3].astype(np.float64), axis=2).max() <= float(sph[3])
    assert float(sph[3]) < 10.0


@pytest.mark.parametrize("cfg_name,expect", [("cfg1", 0), ("cfg2", 0), ("cfg3", 0), ("cfg5", 126)])
def test_rounding_dominated_patches_are_always_tested(bzr, cfg_name, expect):
    """Culling is exact by construction: a patch is in the tree only if its gate region is proven
    (bvh.cpp: I - gamma_3 |M^-1| |M| a nonsingular M-matrix; build_bvh throws if a reachable leaf is not),
    and the others -- none of cfg1/cfg2/cfg3's or the north-star lens's (cfg4), 126 rounding-dominated + 5
    non-finite of cfg5's 301 056 -- form the always list every wave-segment gate-tests (both tiers, identical)."""
    patches = build_lens(bzr.TriMesh, CONFIGS[cfg_name].lenses[0]).bezier_patches()
    dom = rounding_dominated(patches)
    assert len(dom) == expect
    # plus the records whose M is not finite (cfg5: 5 degenerate patches; they had the always-hit box before)
    nonfinite = np.nonzero(~np.isfinite(patches[:, 49:58]).all(axis=1))[0]
    assert len(nonfinite) == (5 if cfg_name == "cfg5" else 0)
    want = np.union1d(dom, nonfinite).astype(np.uint32)
    for tier in TIERS:
        alw = always_list(bzr, patches, tier)
        assert np.array_equal(alw, want), tier
        if len(alw):  # their boxes are the always-hit box
            boxes, _ = gate_boxes(bzr, patches, tier)
            assert np.isinf(boxes[alw]).all()


def test_always_list_in_traversal_replay(bzr):
    """The host replay of the device walk reaches every always-listed patch for every active ray: 4000
    of cfg5's patch records including its 131 unproven ones (the walk reads the records only)."""
    full = build_lens(bzr.TriMesh, CONFIGS["cfg5"].lenses[0]).bezier_patches()
    rng = np.random.default_rng(3)
    pick = np.union1d(rng.choice(len(full), 4000, replace=False), np.union1d(
        rounding_dominated(full), np.nonzero(~np.isfinite(full[:, 49:58]).all(axis=1))[0]))
    patches = np.ascontiguousarray(full[pick])
    alw = always_list(bzr, patches, 0)
    assert len(alw) >= 131
    rays = random_rays(rng, 256, (10.0, 0.0, 0.0), 3.0)
    L = bzr.lib()
    fn = L.bzr_debug_traverse
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                   ctypes.c_void_p, ctypes.c_void_p]
    fn.restype = ctypes.c_int32
    hits = np.zeros((rays.shape[1], len(patches)), np.uint8)
    stats = np.zeros(4, np.uint64)
    p = np.ascontiguousarray(patches, np.float32)
    r = np.ascontiguousarray(rays)
    assert fn(p.ctypes.data, len(p), 264, r.ctypes.data, r.shape[1], hits.ctypes.data, stats.ctypes.data) == 0
    assert hits[:, alw].all()


@pytest.mark.parametrize("cfg_name", ["cfg2", "cfg5"])
def test_plane_point_rounding_within_derived_bounds(bzr, cfg_name):
    """bvh.cpp's slab and padding allowances rest on two derived bounds for the float ray/plane point p^
    of the planar gate (plane_ray, reference/3dGeomUtil.h:279-296, evaluated here in float32 in the
    kernel's operation order): off-plane distance <= 16 u (|p^| + |s|) and distance from the ray line
    <= 2 sqrt3 u (|p^| + |s|) (inf-norms, u = 2^-24).  Random, aimed and grazing rays on the config's
    patches must stay within them; the allowances themselves are 1.5x and 2x larger."""
    f, u = np.float32, 2.0 ** -24
    p = build_lens(bzr.TriMesh, CONFIGS[cfg_name].lenses[0]).bezier_patches()
    rng = np.random.default_rng(23)
    m = 200_000
    idx = rng.integers(0, len(p), m)
    n, c = p[idx, 0:3].astype(f), p[idx, 3].astype(f)
    cp = p[idx, 19:22].astype(np.float64)
    s = (cp + rng.uniform(-1, 1, (m, 3)) * rng.choice([1.0, 10.0, 80.0], (m, 1))).astype(f)
    tgt = cp + rng.normal(size=(m, 3)) * 0.3
    d = tgt - s.astype(np.float64)
    graze = rng.random(m) < 0.3  # project a third of the directions almost into the plane
    nd = n.astype(np.float64) / np.linalg.norm(n.astype(np.float64), axis=1, keepdims=True)
    d[graze] -= (d[graze] * nd[graze]).sum(1, keepdims=True) * nd[graze] * (1 - rng.uniform(1e-5, 1e-3, (graze.sum(), 1)))
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(f)

    def dot(a, b):
        return (a[:, 0] * b[:, 0] + (a[:, 1] * b[:, 1] + a[:, 2] * b[:, 2])).astype(f)

    cs = dot(d, n)
    with np.errstate(all="ignore"):
        t = ((c - dot(n, s)).astype(f) / cs).astype(f)
        ph = (s + (d * t[:, None]).astype(f)).astype(f)
    ok = (np.abs(cs) >= f(1e-5)) & (t > 0) & np.isfinite(ph).all(axis=1)
    assert ok.sum() > m // 2 and (ok & graze).sum() > m // 10
    p64, s64, d64, n64 = ph[ok].astype(np.float64), s[ok].astype(np.float64), d[ok].astype(np.float64), n[ok].astype(np.float64)
    scale = u * (np.abs(p64).max(1) + np.abs(s64).max(1))
    off = np.abs((n64 * p64).sum(1) - c[ok].astype(np.float64)) / np.linalg.norm(n64, axis=1)
    w = p64 - s64
    line = np.linalg.norm(w - (w * d64).sum(1, keepdims=True) * d64 / (d64 * d64).sum(1, keepdims=True), axis=1)
    assert (off <= 16 * scale).all(), (off / scale).max()
    assert (line <= 2 * np.sqrt(3) * scale).all(), (line / scale).max()


def always_wedges(bzr, patches, tier, count):
    L = bzr.lib()
    fn = L.bzr_debug_always_wedges
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int32, ctypes.c_void_p]
    fn.restype = ctypes.c_int32
    p = np.ascontiguousarray(patches, np.float32)
    out = np.zeros((count, 8), np.float32)
    assert fn(p.ctypes.data, len(p), 264, tier, out.ctypes.data) == 0
    return out


def wedge_keep_f32(patches, wedges, rays):
    """float32 replica of trace.hip always_gate's two pre-tests: keep[r, k] unless the lane surely fails
    (fma steps rounded once via float64; 1/x where the device uses v_rcp_f32, which the C term covers)."""
    f = np.float32
    s = rays[:3].T.astype(f)[:, None, :]
    d = rays[3:].T.astype(f)[:, None, :]
    n, c = patches[None, :, 0:3].astype(f), patches[None, :, 3].astype(f)

    def dot(a, b):
        return (a[..., 0] * b[..., 0] + (a[..., 1] * b[..., 1] + a[..., 2] * b[..., 2])).astype(f)

    with np.errstate(all="ignore"):
        cs = dot(d, n)
        num = (c - dot(n, s)).astype(f)
        keep = (np.abs(cs) >= f(1e-5)) & (((num > 0) & (cs > 0)) | ((num < 0) & (cs < 0)))
        keep |= np.isnan(num) | np.isnan(cs)
        tt = (num * (f(1) / cs)).astype(f)
        p = (d.astype(np.float64) * tt[..., None] + s.astype(np.float64)).astype(f)
        pm, sm = np.abs(p).max(-1), np.abs(s).max(-1)
        w = wedges[None, :, :3].astype(np.float64)
        z = (w[..., 2] * p[..., 2]).astype(f).astype(np.float64)
        y = (w[..., 1] * p[..., 1] + z).astype(f).astype(np.float64)
        wd = (w[..., 0] * p[..., 0] + y).astype(f)
        slack = (wedges[None, :, 5].astype(np.float64) * pm + (wedges[None, :, 6] * (sm + pm)).astype(f)).astype(f)
        hi = (wedges[None, :, 4] + slack).astype(f)
        lo = (wedges[None, :, 3] - slack).astype(f)
        keep &= ~(wd > hi) & ~(wd < lo)
    return keep


@pytest.mark.slow
def test_always_wedge_keeps_every_gate_pass(bzr, orc):
    """The always list's wedge pre-test (bvh.cpp always_wedge, trace.hip always_gate) may only reject lanes
    whose planar gate fails: every gate pass of cfg5's always-listed patches -- config rays and rays aimed
    at those patches from near the origin -- is kept, and most pairs are rejected (the point of it)."""
    cfg = CONFIGS["cfg5"]
    patches = build_lens(bzr.TriMesh, cfg.lenses[0]).bezier_patches()
    alw = always_list(bzr, patches, 0)
    wed = always_wedges(bzr, patches, 0, len(alw))
    assert np.array_equal(wed, always_wedges(bzr, patches, 1, len(alw)))
    pa = patches[alw]
    fin = np.isfinite(pa[:, 49:58]).all(axis=1)
    assert (np.isinf(wed[~fin, 3]) & np.isinf(wed[~fin, 4])).all()  # non-finite records: open wedge
    rng = np.random.default_rng(29)
    from bzr_amd.configs import pixel_coords, rays_for
    r, c = pixel_coords(cfg, side=8192, order="rows")
    pick = rng.choice(len(r), 60000, replace=False)
    sets = [rays_for(cfg, r[pick], c[pick], side=8192)]
    for m, jitter, spread in ((40000, 0.05, 6.0), (40000, 0.5, 20.0)):
        o = rng.uniform(-spread, spread, (m, 3))
        tgt = pa[fin][rng.integers(0, fin.sum(), m), 19:22] + rng.normal(size=(m, 3)) * jitter
        d = tgt - o
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        sets.append(np.concatenate([o.T, d.T]).astype(np.float32))
    passes = kept = total = 0
    for k, rays in enumerate(sets):
        gate = orc.planar_gate(pa, rays, threads=8)
        keep = wedge_keep_f32(pa, wed, rays)
        missed = gate & ~keep
        assert not missed.any(), f"set {k}: {int(missed.sum())} gate passes rejected, e.g. {np.argwhere(missed)[:4]}"
        passes += int(gate.sum())
        if k == 0:
            kept, total = int(keep.sum()), keep.size
    assert passes > 100
    assert kept < 0.1 * total  # the config rays: most (ray, always patch) pairs never reach the gate


def bundle_keep_f32(patches, wedges, rays):
    """float32 replica of trace.hip always_bundle_keep: keep[w, k] for waves of 64 consecutive rays
    (all active) against always-listed patches (records `patches`, wedge words `wedges`)."""
    f = np.float32
    u = f(2.0 ** -24)
    nw = rays.shape[1] // 64
    r = rays[:, :nw * 64].reshape(6, nw, 64).astype(f)
    slo, shi = r[:3].min(axis=2).T, r[:3].max(axis=2).T  # [nw, 3]
    dlo, dhi = r[3:].min(axis=2).T, r[3:].max(axis=2).T
    fin = np.abs(np.concatenate([slo, shi, dlo, dhi], 1)).max(1) <= f(1e30)
    S = lambda a: a[:, None, :]  # noqa: E731  [nw, 1, 3]
    n = patches[None, :, 0:3].astype(f)
    c = patches[None, :, 3].astype(f)

    def ivdot(v, lo, hi):
        a = np.where(v >= 0, v * lo, v * hi).astype(f)
        b = np.where(v >= 0, v * hi, v * lo).astype(f)
        return (((a[..., 0] + a[..., 1]).astype(f) + a[..., 2]).astype(f),
                ((b[..., 0] + b[..., 1]).astype(f) + b[..., 2]).astype(f))

    def amax(lo, hi):
        return np.maximum(np.abs(lo), np.abs(hi))

    with np.errstate(all="ignore"):
        csl, csh = ivdot(n, S(dlo), S(dhi))
        nsl, nsh = ivdot(n, S(slo), S(shi))
        ad, asv = amax(S(dlo), S(dhi)), amax(S(slo), S(shi))
        mc = (f(8) * u * ((np.abs(n[..., 0]) * ad[..., 0] + np.abs(n[..., 1]) * ad[..., 1]).astype(f) + np.abs(n[..., 2]) * ad[..., 2])).astype(f)
        ms = (f(8) * u * (((np.abs(n[..., 0]) * asv[..., 0] + np.abs(n[..., 1]) * asv[..., 1]).astype(f) + np.abs(n[..., 2]) * asv[..., 2]).astype(f) + np.abs(c))).astype(f)
        csl, csh = (csl - mc).astype(f), (csh + mc).astype(f)
        numl, numh = ((c - nsh) - ms).astype(f), ((c - nsl) + ms).astype(f)
        tiny = (csl > f(-1e-5)) & (csh < f(1e-5))
        open_ = ~((csl > 0) | (csh < 0))
        r1, r2 = (f(1) / csl).astype(f), (f(1) / csh).astype(f)
        a = np.stack([numl * r1, numl * r2, numh * r1, numh * r2]).astype(f)
        tlo, thi = np.fmin.reduce(a, 0), np.fmax.reduce(a, 0)
        tlo = (tlo - f(6) * u * np.abs(tlo)).astype(f)
        thi = (thi + f(6) * u * np.abs(thi)).astype(f)
        unb = ~(thi <= f(1e30))
        neg = thi <= 0
        tlo = np.maximum(tlo, f(0))
        plo, phi = [], []
        for ax in range(3):
            x = np.stack([S(dlo)[..., ax] * tlo, S(dlo)[..., ax] * thi, S(dhi)[..., ax] * tlo, S(dhi)[..., ax] * thi]).astype(f)
            plo.append((S(slo)[..., ax] + np.fmin.reduce(x, 0)).astype(f))
            phi.append((S(shi)[..., ax] + np.fmax.reduce(x, 0)).astype(f))
        plo, phi = np.stack(plo, -1), np.stack(phi, -1)
        smax = amax(slo, shi).max(1)[:, None]
        pm0 = amax(plo, phi).max(-1)
        e = (f(8) * u * (smax + pm0)).astype(f)
        pmax = (pm0 + e).astype(f)
        w = wedges[None, :, 0:3].astype(f)
        wlo, whi = ivdot(w, plo - e[..., None], phi + e[..., None])
        slack = (wedges[None, :, 5] * pmax + (wedges[None, :, 6] + f(64) * u) * (smax + pmax)).astype(f)
        keep = ~(wlo > wedges[None, :, 4] + slack) & ~(whi < wedges[None, :, 3] - slack)
    keep = np.where(open_ | unb, True, np.where(tiny | neg, False, keep))
    return np.where(fin[:, None], keep, True)


@pytest.mark.slow
def test_always_bundle_keeps_every_wave_with_a_gate_pass(bzr, orc):
    """The wave-level bundle test (trace.hip always_bundle_keep) may only drop an always-listed patch for a
    wave when no ray of that wave passes the patch's gate: cfg5 grid waves (8x8 pixel blocks) and waves of
    rays aimed at those patches from near the origin (64 rays per target, jittered origins and targets).
    Most (wave, patch) pairs of the grid are dropped."""
    cfg = CONFIGS["cfg5"]
    patches = build_lens(bzr.TriMesh, cfg.lenses[0]).bezier_patches()
    alw = always_list(bzr, patches, 0)
    wed = always_wedges(bzr, patches, 0, len(alw))
    pa = patches[alw]
    fin = np.isfinite(pa[:, 49:58]).all(axis=1)
    from bzr_amd.configs import pixel_coords, rays_for
    rng = np.random.default_rng(31)
    r, c = pixel_coords(cfg, side=8192, order="tiles")
    starts = rng.integers(0, len(r) // 64, 600) * 64
    idx = (starts[:, None] + np.arange(64)[None, :]).reshape(-1)
    sets = [rays_for(cfg, r[idx], c[idx], side=8192)]
    for jitter_o, jitter_t in ((0.05, 0.01), (0.5, 0.05)):
        m = 64 * 400
        tk = rng.integers(0, fin.sum(), 400).repeat(64)
        o0 = rng.uniform(-6, 6, (400, 3)).repeat(64, 0)
        o = o0 + rng.normal(size=(m, 3)) * jitter_o
        tgt = pa[fin][tk, 19:22] + rng.normal(size=(m, 3)) * jitter_t
        d = tgt - o
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        sets.append(np.concatenate([o.T, d.T]).astype(np.float32))
    passes = 0
    for k, rays in enumerate(sets):
        gate = orc.planar_gate(pa, rays, threads=8).reshape(-1, 64, len(pa)).any(axis=1)
        keep = bundle_keep_f32(pa, wed, rays)
        missed = gate & ~keep
        assert not missed.any(), f"set {k}: {int(missed.sum())} (wave, patch) gate passes dropped"
        passes += int(gate.sum())
        if k == 0:
            assert keep.mean() < 0.15, keep.mean()
    assert passes > 50


def traverse_bundle(bzr, patches, rays):
    """bzr_debug_traverse_bundle stats: waves, batches, bundle leaves, lane node visits, lane leaves,
    lane leaves the bundle walk missed, child slots, deepest work stack."""
    L = bzr.lib()
    fn = L.bzr_debug_traverse_bundle
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_float,
                   ctypes.c_void_p]
    fn.restype = ctypes.c_int32
    p = np.ascontiguousarray(patches, np.float32)
    r = np.ascontiguousarray(rays, np.float32)
    st = np.zeros(12, np.uint64)
    assert fn(p.ctypes.data, len(p), 264, r.ctypes.data, r.shape[1], np.float32(np.inf), st.ctypes.data) == 0
    return st


def coherent_waves(rng, waves, centre, spread, jitter):
    """Waves of 64 nearly parallel rays: a random origin and direction per wave, origins spread over a small
    square, directions jittered; a quarter of the waves get one exactly-zero direction component."""
    c = np.asarray(centre, np.float64)
    out = []
    for _ in range(waves):
        o0 = c + rng.uniform(-spread, spread, 3) * 3.0
        d0 = c + rng.uniform(-spread, spread, 3) - o0
        d0 /= np.linalg.norm(d0)
        o = o0 + rng.uniform(-1, 1, (64, 3)) * jitter * spread
        d = d0 + rng.uniform(-1, 1, (64, 3)) * jitter
        if rng.random() < 0.25:
            d[:, rng.integers(0, 3)] = 0.0
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        out.append(np.concatenate([o.T, d.T]))
    return np.concatenate(out, axis=1).astype(np.float32)


@pytest.mark.parametrize("cfg_name", ["cfg2", "cfg3", "cfg5"])
def test_bundle_walk_keeps_every_lane_leaf(bzr, cfg_name):
    """The bundle walk (trace.hip bundle_box, BZR_TRACE_BUNDLE; host mirror bvh.cpp bundle_box_h) reaches
    every leaf the per-lane slab walk reaches, for every wave: config primaries (8x8 tiles) and coherent
    random waves of several spreads, including axis-parallel directions -- a wave-level box test that dropped
    one would lose a candidate patch."""
    cfg = CONFIGS[cfg_name]
    patches = build_lens(bzr.TriMesh, cfg.lenses[0]).bezier_patches()
    if cfg_name == "cfg5":
        rng0 = np.random.default_rng(5)
        keep = np.sort(rng0.choice(len(patches), 20000, replace=False))
        patches = np.ascontiguousarray(patches[keep])
    rng = np.random.default_rng(11)
    side = 256 if cfg_name != "cfg3" else 512
    grid = grid_rays(cfg, side=side)
    lo, hi = patches[:, 19:49].reshape(-1, 10, 3).min(axis=(0, 1)), patches[:, 19:49].reshape(-1, 10, 3).max(axis=(0, 1))
    centre, spread = (lo + hi) / 2, float((hi - lo).max()) / 2
    for rays in (grid, coherent_waves(rng, 150, centre, spread, 1e-3), coherent_waves(rng, 150, centre, spread, 3e-2)):
        st = traverse_bundle(bzr, patches, rays)
        assert st[0] > 0 and st[4] > 0
        assert st[5] == 0, f"bundle walk missed {int(st[5])} leaves"
        assert st[11] == 0, f"leaf pre-test rejected {int(st[11])} leaves with a passing gate"
        assert st[2] >= st[4]  # a superset of the per-lane walk's leaves (each counted once per wave)
