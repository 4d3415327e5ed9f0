"""GPU parity: libbzr's HIP kernels vs the CPU oracle on identical rays and patch records.

Parity mode evaluates with the reference's operation order and no contraction,
so the bar is bit-identical output.  BASELINE.json's north-star tolerance
(t and barycentrics within 1e-5 relative) is asserted too, so a failure report
says which bar broke.  Oracle pinning status: oracle/bzr_oracle.h.
"""
import numpy as np
import pytest

from bzr_amd.configs import CONFIGS, build_lens, grid_rays, pixel_coords, rays_for, shard_pixels

pytestmark = pytest.mark.gpu

REL_TOL = 1e-5  # north_star: t-values and barycentrics within 1e-5 relative fp32


def hits_report(got, want):
    gu, wu = got.view(np.uint32), want.view(np.uint32)
    differ = (gu != wu).any(axis=0)
    same_class = (gu[11] == wu[11]) & (gu[12] == wu[12])
    hit = same_class & (wu[11] == 4)
    def rel(a, b):
        return np.abs(a - b) / np.maximum(np.abs(b), 1e-30)
    worst_t = float(rel(got[0][hit], want[0][hit]).max()) if hit.any() else 0.0
    worst_b = float(max(rel(got[k][hit], want[k][hit]).max() for k in (5, 6, 7))) if hit.any() else 0.0
    return int(differ.sum()), int((~same_class).sum()), worst_t, worst_b


def assert_hits_equal(got, want, label=""):
    n_diff, n_class, worst_t, worst_b = hits_report(got, want)
    assert n_class == 0, f"{label}: {n_class} rays hit a different patch / class than the oracle"
    assert worst_t <= REL_TOL and worst_b <= REL_TOL, f"{label}: t rel {worst_t:.3g}, bary rel {worst_b:.3g}"
    assert n_diff == 0, f"{label}: {n_diff} rays not bit-identical (within 1e-5 rel though)"


@pytest.fixture(scope="module")
def meshes(bzr):
    out = {}
    for name in ("cfg1", "cfg2", "cfg3"):
        out[name] = [build_lens(bzr.TriMesh, lens).bezier_patches() for lens in CONFIGS[name].lenses]
    return out


def test_cfg1_full_grid_intersect(bzr, orc, ctx, meshes, pipe):
    cfg = CONFIGS["cfg1"]
    patches = meshes["cfg1"][0]
    rays = grid_rays(cfg)  # the full 256x256 config
    got = bzr.intersect(ctx, bzr.DeviceMesh(ctx, patches), rays, mode=pipe)
    want = orc.intersect(patches, rays)
    assert_hits_equal(got, want, "cfg1")
    assert abs((want.view(np.uint32)[11] == 4).mean() - 0.3433) < 5e-4  # 34.33 % hits


def test_cfg2_chain_and_single_refracts(bzr, orc, ctx, meshes, pipe):
    cfg = CONFIGS["cfg2"]
    lens = meshes["cfg2"][0]
    rays = grid_rays(cfg, side=128)
    dm = bzr.DeviceMesh(ctx, lens)
    o, s, g = bzr.trace_chain(ctx, [dm], [1.3], rays, mode=pipe)
    wo, ws, wg = orc.trace_chain([lens], [1.3], rays)
    assert np.array_equal(s, ws) and np.array_equal(g, wg)
    assert np.array_equal(o.view(np.uint32), wo.view(np.uint32))
    # the same chain as two single refract() calls
    n = rays.shape[1]
    o1, s1 = bzr.refract(ctx, dm, 1.3, rays, np.full(n, 1, np.uint32), mode=pipe)
    w1, ws1 = orc.refract(lens, 1.3, rays, np.full(n, 1, np.uint32))
    assert np.array_equal(s1, ws1) and np.array_equal(o1.view(np.uint32), w1.view(np.uint32))
    o2, s2 = bzr.refract(ctx, dm, 1.3, o1, None, expected_all=2, mode=pipe)
    w2, ws2 = orc.refract(lens, 1.3, w1, np.full(n, 2, np.uint32))
    alive = ws1 != 0
    assert np.array_equal(s2[alive], ws2[alive])
    assert abs(g.mean() - 1.68) < 0.02  # 1.68 segments / primary


def test_cfg4_two_lens_chain(bzr, orc, ctx, meshes, pipe):
    cfg = CONFIGS["cfg4"]
    lenses = [build_lens(bzr.TriMesh, l).bezier_patches() for l in cfg.lenses]
    rays = grid_rays(cfg, side=96)
    dms = [bzr.DeviceMesh(ctx, p) for p in lenses]
    o, s, g = bzr.trace_chain(ctx, dms, [1.3, 1.3], rays, mode=pipe)
    wo, ws, wg = orc.trace_chain(lenses, [1.3, 1.3], rays)
    assert np.array_equal(s, ws) and np.array_equal(g, wg)
    assert np.array_equal(o.view(np.uint32), wo.view(np.uint32))


def test_cfg3_robot_intersect(bzr, orc, ctx, meshes, pipe):
    cfg = CONFIGS["cfg3"]
    patches = meshes["cfg3"][0]
    assert len(patches) == 28800
    r, c = pixel_coords(cfg, side=2048)
    pick = np.random.default_rng(3).choice(len(r), 3000, replace=False)
    rays = rays_for(cfg, r[pick], c[pick], side=2048)
    got = bzr.intersect(ctx, bzr.DeviceMesh(ctx, patches), rays, mode=pipe)
    want = orc.intersect(patches, rays)
    assert_hits_equal(got, want, "cfg3")


def test_patch_intersect_aimed_rays(bzr, orc, ctx, meshes):
    """BezierTriangle::intersect directly, both limits, rays aimed at random points of random patches."""
    patches = meshes["cfg2"][0]
    rng = np.random.default_rng(11)
    n = 2000
    idx = rng.integers(0, len(patches), n).astype(np.uint32)
    limit = rng.integers(0, 2, n).astype(np.uint32)
    cp = patches[:, 19:49].reshape(-1, 10, 3)
    w = rng.dirichlet((1, 1, 1), n).astype(np.float32)
    target = (cp[idx, 0] * w[:, :1] + cp[idx, 1] * w[:, 1:2] + cp[idx, 2] * w[:, 2:3]).astype(np.float32)
    origin = np.stack([np.zeros(n), rng.uniform(-5, 5, n), rng.uniform(-3, 3, n)], 1).astype(np.float32)
    d = target - origin
    d = d / np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([origin.T, d.T.astype(np.float32)]).astype(np.float32)
    dm = bzr.DeviceMesh(ctx, patches)
    got = bzr.patch_intersect(ctx, dm, idx, limit, rays)
    want = orc.patch_intersect(patches, idx, limit, rays)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    assert (want.view(np.uint32)[11] == 4).sum() > n // 4  # most aimed rays hit their patch


@pytest.mark.parametrize("center", [0.0, 10.0])
def test_seeded_cone_rays(bzr, orc, ctx, center, pipe):
    """SURVEY 8c fixture F4: 4096 rays, jittered origins on x=0, directions in a +-15 degree cone."""
    m = bzr.TriMesh().make_ellipsoid(32, 16, (1.0, 4.0, 2.0)).translate((center, 0.0, 0.0)).standardize()
    patches = m.bezier_patches()
    rng = np.random.default_rng(0x5EED)
    n = 4096
    start_x = -3.0 if center == 0.0 else 0.0
    org = np.stack([np.full(n, start_x), rng.uniform(-4, 4, n), rng.uniform(-2, 2, n)], 1)
    ang = np.radians(15.0)
    th, ph = rng.uniform(0, ang, n), rng.uniform(0, 2 * np.pi, n)
    d = np.stack([np.cos(th), np.sin(th) * np.cos(ph), np.sin(th) * np.sin(ph)], 1).astype(np.float32)
    rays = np.concatenate([org.T, d.T]).astype(np.float32)
    got = bzr.intersect(ctx, bzr.DeviceMesh(ctx, patches), rays, mode=pipe)
    want = orc.intersect(patches, rays)
    assert_hits_equal(got, want, f"cone@{center}")


def test_edge_cases(bzr, orc, ctx, meshes, pipe):
    patches = meshes["cfg1"][0]
    dm = bzr.DeviceMesh(ctx, patches)
    cfg = CONFIGS["cfg1"]
    # empty batch
    out = bzr.intersect(ctx, dm, np.zeros((6, 0), np.float32))
    assert out.shape == (13, 0)
    # ragged sizes around the 256-thread block
    for n in (1, 63, 255, 257, 1000):
        rays = grid_rays(cfg, side=64, order="rows")[:, :n].copy()
        assert_hits_equal(bzr.intersect(ctx, dm, rays, mode=pipe), orc.intersect(patches, rays), f"n={n}")
    # empty mesh: every ray misses
    empty = bzr.DeviceMesh(ctx, np.zeros((0, 66), np.float32))
    h = bzr.intersect(ctx, empty, grid_rays(cfg, side=16), mode=pipe)
    assert (h.view(np.uint32)[11] == 3).all() and (h[0] == np.finfo(np.float32).max).all()
    # degenerate directions: zero vector, grazing (parallel to x planes), backwards
    rays = np.zeros((6, 4), np.float32)
    rays[:, 1] = (-5, 0.1, 0.2, 0, 1, 0)
    rays[:, 2] = (-5, 0.1, 0.2, -1, 0, 0)
    rays[:, 3] = (0.0, 0.0, 0.0, 1, 0, 0)  # starts inside the sphere
    assert_hits_equal(bzr.intersect(ctx, dm, rays, mode=pipe), orc.intersect(patches, rays), "degenerate")


def test_device_pointer_path_and_determinism(bzr, orc, ctx, meshes):
    torch = pytest.importorskip("torch")
    cfg = CONFIGS["cfg2"]
    lens = meshes["cfg2"][0]
    rays = grid_rays(cfg, side=64)
    dm = bzr.DeviceMesh(ctx, lens)
    stream = torch.cuda.Stream()
    ctx.use_torch_stream(stream)
    try:
        torch.cuda.set_stream(stream)
        tr = torch.from_numpy(rays).cuda()
        o, s, g = bzr.trace_chain(ctx, [dm], [1.3], tr)
        torch.cuda.synchronize()
        o2, s2, g2 = bzr.trace_chain(ctx, [dm], [1.3], tr)
        torch.cuda.synchronize()
    finally:
        torch.cuda.set_stream(torch.cuda.default_stream())
        ctx.use_own_stream()
    ho, hs, hg = bzr.trace_chain(ctx, [dm], [1.3], rays)
    assert np.array_equal(o.cpu().numpy().view(np.uint32), ho.view(np.uint32))
    assert np.array_equal(s.cpu().numpy().astype(np.uint32), hs) and np.array_equal(g.cpu().numpy().astype(np.uint32), hg)
    assert torch.equal(o, o2) and torch.equal(s, s2) and torch.equal(g, g2)


@pytest.mark.slow
def test_cfg2_full_size_chain(bzr, orc, ctx, meshes, pipe):
    """BASELINE configs[1] at its full 1024x1024 size against the oracle (a few seconds of CPU)."""
    cfg = CONFIGS["cfg2"]
    lens = meshes["cfg2"][0]
    rays = grid_rays(cfg)
    o, s, g = bzr.trace_chain(ctx, [bzr.DeviceMesh(ctx, lens)], [1.3], rays, mode=pipe)
    wo, ws, wg = orc.trace_chain([lens], [1.3], rays)
    assert np.array_equal(s, ws) and np.array_equal(g, wg)
    assert np.array_equal(o.view(np.uint32), wo.view(np.uint32))


@pytest.mark.slow
def test_cfg4_full_size_properties(bzr, orc, ctx):
    """cfg4 at 4096x4096: too slow for the oracle in full, so check size-independent properties --
    sharded runs reassemble to the unsharded result, and a random sample matches the oracle."""
    torch = pytest.importorskip("torch")
    cfg = CONFIGS["cfg4"]
    lenses = [build_lens(bzr.TriMesh, l).bezier_patches() for l in cfg.lenses]
    dms = [bzr.DeviceMesh(ctx, p) for p in lenses]
    rays = torch.from_numpy(grid_rays(cfg)).cuda()
    torch.cuda.synchronize()
    ctx.use_torch_stream()  # torch's current (null) stream: torch ops below are ordered with the kernels
    try:
        o, s, g = bzr.trace_chain(ctx, dms, [1.3, 1.3], rays)
        # two-rank sharding of the same image, computed separately and scattered back
        r, c = pixel_coords(cfg)
        flat = (r * cfg.side + c)
        order = np.empty_like(flat)
        order[flat] = np.arange(len(flat))
        parts = []
        for rank in range(2):
            rr, cc = shard_pixels(cfg, rank, 2)
            sub = torch.from_numpy(rays_for(cfg, rr, cc)).cuda()
            so, ss, sg = bzr.trace_chain(ctx, dms, [1.3, 1.3], sub)
            parts.append((order[rr * cfg.side + cc], so, ss, sg))
        torch.cuda.synchronize()
    finally:
        ctx.use_own_stream()
    for pos, so, ss, sg in parts:
        p = torch.from_numpy(pos).cuda()
        assert torch.equal(o[:, p], so) and torch.equal(s[p], ss) and torch.equal(g[p], sg)
    pick = np.random.default_rng(4).choice(rays.shape[1], 2048, replace=False)
    sample = rays[:, torch.from_numpy(pick).cuda()].cpu().numpy()
    wo, ws, wg = orc.trace_chain(lenses, [1.3, 1.3], sample)
    assert np.array_equal(s[torch.from_numpy(pick).cuda()].cpu().numpy().astype(np.uint32), ws)
    assert np.array_equal(o[:, torch.from_numpy(pick).cuda()].cpu().numpy().view(np.uint32), wo.view(np.uint32))


# ---------------------------------------------------------------- culled == brute force
def test_culled_equals_bruteforce_cfg2_full(bzr, ctx, meshes, pipe):
    """Default (BVH-culled) chain vs the brute-force scan over the full cfg2 image: every bit equal."""
    cfg = CONFIGS["cfg2"]
    dm = bzr.DeviceMesh(ctx, meshes["cfg2"][0])
    rays = grid_rays(cfg)
    a = bzr.trace_chain(ctx, [dm], [1.3], rays, mode=pipe)
    b = bzr.trace_chain(ctx, [dm], [1.3], rays, mode=bzr.ACCEL_NONE)
    for x, y in zip(a, b):
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32))


def test_culled_equals_bruteforce_robot_and_random(bzr, orc, ctx, meshes, pipe):
    cfg = CONFIGS["cfg3"]
    dm = bzr.DeviceMesh(ctx, meshes["cfg3"][0])
    rays = grid_rays(cfg, side=512)
    a = bzr.intersect(ctx, dm, rays, mode=pipe)
    b = bzr.intersect(ctx, dm, rays, mode=bzr.ACCEL_NONE)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    # far origins on the robot mesh: every ray takes the overflow scan, which splits the 28800 patches
    # into 15 slices per ray (k_overflow), so the cross-slice (t, patch) minimum is exercised
    rng = np.random.default_rng(22)
    lo, hi = meshes["cfg3"][0][:, 19:49].reshape(-1, 3).min(0), meshes["cfg3"][0][:, 19:49].reshape(-1, 3).max(0)
    tgt = rng.uniform(lo, hi, (20000, 3))
    o = tgt + rng.normal(size=(20000, 3)) * 1e4 * np.abs(hi - lo).max()
    d = (tgt - o) / np.linalg.norm(tgt - o, axis=1, keepdims=True)
    far = np.concatenate([o.T, d.T]).astype(np.float32)
    a = bzr.intersect(ctx, dm, far, mode=pipe)
    b = bzr.intersect(ctx, dm, far, mode=bzr.ACCEL_NONE)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert (a.view(np.uint32)[11] == 4).mean() > 0.05
    # random rays from everywhere around the cfg2 lens, incl. axis-parallel directions and far origins
    rng = np.random.default_rng(21)
    n = 200000
    o = rng.uniform(-20, 30, (n, 3)).astype(np.float32)
    tgt = (np.array([10, 0, 0]) + rng.uniform(-2, 2, (n, 3)) * np.array([1, 4, 2])).astype(np.float32)
    d = tgt - o
    z = rng.random(n) < 0.2
    d[z, rng.integers(0, 3, z.sum())] = 0.0
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    far = rng.random(n) < 0.01
    o[far] *= 1e4  # beyond the culling radius: full-scan fallback
    rays = np.concatenate([o.T, d.T]).astype(np.float32)
    dm2 = bzr.DeviceMesh(ctx, meshes["cfg2"][0])
    a = bzr.intersect(ctx, dm2, rays, mode=pipe)
    b = bzr.intersect(ctx, dm2, rays, mode=bzr.ACCEL_NONE)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert (a.view(np.uint32)[11] == 4).mean() > 0.1
    o1, s1 = bzr.refract(ctx, dm2, 1.3, rays, None, expected_all=1, mode=pipe)
    o2, s2 = bzr.refract(ctx, dm2, 1.3, rays, None, expected_all=1, mode=bzr.ACCEL_NONE)
    assert np.array_equal(s1, s2) and np.array_equal(o1.view(np.uint32), o2.view(np.uint32))


@pytest.mark.slow
def test_cfg5_sample_against_oracle(bzr, orc, ctx, pipe):
    """cfg5 (301056 patches): a sample of its 8192^2 grid, culled GPU path vs the oracle."""
    cfg = CONFIGS["cfg5"]
    patches = build_lens(bzr.TriMesh, cfg.lenses[0]).bezier_patches()
    r, c = pixel_coords(cfg, side=8192, order="rows")
    pick = np.random.default_rng(5).choice(len(r), 384, replace=False)
    rays = rays_for(cfg, r[pick], c[pick], side=8192)
    got = bzr.intersect(ctx, bzr.DeviceMesh(ctx, patches), rays, mode=pipe)
    want = orc.intersect(patches, rays, threads=16)
    assert_hits_equal(got, want, "cfg5")


def test_mixed_size_lenses_and_mesh_switching(bzr, orc, ctx, meshes, pipe):
    """Lenses of different patch counts in one chain, and one context switching between meshes of
    different sizes (small-scan and hipCUB paths): every segment must start from zeroed counters and
    histogram whichever mesh ran before it."""
    small = bzr.TriMesh().make_ellipsoid(8, 4, (1.0, 3.0, 1.5)).translate((13.0, 0.0, 0.0)).standardize()
    lenses = [meshes["cfg2"][0], small.bezier_patches()]
    assert len(lenses[0]) != len(lenses[1])
    rays = grid_rays(CONFIGS["cfg2"], side=96)
    dms = [bzr.DeviceMesh(ctx, p) for p in lenses]
    for order in ([0, 1], [1, 0]):
        got = bzr.trace_chain(ctx, [dms[k] for k in order], [1.3, 1.5], rays, mode=pipe)
        want = orc.trace_chain([lenses[k] for k in order], [1.3, 1.5], rays)
        for g, w in zip(got, want):
            assert np.array_equal(np.asarray(g).view(np.uint32), np.asarray(w).view(np.uint32))
    # intersect calls alternating between a small mesh, the robot (hipCUB scan) and cfg2
    robot = bzr.DeviceMesh(ctx, meshes["cfg3"][0])
    seq = [(dms[1], lenses[1]), (robot, meshes["cfg3"][0]), (dms[0], lenses[0]), (dms[1], lenses[1]), (dms[0], lenses[0])]
    r3 = grid_rays(CONFIGS["cfg3"], side=32)
    for dm, p in seq:
        rr = r3 if dm is robot else rays[:, :2048]
        got = bzr.intersect(ctx, dm, rr, mode=pipe)
        assert np.array_equal(got.view(np.uint32), orc.intersect(p, rr).view(np.uint32))


@pytest.mark.slow
def test_culled_equals_bruteforce_cfg3_full(bzr, ctx, meshes, pipe):
    """cfg3 (robot.stl x8 split, 28 800 patches) at its full 2048x2048 grid: culled == brute force, every bit."""
    dm = bzr.DeviceMesh(ctx, meshes["cfg3"][0])
    rays = grid_rays(CONFIGS["cfg3"])
    assert rays.shape[1] == 2048 * 2048
    a = bzr.intersect(ctx, dm, rays, mode=pipe)
    b = bzr.intersect(ctx, dm, rays, mode=bzr.ACCEL_NONE)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert abs((a.view(np.uint32)[11] == 4).mean() - 0.2505) < 0.001  # 25.05 % of the 2048^2 grid (27.0 % on a 64^2 grid)


@pytest.mark.slow
def test_culled_equals_bruteforce_cfg5_ill_conditioned(bzr, ctx, pipe):
    """cfg5 (301 056 patches, ~1200 of them rounding-dominated): culled == brute force on
    131 072 grid rays and 131 072 rays from near the origin aimed at the ill-conditioned patches."""
    cfg = CONFIGS["cfg5"]
    patches = build_lens(bzr.TriMesh, cfg.lenses[0]).bezier_patches()
    M = patches[:, 49:58].astype(np.float64).reshape(-1, 3, 3).transpose(0, 2, 1)
    fin = np.isfinite(M).all(axis=(1, 2))
    Mf = np.where(fin[:, None, None], M, np.eye(3))
    kappa = 3.0000002 * 2.0 ** -24 * np.abs(Mf).sum(axis=2).max(axis=1) * np.abs(np.linalg.inv(Mf)).max(axis=1).sum(axis=1)
    ill = np.nonzero(fin & (kappa >= 0.5))[0]
    rng = np.random.default_rng(55)
    r, c = pixel_coords(cfg, side=8192, order="tiles")
    start = rng.integers(0, len(r) // 64 - 2048) * 64
    grid = rays_for(cfg, r[start:start + 131072], c[start:start + 131072], side=8192)
    n = 131072
    o = rng.uniform(-6, 6, (n, 3))
    o[:, 0] = rng.uniform(-2, 2, n)
    tgt = patches[ill[rng.integers(0, len(ill), n)], 19:22] + rng.normal(size=(n, 3)) * 0.5
    d = (tgt - o) / np.linalg.norm(tgt - o, axis=1, keepdims=True)
    rays = np.concatenate([grid, np.concatenate([o.T, d.T]).astype(np.float32)], axis=1)
    dm = bzr.DeviceMesh(ctx, patches)
    a = bzr.intersect(ctx, dm, rays, mode=pipe)
    b = bzr.intersect(ctx, dm, rays, mode=bzr.ACCEL_NONE)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert (a.view(np.uint32)[11] == 4).mean() > 0.2


@pytest.mark.slow
def test_staged_ragged_chunks_equal_bruteforce(bzr, ctx, meshes):
    """The staged pipeline over a batch of two chunks of unequal, non-wave-multiple length (2900^2 = 8 410 000 rays
    against 8 M-ray chunks: the batch is split into 4 205 056 + 4 204 944 rays), intersect and the chain: every bit
    equal to the brute-force scan, so no ray is lost or doubled at the chunk seam and each chunk starts from zeroed
    counters and histogram."""
    cfg = CONFIGS["cfg2"]
    dm = bzr.DeviceMesh(ctx, meshes["cfg2"][0])
    rays = grid_rays(cfg, side=2900)
    assert rays.shape[1] == 8_410_000 > 1 << 23
    a = bzr.intersect(ctx, dm, rays, mode=bzr.PIPELINE_STAGED)
    b = bzr.intersect(ctx, dm, rays, mode=bzr.ACCEL_NONE)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert (a.view(np.uint32)[11] == 4).mean() > 0.2
    del a, b
    x = bzr.trace_chain(ctx, [dm], [1.3], rays, mode=bzr.PIPELINE_STAGED)
    y = bzr.trace_chain(ctx, [dm], [1.3], rays, mode=bzr.ACCEL_NONE)
    for p, q in zip(x, y):
        assert np.array_equal(np.asarray(p).view(np.uint32), np.asarray(q).view(np.uint32))
