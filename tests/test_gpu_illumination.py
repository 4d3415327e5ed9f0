"""Illumination pipeline (reference/README.md:159-194) on the GPU vs the oracle.

emitter (UniformHemisphere's distribution, counter-based stream) -> Ritter bounding-sphere pre-cull ->
refraction chain -> target-plane counts.  The emitted rays must equal the oracle's restatement bit
for bit; the pipeline's counts must equal the oracle's brute-force chain over *every* emitted ray
(no cull) followed by the same binning -- which also proves the sphere cull drops only rays the
reference would have missed.
"""
import numpy as np
import pytest

from bzr_amd.configs import CONFIGS, build_lens

pytestmark = pytest.mark.gpu


def emitter(bzr_or_orc, seed=7, parts=(2, 2), points=64, rays=128, belts=16, x=0.0):
    return bzr_or_orc.Emitter(origin=(x, -0.5, -0.5), edge_u=(0.0, 1.0, 0.0), edge_v=(0.0, 0.0, 1.0),
                              parts_u=parts[0], parts_v=parts[1], points_per_part=points, rays_per_point=rays,
                              belts=belts, seed=seed)


def target(mod, x=25.0):
    return mod.Target(origin=(x, -12.0, -12.0), axis_u=(0.0, 1.0, 0.0), axis_v=(0.0, 0.0, 1.0), size_u=24.0,
                      size_v=24.0, bins_u=48, bins_v=48)


def test_emit_matches_oracle(bzr, orc, ctx):
    first, n = 12345, 100000
    rays, patch = bzr.emit(ctx, emitter(bzr), first, n)
    want_rays, want_patch = orc.emit(emitter(orc), first, n)
    assert np.array_equal(rays.view(np.uint32), want_rays.view(np.uint32))
    assert np.array_equal(patch, want_patch)
    # the distribution UniformHemisphere::getRandom samples: cos(incidence) uniform in [0, 1), unit
    # directions, patch numbers within UniformHemisphere(16)'s count
    assert np.allclose(np.linalg.norm(rays[3:], axis=0), 1.0, atol=1e-6)
    assert (rays[3] >= 0).all() and abs(float(rays[3].mean()) - 0.5) < 0.01
    count = orc.Hemisphere(16).patch_count
    assert patch.max() < count
    hist = np.bincount(patch, minlength=count)
    assert hist.min() > 0.5 * n / count and hist.max() < 1.6 * n / count  # equal-area patches
    # origins on the emitter rectangle x = 0, y, z in [-0.5, 0.5)
    assert (rays[0] == 0).all() and (np.abs(rays[1:3]) <= 0.5).all()


def test_emit_device_buffers(bzr, ctx):
    torch = pytest.importorskip("torch")
    n = 4096
    r = torch.empty((6, n), dtype=torch.float32, device="cuda")
    p = torch.empty(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ctx.use_torch_stream()
    try:
        bzr.emit(ctx, emitter(bzr), 0, n, rays=r, patch=p)
        torch.cuda.synchronize()
    finally:
        ctx.use_own_stream()
    hr, hp = bzr.emit(ctx, emitter(bzr), 0, n)
    assert np.array_equal(r.cpu().numpy().view(np.uint32), hr.view(np.uint32))
    assert np.array_equal(p.cpu().numpy().astype(np.uint32), hp)


def oracle_illuminate(orc, lenses, ris, em, n, tg):
    rays, _ = orc.emit(em, 0, n)
    out, status, seg = orc.trace_chain(lenses, ris, rays, threads=16)
    hist, exited, landed = orc.land(tg, out, status)
    return rays, status, seg, hist, exited, landed


@pytest.mark.parametrize("cfg_name,n,x", [("cfg2", 1 << 16, 0.0), ("cfg2", 1 << 16, -60.0), ("cfg4", 1 << 15, 0.0)])
def test_illuminate_matches_oracle(bzr, orc, ctx, cfg_name, n, x):
    """x = 0: the emitter inside the lens's bounding sphere (nothing culled, many rays land);
    x = -60: far behind it (most of the hemisphere culled)."""
    cfg = CONFIGS[cfg_name]
    lenses = [build_lens(bzr.TriMesh, lens).bezier_patches() for lens in cfg.lenses]
    ris = [lens.ri for lens in cfg.lenses]
    dms = [bzr.DeviceMesh(ctx, p) for p in lenses]
    hist, stats = bzr.illuminate(ctx, dms, ris, emitter(bzr, x=x), n, target(bzr))
    rays, status, seg, want_hist, exited, landed = oracle_illuminate(orc, lenses, ris, emitter(orc, x=x), n,
                                                                     target(orc))
    assert stats["emitted"] == n
    assert stats["exited"] == exited and stats["landed"] == landed
    assert np.array_equal(hist, want_hist)
    if x == 0.0:
        assert landed > 50
    else:
        assert stats["culled"] > n // 2 and exited > 0
    # every ray the sphere dropped is one the reference misses at its first BezierMesh::intersect
    c = bzr.bounding_sphere(dms[0]).astype(np.float64)
    o, d = rays[:3].astype(np.float64), rays[3:].astype(np.float64)
    oc = o - c[:3, None]
    cc = (oc * oc).sum(0) - c[3] ** 2
    b = (oc * d).sum(0)
    culled = (cc > 0) & ((b >= 0) | (b * b - cc < 0))
    assert culled.sum() == stats["culled"]
    assert (status[culled] == 0).all() and (seg[culled] == 1).all()


def test_illuminate_with_an_always_listed_patch(bzr, orc, ctx):
    """A lens with a rounding-dominated patch (no proven gate region: always listed): the sphere covers the
    proven boxes only, and a ray outside it is culled only if no always-listed gate passes -- the counts
    still equal the oracle's uncut chain, and the cull still drops most of an emitter far behind the lens."""
    from test_culling_conservative import dominated_lens

    lens = dominated_lens(bzr)
    dm = bzr.DeviceMesh(ctx, lens)
    sph = bzr.bounding_sphere(dm)
    assert np.isfinite(sph).all()
    n = 1 << 15
    for x in (0.0, -60.0):
        hist, stats = bzr.illuminate(ctx, [dm], [1.3], emitter(bzr, x=x), n, target(bzr))
        rays, status, seg, want_hist, exited, landed = oracle_illuminate(orc, [lens], [1.3], emitter(orc, x=x), n,
                                                                         target(orc))
        assert stats["exited"] == exited and stats["landed"] == landed
        assert np.array_equal(hist, want_hist)
        c = sph.astype(np.float64)
        oc = rays[:3].astype(np.float64) - c[:3, None]
        cc = (oc * oc).sum(0) - c[3] ** 2
        b = (oc * rays[3:].astype(np.float64)).sum(0)
        outside = (cc > 0) & ((b >= 0) | (b * b - cc < 0))
        assert stats["culled"] <= outside.sum()
        if x == -60.0:
            assert stats["culled"] > n // 2


@pytest.mark.slow
def test_illuminate_two_batches(bzr, orc, ctx):
    """More rays than one 1M-ray batch: the batches continue the global ray numbering."""
    cfg = CONFIGS["cfg2"]
    lens = build_lens(bzr.TriMesh, cfg.lenses[0]).bezier_patches()
    n = (1 << 20) + 3000
    em_b, em_o = emitter(bzr, seed=99, rays=256), emitter(orc, seed=99, rays=256)
    hist, stats = bzr.illuminate(ctx, [bzr.DeviceMesh(ctx, lens)], [1.3], em_b, n, target(bzr))
    _, _, _, want_hist, exited, landed = oracle_illuminate(orc, [lens], [1.3], em_o, n, target(orc))
    assert stats["emitted"] == n and stats["landed"] == landed and stats["exited"] == exited
    assert np.array_equal(hist, want_hist)
