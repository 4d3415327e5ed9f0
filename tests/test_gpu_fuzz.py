"""Randomised lenses and rays: the culled GPU pipelines and the brute-force scan against the oracle, bit for bit.

Each seed builds a lens the reference's way (Mesh::makeEllipsoid or makeSolidOfRevolution with the test-lens
envelope, random sectors / belts / size, a random rotation and displacement, standardizeVertices /
standardizeNormals, BezierMesh) and fires rays at it: at random control points (edge and vertex regions, where
follow-side retries and ties live), at random points of its box, with axis-parallel direction components, and
from far beyond the culling radius (the in-order full scan).  Every output word of bzr_intersect and of a
one-lens refraction chain must equal the oracle's on both pipelines.  A shape the reference's preprocessing
refuses ("Vertex on edge detected.") is skipped, as the reference would refuse it.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEEDS = list(range(24))


def _rotation(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]], np.float32)


def _lens(bzr, seed):
    rng = np.random.default_rng(1000 + seed)
    m = bzr.TriMesh()
    sectors, belts = int(rng.integers(3, 41)), int(rng.integers(2, 25))
    # x size 1: makeEllipsoid applies aSize(0) twice (reference/mesh.cpp:456-460), so any other x leaves cracks the
    # reference's standardizeNormals refuses (tests/test_host_parity.py); the random transform stretches instead
    size = (1.0, float(rng.integers(1, 6)), float(rng.integers(1, 6)))
    if seed % 3 == 2:
        m.make_solid_of_revolution(sectors, belts, bzr.ENVELOPE_TESTLENS, size)
    else:
        m.make_ellipsoid(sectors, belts, size)
    m.transform(_rotation(rng) * np.float32(rng.uniform(0.5, 3.0)), rng.uniform(-20, 20, 3))
    try:
        m.standardize()
        patches = m.bezier_patches()
    except bzr.BzrError as e:
        if "Vertex on edge" in str(e):
            return None, None
        raise
    return patches, rng


def _rays(patches, rng, n=3000):
    cp = patches[:, 19:49].reshape(-1, 3).astype(np.float64)
    lo, hi = cp.min(0), cp.max(0)
    span = float(np.abs(hi - lo).max())
    k = n // 4
    tgt = np.concatenate([cp[rng.integers(0, len(cp), 2 * k)],                # control points: edges, vertices
                          rng.uniform(lo, hi, (n - 2 * k, 3))])               # anywhere in the box
    o = tgt + rng.normal(size=(n, 3)) * span * rng.uniform(0.2, 3.0, (n, 1))
    o[-k // 2:] = tgt[-k // 2:] + rng.normal(size=(k // 2, 3)) * span * 1e4  # beyond the culling radius
    d = tgt - o
    ax = rng.random(n) < 0.15
    d[ax, rng.integers(0, 3, ax.sum())] = 0.0                                  # axis-parallel components
    d /= np.maximum(np.linalg.norm(d, axis=1, keepdims=True), 1e-30)
    return np.concatenate([o.T, d.T]).astype(np.float32)


@pytest.mark.parametrize("seed", SEEDS)
def test_random_lens_against_oracle(bzr, orc, ctx, seed):
    patches, rng = _lens(bzr, seed)
    if patches is None:
        pytest.skip("the reference's preprocessing refuses this shape (Vertex on edge detected.)")
    rays = _rays(patches, rng)
    dm = bzr.DeviceMesh(ctx, patches)
    want = orc.intersect(patches, rays, threads=16)
    wu = want.view(np.uint32)
    assert (wu[11] == bzr.WHAT_INTERSECT).mean() > 0.05  # the rays do meet the lens
    for mode in (bzr.PIPELINE_FUSED, bzr.PIPELINE_STAGED, bzr.ACCEL_NONE):
        got = bzr.intersect(ctx, dm, rays, mode=mode)
        bad = (got.view(np.uint32) != wu).any(axis=0)
        assert not bad.any(), f"seed {seed} mode {mode}: {int(bad.sum())} of {rays.shape[1]} rays differ"
    ri = float(rng.uniform(1.1, 1.9))
    w_rays, w_st, w_seg = orc.trace_chain([patches], [ri], rays, threads=16)
    for mode in (bzr.PIPELINE_FUSED, bzr.PIPELINE_STAGED):
        g_rays, g_st, g_seg = bzr.trace_chain(ctx, [dm], [ri], rays, mode=mode)
        assert np.array_equal(g_st, w_st) and np.array_equal(g_seg, w_seg), f"seed {seed} mode {mode}: status"
        assert np.array_equal(g_rays.view(np.uint32), w_rays.view(np.uint32)), f"seed {seed} mode {mode}: rays"


@pytest.mark.parametrize("seed", list(range(8)))
def test_random_two_lens_chain_against_oracle(bzr, orc, ctx, seed):
    """Two random lenses, the second behind the first along a beam: the chain's lens-to-lens hand-over (refract
    inside / outside per lens, a NONE ends the ray) on both pipelines and the brute-force scan, against the
    oracle."""
    a, rng = _lens(bzr, 100 + seed)
    if a is None:
        pytest.skip("the reference's preprocessing refuses this shape")
    cpa = a[:, 19:49].reshape(-1, 3).astype(np.float64)
    ca, span = cpa.mean(0), float(np.abs(cpa.max(0) - cpa.min(0)).max())
    u = rng.normal(size=3)
    u /= np.linalg.norm(u)
    # the second lens: a random shape like the first, moved to 1.5 spans behind it along u
    rb = np.random.default_rng(5000 + seed)
    m = bzr.TriMesh()
    sectors, belts = int(rb.integers(3, 41)), int(rb.integers(2, 25))
    m.make_ellipsoid(sectors, belts, (1.0, float(rb.integers(1, 6)), float(rb.integers(1, 6))))
    m.transform(_rotation(rb) * np.float32(0.5 * span), ca + u * 1.5 * span)
    try:
        m.standardize()
        b = m.bezier_patches()
    except bzr.BzrError as e:
        if "Vertex on edge" in str(e):
            pytest.skip("the reference's preprocessing refuses the second shape")
        raise
    # a beam along u through lens a: origins 3 spans before its centre, spread over its width, small jitter
    n = 3000
    p = rng.normal(size=(n, 3))
    p -= np.outer(p @ u, u)
    o = ca - 3.0 * span * u + p * 0.4 * span
    d = u + rng.normal(size=(n, 3)) * 0.05
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([o.T, d.T]).astype(np.float32)
    ri = [float(rng.uniform(1.1, 1.9)), float(rng.uniform(1.1, 1.9))]
    w_rays, w_st, w_seg = orc.trace_chain([a, b], ri, rays, threads=16)
    assert (w_seg > 2).sum() > 10  # rays reach the second lens
    lenses = [bzr.DeviceMesh(ctx, a), bzr.DeviceMesh(ctx, b)]
    for mode in (bzr.PIPELINE_FUSED, bzr.PIPELINE_STAGED, bzr.ACCEL_NONE):
        g_rays, g_st, g_seg = bzr.trace_chain(ctx, lenses, ri, rays, mode=mode)
        assert np.array_equal(g_st, w_st) and np.array_equal(g_seg, w_seg), f"seed {seed} mode {mode}: status"
        assert np.array_equal(g_rays.view(np.uint32), w_rays.view(np.uint32)), f"seed {seed} mode {mode}: rays"
