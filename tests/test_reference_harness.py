"""The reference's own refraction harness, restated: testBezierRefraction("21x15", 21, 15, (1,4,2),
3, 3, 4, 4) (reference/test.cpp:330-427; its call is at reference/test.cpp:513).

The harness does the following:
- builds the test lens (makeSolidOfRevolution with the harness envelope, test.cpp:334-338);
- shoots 4x4 rays from the origin;
- repeats ten times: move the SAME mesh by +10 in x and re-standardize it in place
  (test.cpp:370-373; the translations accumulate in float), then refract every still-valid ray
  with expected cInside, then with expected cOutside (test.cpp:379-400).

SURVEY.md 8(c) records what running the reference harness printed: 22 "inside" and 22 "outside"
events.  That is the pin here: the oracle must reproduce it (CPU), and the product must reproduce
the oracle bit for bit, event by event (GPU).
"""
import math

import numpy as np
import pytest

SECTORS, BELTS, SIZE = 21, 15, (1.0, 4.0, 2.0)
DEG_V = DEG_W = 3.0
COUNT_V = COUNT_W = 4
EXPECTED_EVENTS = (22, 22)  # (inside, outside), SURVEY.md 8(c) probe of the reference harness
INSIDE, OUTSIDE = 1, 2


def harness_rays():
    """Rays of test.cpp:352-361: Ray({0,0,0}, {sqrt(1 - sinV^2 - sinW^2), sinV, sinW}); the Ray
    constructor normalizes (3dGeomUtil.h:176-178).  float32 throughout (cgPi is a float)."""
    f = np.float32
    pi = f(math.pi)
    cols = []
    for v in range(COUNT_V):
        for w in range(COUNT_W):
            sv = f(np.sin(f(f(f(v) * f(DEG_V) + f(1.0)) * pi) / f(180.0)))
            sw = f(np.sin(f(f(f(w) * f(DEG_W) + f(1.0)) * pi) / f(180.0)))
            d = np.array([np.sqrt(f(f(1.0) - sv * sv - sw * sw)), sv, sw], np.float32)
            z = f(d[0] * d[0] + f(d[1] * d[1] + d[2] * d[2]))
            d = d / np.sqrt(z) if z > 0 else d
            cols.append([0.0, 0.0, 0.0, d[0], d[1], d[2]])
    return np.array(cols, np.float32).T.copy()


def run_harness(mesh, refract):
    """Drive the harness loop; `mesh` is a mesh object with translate/standardize_* / bezier_patches,
    `refract(patches, rays [6, k], expected) -> (rays', status)`.  Returns the event log
    [(lens, pass, ray, status, ray')] and the (inside, outside) counts."""
    rays = harness_rays()
    valid = np.ones(rays.shape[1], bool)
    log, inside, outside = [], 0, 0
    for lens in range(10):
        if not valid.any():
            break
        mesh.translate((10.0, 0.0, 0.0))
        mesh.standardize_vertices()
        mesh.standardize_normals()
        patches = mesh.bezier_patches()
        for j in range(2):
            idx = np.nonzero(valid)[0]
            out, st = refract(patches, rays[:, idx], np.full(len(idx), INSIDE if j == 0 else OUTSIDE, np.uint32))
            for k, r in enumerate(idx):
                log.append((lens, j, int(r), int(st[k]), out[:, k].copy()))
                if st[k] != 0:
                    rays[:, r] = out[:, k]
                    inside += st[k] == INSIDE
                    outside += st[k] == OUTSIDE
                else:
                    valid[r] = False
    return log, (inside, outside)


def test_oracle_reproduces_reference_harness(orc):
    mesh = orc.OMesh().make_solid_of_revolution(SECTORS, BELTS, 1, SIZE)
    _, counts = run_harness(mesh, lambda p, r, e: orc.refract(p, 1.3, r, e))
    assert counts == EXPECTED_EVENTS


@pytest.mark.gpu
def test_product_matches_oracle_on_reference_harness(bzr, orc, ctx):
    omesh = orc.OMesh().make_solid_of_revolution(SECTORS, BELTS, 1, SIZE)
    olog, ocounts = run_harness(omesh, lambda p, r, e: orc.refract(p, 1.3, r, e))

    def gpu_refract(patches, rays, expected):
        mesh = bzr.DeviceMesh(ctx, patches)
        return bzr.refract(ctx, mesh, 1.3, rays, expected)

    pmesh = bzr.TriMesh().make_solid_of_revolution(SECTORS, BELTS, bzr.ENVELOPE_TESTLENS, SIZE)
    plog, pcounts = run_harness(pmesh, gpu_refract)
    assert pcounts == ocounts == EXPECTED_EVENTS
    assert len(plog) == len(olog)
    for (l1, j1, r1, s1, o1), (l2, j2, r2, s2, o2) in zip(plog, olog):
        assert (l1, j1, r1, s1) == (l2, j2, r2, s2)
        if s1:
            assert np.array_equal(o1.view(np.uint32), o2.view(np.uint32)), (l1, j1, r1)
