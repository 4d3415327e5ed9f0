"""Work counters of the culled path vs the oracle's brute-force scan (cfg2 chain, 256^2 primaries).

Culling is exact, so the GPU sees the same candidate set as the reference's in-order scan: the
Newton runs (pairs that passed the planar gate) and follow-side retries must equal the oracle's
counts, rays on the overflow list excepted (the full scan resolves those; their pairs are not
counted on the GPU).  These counters are also what bench.py prices the Newton kernels with.
"""
import numpy as np
import pytest

from bzr_amd.configs import CONFIGS, build_lens, grid_rays


@pytest.mark.gpu
def test_counters_match_oracle_work(bzr, orc, ctx):
    cfg = CONFIGS["cfg2"]
    patches = build_lens(bzr.TriMesh, cfg.lenses[0]).bezier_patches()
    rays = grid_rays(cfg, side=256)
    mesh = bzr.DeviceMesh(ctx, patches)
    ctx.counters(True)
    ctx.counters_report()
    _, _, seg = bzr.trace_chain(ctx, [mesh], [1.3], rays)
    got = ctx.counters_report()
    ctx.counters(False)

    orc.counters_reset()
    _, _, oseg = orc.trace_chain([patches], [1.3], rays)
    want = orc.counters()

    assert np.array_equal(seg, oseg)
    assert got["segments"] == want["segments"] == int(oseg.sum())
    if got["overflow_rays"] == 0:
        assert got["pairs"] == want["newton"]
        assert got["follows"] == want["follow"]
    else:
        assert got["pairs"] <= want["newton"] and got["follows"] <= want["follow"]
    assert got["overflow_rays"] <= 0.001 * got["segments"]
