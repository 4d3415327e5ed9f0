"""bzr_trace_tiled: the refraction chain dealt over several contexts from one process.

The GPU box has one device, so the multi-device path runs with two and three contexts on device 0
(separate streams, separate host threads): the tile dealing, packing and scatter-back are the same
code as across 8 devices.  The bar is bit-identity with one bzr_trace_chain over all rays, which
tests/test_gpu_parity.py pins to the oracle.
"""
import numpy as np
import pytest

from bzr_amd.configs import CONFIGS, build_lens, grid_rays

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nctx,tile", [(1, 4096), (2, 4096), (3, 1000)])
def test_tiled_equals_single_chain(bzr, ctx, nctx, tile):
    cfg = CONFIGS["cfg4"]  # two stacked lenses
    patches = [build_lens(bzr.TriMesh, lens).bezier_patches() for lens in cfg.lenses]
    ri = [lens.ri for lens in cfg.lenses]
    rays = grid_rays(cfg, side=256)  # tile-major order: 16 tiles of 64x64
    want = bzr.trace_chain(ctx, [bzr.DeviceMesh(ctx, p) for p in patches], ri, rays)
    ctxs = [bzr.Context(0) for _ in range(nctx)]
    lenses = [[bzr.DeviceMesh(c, p) for p in patches] for c in ctxs]
    got = bzr.trace_tiled(ctxs, lenses, ri, rays, tile_rays=tile)
    for g, w in zip(got, want):
        assert np.array_equal(np.asarray(g).view(np.uint32), np.asarray(w).view(np.uint32))
    assert int(got[2].sum()) > rays.shape[1]  # refracted segments were traced


def test_tiled_fast_mode_passes_through(bzr, ctx):
    cfg = CONFIGS["cfg2"]
    patches = build_lens(bzr.TriMesh, cfg.lenses[0]).bezier_patches()
    rays = grid_rays(cfg, side=128)
    want = bzr.trace_chain(ctx, [bzr.DeviceMesh(ctx, patches)], [1.3], rays, mode=bzr.MODE_FAST)
    ctxs = [bzr.Context(0) for _ in range(2)]
    got = bzr.trace_tiled(ctxs, [[bzr.DeviceMesh(c, patches)] for c in ctxs], [1.3], rays, mode=bzr.MODE_FAST)
    for g, w in zip(got, want):
        assert np.array_equal(np.asarray(g).view(np.uint32), np.asarray(w).view(np.uint32))
