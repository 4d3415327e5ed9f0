"""bzr_trace_tiled: the refraction chain dealt over several contexts from one process.

The GPU box has one device, so the multi-device path runs with two and three contexts on device 0
(separate streams): the tile dealing, per-device packing, device-side gather (peer copies; RCCL with a
one-device communicator) and the unpack on device 0 are the same code as across 8 devices.  The bar is
bit-identity with one bzr_trace_chain over all rays, which tests/test_gpu_parity.py pins to the oracle.
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


def _cfg4(bzr):
    cfg = CONFIGS["cfg4"]
    patches = [build_lens(bzr.TriMesh, lens).bezier_patches() for lens in cfg.lenses]
    return cfg, patches, [lens.ri for lens in cfg.lenses]


def _same(got, want):
    for g, w in zip(got, want):
        g = g.cpu().numpy() if hasattr(g, "cpu") else np.asarray(g)
        w = w.cpu().numpy() if hasattr(w, "cpu") else np.asarray(w)
        assert np.array_equal(g.view(np.uint32), w.view(np.uint32))


def test_tiled_device_pointers_equal_single_chain(bzr, ctx):
    """bzr_trace_tiled with BZR_DEVICE_PTRS: rays and outputs on device 0, the gather on the device."""
    import torch

    cfg, patches, ri = _cfg4(bzr)
    rays = grid_rays(cfg, side=256)
    want = bzr.trace_chain(ctx, [bzr.DeviceMesh(ctx, p) for p in patches], ri, rays)
    ctxs = [bzr.Context(0) for _ in range(3)]
    got = bzr.trace_tiled(ctxs, [[bzr.DeviceMesh(c, p) for p in patches] for c in ctxs], ri,
                          torch.from_numpy(rays).cuda(), tile_rays=4096)
    assert got[0].is_cuda
    _same(got, want)


@pytest.mark.parametrize("transport,ndev", [("peer", 1), ("peer", 2), ("peer", 3), ("rccl", 1), ("auto", 1),
                                           ("direct", 1), ("auto", 2)])
def test_tiled_plan_frames_in_flight(bzr, ctx, transport, ndev):
    """A bzr_tiled plan over `ndev` list devices (all device 0 on this box: the peer path; the RCCL path is
    the world-size-1 communicator with its self send/recv; the one-device DIRECT path traces into the
    outputs), 2 slots, 5 frames queued back to back with a different refractive index per frame: each
    frame's device-0 outputs equal one bzr_trace_chain with that index, so a slot buffer reused before its
    gather completed would fail."""
    import torch

    cfg, patches, _ = _cfg4(bzr)
    rays = grid_rays(cfg, side=256)
    n = rays.shape[1]
    tp = {"peer": bzr.GATHER_PEER, "rccl": bzr.GATHER_RCCL, "auto": bzr.GATHER_AUTO, "direct": bzr.GATHER_DIRECT}[transport]
    slots = [[bzr.Context(0) for _ in range(ndev)] for _ in range(2)]
    lenses = [[bzr.DeviceMesh(c, p) for p in patches] for c in slots[0]]  # device d's copy (same device here)
    plan = bzr.TiledPlan(slots, n, tile_rays=4096, transport=tp)
    got_tp, share, npad = plan.info()
    # AUTO: DIRECT for one device; two list entries on one device are not distinct devices -> peer copies
    assert got_tp == {"rccl": bzr.GATHER_RCCL, "peer": bzr.GATHER_PEER, "direct": bzr.GATHER_DIRECT,
                      "auto": bzr.GATHER_DIRECT if ndev == 1 else bzr.GATHER_PEER}[transport]
    assert int(share.sum()) == n and npad == -(-16 // ndev) * 4096
    plan.set_rays(torch.from_numpy(rays).cuda())
    ris = [1.3, 1.45, 1.2, 1.6, 1.3]
    outs = [(torch.empty((6, n), device="cuda"), torch.empty(n, dtype=torch.int32, device="cuda"),
             torch.empty(n, dtype=torch.int32, device="cuda")) for _ in ris]
    for r, o in zip(ris, outs):
        plan.trace(lenses, [r, r], *o)
    plan.sync()
    single = [bzr.DeviceMesh(ctx, p) for p in patches]
    for r, o in zip(ris, outs):
        _same(o, bzr.trace_chain(ctx, single, [r, r], rays))
    plan.close()


class _DevArray:
    """A raw device pointer as a torch-viewable array (__cuda_array_interface__, no copy)."""

    def __init__(self, ptr, shape):
        self.__cuda_array_interface__ = {"shape": shape, "typestr": "<f4", "data": (ptr, False), "version": 2,
                                         "strides": None}


def test_tiled_plan_share_rays_and_host_outputs(bzr, ctx):
    """Rays written straight into each device's share (bzr_tiled_share_rays), host-pointer outputs, a
    ragged last tile (n not a multiple of tile_rays)."""
    import ctypes

    import torch

    cfg, patches, ri = _cfg4(bzr)
    rays = grid_rays(cfg, side=256)[:, :60000].copy()
    n, tile = rays.shape[1], 1000
    slots = [[bzr.Context(0) for _ in range(3)]]
    plan = bzr.TiledPlan(slots, n, tile_rays=tile, transport=bzr.GATHER_PEER)
    _, share, npad = plan.info()
    assert npad == 20 * tile
    for d in range(3):
        cols = np.concatenate([np.arange(k * tile, min(n, (k + 1) * tile)) for k in range(d, -(-n // tile), 3)])
        assert len(cols) == share[d]
        p = ctypes.c_void_p()
        bzr._check(bzr.lib().bzr_tiled_share_rays(plan.handle, d, ctypes.byref(p)))
        view = torch.as_tensor(_DevArray(p.value, (6, int(share[d]))), device="cuda")
        view.copy_(torch.from_numpy(np.ascontiguousarray(rays[:, cols])).cuda())
    torch.cuda.synchronize()
    out = (np.empty((6, n), np.float32), np.empty(n, np.uint32), np.empty(n, np.uint32))
    lenses = [[bzr.DeviceMesh(c, p) for p in patches] for c in slots[0]]
    plan.trace(lenses, ri, *out)
    _same(out, bzr.trace_chain(ctx, [bzr.DeviceMesh(ctx, p) for p in patches], ri, rays))


@pytest.mark.parametrize("transport,ndev", [("peer", 3), ("rccl", 1), ("direct", 1)])
def test_tiled_plan_compact_gather(bzr, ctx, transport, ndev):
    """The compact layout (bzr_tiled_calibrate: one counted frame, then survivors only up to a capacity):
    frames bit-identical to one bzr_trace_chain, the rays that never refracted returned from device 0's copy
    of the frame; a capacity below the survivors is reported by bzr_tiled_sync (BZR_ERR_CAPACITY)."""
    import torch

    cfg, patches, ri = _cfg4(bzr)
    rays = grid_rays(cfg, side=256)
    n = rays.shape[1]
    tp = {"peer": bzr.GATHER_PEER, "rccl": bzr.GATHER_RCCL, "direct": bzr.GATHER_DIRECT}[transport]
    slots = [[bzr.Context(0) for _ in range(ndev)] for _ in range(2)]
    lenses = [[bzr.DeviceMesh(c, p) for p in patches] for c in slots[0]]
    plan = bzr.TiledPlan(slots, n, tile_rays=4096, transport=tp)
    plan.set_rays(torch.from_numpy(rays).cuda())
    want = bzr.trace_chain(ctx, [bzr.DeviceMesh(ctx, p) for p in patches], ri, rays)
    survivors = int(((want[2] >= 2) | (want[1] != 0)).sum())
    cap = plan.calibrate(lenses, ri)
    _, share, npad = plan.info()
    assert 0 < cap <= npad and cap * ndev >= survivors
    outs = [(torch.empty((6, n), device="cuda"), torch.empty(n, dtype=torch.int32, device="cuda"),
             torch.empty(n, dtype=torch.int32, device="cuda")) for _ in range(4)]
    for o in outs:
        plan.trace(lenses, ri, *o)
    plan.sync()
    for o in outs:
        _same(o, want)
    # host outputs through the same layout
    ho = (np.empty((6, n), np.float32), np.empty(n, np.uint32), np.empty(n, np.uint32))
    plan.trace(lenses, ri, *ho)
    _same(ho, want)
    if transport == "direct":  # nothing is gathered: the capacity cannot be exceeded
        plan.set_layout("compact", cap=64)
        plan.trace(lenses, ri, *ho)
        _same(ho, want)
        plan.close()
        return
    # too small a capacity: the frame is incomplete and sync says so
    plan.set_layout("compact", cap=64)
    plan.trace(lenses, ri, *outs[0])
    with pytest.raises(bzr.BzrError, match="capacity"):
        plan.sync()
    plan.sync()  # the flag was reported once
    # ... and a synchronous host-output frame says so itself
    with pytest.raises(bzr.BzrError, match="capacity"):
        plan.trace(lenses, ri, *ho)
    plan.sync()  # reported by the trace, not again here
    plan.close()


def test_tiled_plan_compact_needs_the_frame_rays(bzr, ctx):
    """Rays written into the shares directly leave device 0 without the frame: compact frames are refused."""
    import ctypes

    cfg, patches, ri = _cfg4(bzr)
    slots = [[bzr.Context(0) for _ in range(2)]]
    plan = bzr.TiledPlan(slots, 8192, tile_rays=4096, transport=bzr.GATHER_PEER)
    p = ctypes.c_void_p()
    bzr._check(bzr.lib().bzr_tiled_share_rays(plan.handle, 0, ctypes.byref(p)))
    plan.set_layout("compact", cap=4096)
    lenses = [[bzr.DeviceMesh(c, q) for q in patches] for c in slots[0]]
    out = (np.empty((6, 8192), np.float32), np.empty(8192, np.uint32), np.empty(8192, np.uint32))
    with pytest.raises(bzr.BzrError, match="set_rays"):
        plan.trace(lenses, ri, *out)


def test_tiled_plan_set_rays_waits_for_frames_in_flight(bzr, ctx):
    """bzr_tiled_set_rays while frames are queued: the queued frames still see the old rays,
    the frames after it the new ones -- on the DIRECT and the peer path."""
    import torch

    cfg, patches, ri = _cfg4(bzr)
    rays_a = grid_rays(cfg, side=256)
    rays_b = rays_a.copy()
    rays_b[2] += np.float32(0.37)  # shifted image: different hits
    n = rays_a.shape[1]
    single = [bzr.DeviceMesh(ctx, p) for p in patches]
    want_a, want_b = bzr.trace_chain(ctx, single, ri, rays_a), bzr.trace_chain(ctx, single, ri, rays_b)
    for tp, ndev in ((bzr.GATHER_DIRECT, 1), (bzr.GATHER_PEER, 2)):
        slots = [[bzr.Context(0) for _ in range(ndev)] for _ in range(3)]
        lenses = [[bzr.DeviceMesh(c, p) for p in patches] for c in slots[0]]
        plan = bzr.TiledPlan(slots, n, tile_rays=4096, transport=tp)
        outs = [(torch.empty((6, n), device="cuda"), torch.empty(n, dtype=torch.int32, device="cuda"),
                 torch.empty(n, dtype=torch.int32, device="cuda")) for _ in range(6)]
        plan.set_rays(torch.from_numpy(rays_a).cuda())
        for o in outs[:3]:
            plan.trace(lenses, ri, *o)
        plan.set_rays(rays_b)  # host rays this time
        for o in outs[3:]:
            plan.trace(lenses, ri, *o)
        plan.sync()
        for o in outs[:3]:
            _same(o, want_a)
        for o in outs[3:]:
            _same(o, want_b)
        plan.close()


def test_tiled_plan_distinct_devices(bzr, ctx):
    """Two distinct HIP devices (the peer path's events live on the device of the stream that
    records them): the peer and RCCL transports, bit-identical to one bzr_trace_chain.  Needs two GPUs."""
    import torch

    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs (the GPU box has one)")
    cfg, patches, ri = _cfg4(bzr)
    rays = grid_rays(cfg, side=256)
    n = rays.shape[1]
    want = bzr.trace_chain(ctx, [bzr.DeviceMesh(ctx, p) for p in patches], ri, rays)
    for tp in (bzr.GATHER_PEER, bzr.GATHER_RCCL):
        slots = [[bzr.Context(0), bzr.Context(1)] for _ in range(2)]
        lenses = [[bzr.DeviceMesh(c, p) for p in patches] for c in slots[0]]
        plan = bzr.TiledPlan(slots, n, tile_rays=4096, transport=tp)
        plan.set_rays(torch.from_numpy(rays).cuda())
        outs = [(torch.empty((6, n), device="cuda:0"), torch.empty(n, dtype=torch.int32, device="cuda:0"),
                 torch.empty(n, dtype=torch.int32, device="cuda:0")) for _ in range(3)]
        for o in outs:
            plan.trace(lenses, ri, *o)
        plan.sync()
        for o in outs:
            _same(o, want)
        plan.close()
