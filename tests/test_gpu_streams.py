"""Stream ordering of device-buffer calls (include/bzr.h bzr_ctx_set_stream; bzr_amd._stream_for).

1. An unbound context given torch tensors launches on torch's current stream: inputs produced there by a
   slow torch op are ready, and torch ops on the outputs see the finished results without a sync.
2. Switching a context from stream A to stream B orders B's launches after A's queued work (the
   event hand-off): B reads what A wrote.
"""
import numpy as np
import pytest

from bzr_amd.configs import CONFIGS, build_lens, grid_rays

pytestmark = pytest.mark.gpu


def test_unbound_context_runs_on_torch_current_stream(bzr):
    torch = pytest.importorskip("torch")
    cfg = CONFIGS["cfg2"]
    lens = build_lens(bzr.TriMesh, cfg.lenses[0]).bezier_patches()
    ctx = bzr.Context(0)  # fresh: not bound to any stream
    assert not ctx.bound
    dm = bzr.DeviceMesh(ctx, lens)
    host = grid_rays(cfg, side=256)
    want = bzr.trace_chain(ctx, [dm], [1.3], host)
    src = torch.from_numpy(host).cuda()
    torch.cuda.synchronize()
    a = torch.randn(4096, 4096, device="cuda")
    big = a @ a @ a  # keeps torch's current stream busy for a while
    rays = torch.empty_like(src)
    rays.copy_(src + 0.0 * big[0, 0])  # the input only exists once `big` is done
    o, s, g = bzr.trace_chain(ctx, [dm], [1.3], rays)
    o2 = o.clone()  # torch op on the same stream: must see the finished output
    s2, g2 = s.clone(), g.clone()
    torch.cuda.synchronize()
    assert np.array_equal(o2.cpu().numpy().view(np.uint32), want[0].view(np.uint32))
    assert np.array_equal(s2.cpu().numpy().astype(np.uint32), want[1])
    assert np.array_equal(g2.cpu().numpy().astype(np.uint32), want[2])
    assert not ctx.bound


def test_stream_switch_orders_after_previous_stream(bzr):
    torch = pytest.importorskip("torch")
    cfg = CONFIGS["cfg2"]
    lens = build_lens(bzr.TriMesh, cfg.lenses[0]).bezier_patches()
    ctx = bzr.Context(0)
    dm = bzr.DeviceMesh(ctx, lens)
    host = grid_rays(cfg, side=1024)
    h1 = bzr.trace_chain(ctx, [dm], [1.3], host)[0]
    want = bzr.intersect(ctx, dm, h1)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    with torch.cuda.stream(sa):
        rays = torch.from_numpy(host).cuda()
        o1 = torch.empty_like(rays)
        st = torch.empty(rays.shape[1], dtype=torch.int32, device="cuda")
        sg = torch.empty_like(st)
        hits = torch.empty((13, rays.shape[1]), device="cuda")
    sa.synchronize()
    ctx.set_stream(sa.cuda_stream)
    for _ in range(3):  # a few frames of queued work on A
        bzr.trace_chain(ctx, [dm], [1.3], rays, o1, st, sg)
    ctx.set_stream(sb.cuda_stream)  # hand-off: B waits for A's queued frames
    bzr.intersect(ctx, dm, o1, hits)
    sb.synchronize()
    ctx.use_own_stream()
    assert np.array_equal(hits.cpu().numpy().view(np.uint32), want.view(np.uint32))


def test_frames_in_flight_on_two_contexts_match_one_stream(bzr):
    """bench.py's frames in flight: two contexts on one device share the lens meshes, each launching on
    its own stream into its own outputs, frames alternating -- every frame's bits equal a lone call's."""
    torch = pytest.importorskip("torch")
    cfg = CONFIGS["cfg4"]
    lenses = [build_lens(bzr.TriMesh, l).bezier_patches() for l in cfg.lenses]
    ris = [l.ri for l in cfg.lenses]
    c0, c1 = bzr.Context(0), bzr.Context(0)
    meshes = [bzr.DeviceMesh(c0, p) for p in lenses]  # device-scoped: usable from c1 too
    rays = torch.from_numpy(grid_rays(cfg, side=512)).cuda()
    n = rays.shape[1]
    want = bzr.trace_chain(c0, meshes, ris, rays.cpu().numpy())
    s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
    c0.use_torch_stream(s0)
    c1.use_torch_stream(s1)
    outs = [(torch.empty((6, n), device="cuda"), torch.empty(n, dtype=torch.int32, device="cuda"),
             torch.empty(n, dtype=torch.int32, device="cuda")) for _ in range(2)]
    for k in range(6):
        ctx, st = (c0, s0) if k % 2 == 0 else (c1, s1)
        with torch.cuda.stream(st):
            bzr.trace_chain(ctx, meshes, ris, rays, *outs[k % 2])
    torch.cuda.synchronize()
    for o, s, g in outs:
        assert np.array_equal(o.cpu().numpy().view(np.uint32), want[0].view(np.uint32))
        assert np.array_equal(s.cpu().numpy().astype(np.uint32), want[1])
        assert np.array_equal(g.cpu().numpy().astype(np.uint32), want[2])


def test_wave_clock_hook_times_every_wave(bzr):
    """bzr_debug_wave_clock (include/bzr_debug.h): one start / duration pair per 64-ray wave of a fused
    call, durations positive; turning it off leaves the buffer alone."""
    import ctypes

    torch = pytest.importorskip("torch")
    cfg = CONFIGS["cfg2"]
    lens = build_lens(bzr.TriMesh, cfg.lenses[0]).bezier_patches()
    ctx = bzr.Context(0)
    ctx.use_torch_stream()
    dm = bzr.DeviceMesh(ctx, lens)
    rays = torch.from_numpy(grid_rays(cfg, side=256)).cuda()
    waves = rays.shape[1] // 64
    clock = torch.zeros(2 * waves, dtype=torch.int64, device="cuda")
    L = bzr.lib()
    assert L.bzr_debug_wave_clock(ctx.handle, ctypes.c_void_p(clock.data_ptr()), waves) == 0
    bzr.trace_chain(ctx, [dm], [1.3], rays, mode=bzr.MODE_PARITY | bzr.PIPELINE_FUSED)
    torch.cuda.synchronize()
    assert L.bzr_debug_wave_clock(ctx.handle, None, 0) == 0
    c = clock.view(-1, 2).cpu().numpy()
    assert (c[:, 1] > 0).all() and (c[:, 0] > 0).all()
    clock.zero_()
    bzr.trace_chain(ctx, [dm], [1.3], rays, mode=bzr.MODE_PARITY | bzr.PIPELINE_FUSED)
    torch.cuda.synchronize()
    assert int(clock.abs().sum()) == 0
