"""The fused culled path (k_trace; the default for dense batches) vs the staged culled path (BZR_PIPELINE_STAGED), the
brute-force scan (BZR_ACCEL_NONE) and the CPU oracle, bit for bit.

k_trace walks the BVH and runs the Newton stage inside the wave; the staged path
materialises (ray, patch) pairs and runs the Newton stage bucketed by patch.  Both keep the
lexicographic (t, scanned patch index) minimum, the reference's strict-< in-order winner
(reference/bezierMesh.cpp:206-227), so every output word must agree.
"""
import numpy as np
import pytest

from bzr_amd.configs import CONFIGS, build_lens, grid_rays

pytestmark = pytest.mark.gpu


def u32(a):
    return np.asarray(a).view(np.uint32)


@pytest.fixture(scope="module")
def cfg2_lens(bzr):
    return build_lens(bzr.TriMesh, CONFIGS["cfg2"].lenses[0]).bezier_patches()


def test_chain_fused_equals_staged_scan_and_oracle(bzr, orc, ctx, cfg2_lens):
    rays = grid_rays(CONFIGS["cfg2"], side=256)
    dm = bzr.DeviceMesh(ctx, cfg2_lens)
    fo, fs, fg = bzr.trace_chain(ctx, [dm], [1.3], rays, mode=bzr.PIPELINE_FUSED)
    so, ss, sg = bzr.trace_chain(ctx, [dm], [1.3], rays, mode=bzr.PIPELINE_STAGED)
    bo, bs, bg = bzr.trace_chain(ctx, [dm], [1.3], rays, mode=bzr.ACCEL_NONE)
    wo, ws, wg = orc.trace_chain([cfg2_lens], [1.3], rays)
    for o, s, g, label in ((fo, fs, fg, "fused"), (so, ss, sg, "staged"), (bo, bs, bg, "scan")):
        assert np.array_equal(u32(s), u32(ws)), label
        assert np.array_equal(u32(g), u32(wg)), label
        assert np.array_equal(u32(o), u32(wo)), label


def test_two_lens_chain_fused_equals_oracle(bzr, orc, ctx):
    cfg = CONFIGS["cfg4"]
    lenses = [build_lens(bzr.TriMesh, l).bezier_patches() for l in cfg.lenses]
    rays = grid_rays(cfg, side=128)
    dms = [bzr.DeviceMesh(ctx, p) for p in lenses]
    fo, fs, fg = bzr.trace_chain(ctx, dms, [1.3, 1.3], rays, mode=bzr.PIPELINE_FUSED)
    wo, ws, wg = orc.trace_chain(lenses, [1.3, 1.3], rays)
    assert np.array_equal(u32(fs), u32(ws)) and np.array_equal(u32(fg), u32(wg))
    assert np.array_equal(u32(fo), u32(wo))
    assert int(fg.sum()) > 2.5 * rays.shape[1]  # 2.97 segments per primary


def test_intersect_and_refract_fused_equal_staged(bzr, ctx, cfg2_lens):
    rays = grid_rays(CONFIGS["cfg2"], side=192)
    dm = bzr.DeviceMesh(ctx, cfg2_lens)
    assert np.array_equal(u32(bzr.intersect(ctx, dm, rays, mode=bzr.PIPELINE_FUSED)), u32(bzr.intersect(ctx, dm, rays, mode=bzr.PIPELINE_STAGED)))
    rng = np.random.default_rng(7)
    exp = rng.integers(1, 3, rays.shape[1]).astype(np.uint32)
    fo, fs = bzr.refract(ctx, dm, 1.3, rays, exp, mode=bzr.PIPELINE_FUSED)
    so, ss = bzr.refract(ctx, dm, 1.3, rays, exp, mode=bzr.PIPELINE_STAGED)
    assert np.array_equal(u32(fs), u32(ss)) and np.array_equal(u32(fo), u32(so))
    assert (fs != 0).any()


def test_fast_mode_fused_agrees_with_staged(bzr, ctx, cfg2_lens):
    """FAST (not bit-exact by design) in the two pipelines: both see the reference's candidates (exact
    gate); their fast:: Newton code is compiled separately, so FMA contraction may differ.  They must
    agree within SURVEY 8c's fast-mode gates: status >= 99.5 %, segment counts >= 99 %."""
    rays = grid_rays(CONFIGS["cfg2"], side=192)
    dm = bzr.DeviceMesh(ctx, cfg2_lens)
    fo, fs, fg = bzr.trace_chain(ctx, [dm], [1.3], rays, mode=bzr.MODE_FAST | bzr.PIPELINE_FUSED)
    so, ss, sg = bzr.trace_chain(ctx, [dm], [1.3], rays, mode=bzr.MODE_FAST | bzr.PIPELINE_STAGED)
    assert (fs == ss).mean() >= 0.995 and (fg == sg).mean() >= 0.99


def test_far_origins_take_the_inline_full_scan(bzr, orc, ctx):
    """Origins beyond the tree's validity radius (s_max) run the reference's in-order scan inside k_trace:
    mixed with near rays in the same waves, on robot.stl (450 patches)."""
    lens = build_lens(bzr.TriMesh, CONFIGS["cfg3"].lenses[0].__class__("stl", split=1)).bezier_patches()
    rng = np.random.default_rng(11)
    n = 4096
    o = rng.uniform(-30, 30, (3, n)).astype(np.float32)
    far = rng.random(n) < 0.25
    o[0, far] = np.float32(-5e4)  # far beyond s_max = max(1e3, 100 x span)
    tgt = rng.uniform(-20, 20, (3, n)).astype(np.float32)
    d = tgt - o
    d /= np.sqrt((d * d).sum(axis=0, keepdims=True)).astype(np.float32)
    rays = np.concatenate([o, d.astype(np.float32)]).astype(np.float32)
    dm = bzr.DeviceMesh(ctx, lens)
    ctx.counters(True)
    ctx.counters_report()
    got = bzr.intersect(ctx, dm, rays, mode=bzr.PIPELINE_FUSED)
    cnt = ctx.counters_report()
    ctx.counters(False)
    want = orc.intersect(lens, rays)
    assert np.array_equal(u32(got), u32(want))
    assert cnt["overflow_rays"] == int(far.sum())
    assert (u32(got)[11][far] == 4).any()  # some far rays hit


def test_fused_counters_match_oracle_work(bzr, orc, ctx, cfg2_lens):
    rays = grid_rays(CONFIGS["cfg2"], side=256)
    dm = bzr.DeviceMesh(ctx, cfg2_lens)
    ctx.counters(True)
    ctx.counters_report()
    _, _, seg = bzr.trace_chain(ctx, [dm], [1.3], rays, mode=bzr.PIPELINE_FUSED)
    got = ctx.counters_report()
    ctx.counters(False)
    orc.counters_reset()
    _, _, oseg = orc.trace_chain([cfg2_lens], [1.3], rays)
    want = orc.counters()
    assert got["segments"] == want["segments"] == int(oseg.sum())
    assert got["overflow_rays"] == 0
    assert got["pairs"] == want["newton"]          # every gate pass ran Newton once
    assert got["follows"] == want["follow"]
    assert got["gate_tests"] >= got["pairs"]
    assert got["node_visits"] > 0 and got["leaf_fetches"] > 0
    # a wave runs a patch's Newton pass at most once per segment: rounds <= pairs + follows
    assert got["newton_rounds"] <= got["pairs"] + got["follows"]


def test_empty_and_ragged_batches(bzr, orc, ctx, cfg2_lens):
    dm = bzr.DeviceMesh(ctx, cfg2_lens)
    empty = np.zeros((6, 0), np.float32)
    o, s, g = bzr.trace_chain(ctx, [dm], [1.3], empty, mode=bzr.PIPELINE_FUSED)
    assert o.shape == (6, 0) and s.shape == (0,)
    rays = grid_rays(CONFIGS["cfg2"], side=64)[:, :1000]  # not a multiple of 64 or 256
    fo, fs, fg = bzr.trace_chain(ctx, [dm], [1.3], np.ascontiguousarray(rays), mode=bzr.PIPELINE_FUSED)
    wo, ws, wg = orc.trace_chain([cfg2_lens], [1.3], rays)
    assert np.array_equal(u32(fo), u32(wo)) and np.array_equal(u32(fs), u32(ws)) and np.array_equal(u32(fg), u32(wg))


@pytest.mark.parametrize("name,side", [("cfg3", 2048), ("cfg4", 4096), ("cfg5", 4096)])
def test_full_size_fused_equals_staged(bzr, name, side):
    """The two culled pipelines are independent implementations of the same selection (k_trace's in-wave
    collected passes vs the staged pair buckets); at the configs' full sizes every output
    word of every ray agrees (cfg5: 4096^2 of its 8192^2 grid, the bench's one-GPU size of round 1)."""
    torch = pytest.importorskip("torch")
    cfg = CONFIGS[name]
    patches = [build_lens(bzr.TriMesh, l).bezier_patches() for l in cfg.lenses]
    ctx = bzr.Context(0)
    ctx.use_torch_stream()
    dms = [bzr.DeviceMesh(ctx, p) for p in patches]
    rays = torch.from_numpy(grid_rays(cfg, side=side)).cuda()
    if cfg.op == "chain":
        f = bzr.trace_chain(ctx, dms, [l.ri for l in cfg.lenses], rays, mode=bzr.PIPELINE_FUSED)
        s = bzr.trace_chain(ctx, dms, [l.ri for l in cfg.lenses], rays, mode=bzr.PIPELINE_STAGED)
        torch.cuda.synchronize()
        for a, b in zip(f, s):
            assert torch.equal(a.view(torch.int32), b.view(torch.int32))
        assert int(f[2].sum()) > 2.5 * rays.shape[1]
    else:
        f = bzr.intersect(ctx, dms[0], rays, mode=bzr.PIPELINE_FUSED)
        s = bzr.intersect(ctx, dms[0], rays, mode=bzr.PIPELINE_STAGED)
        torch.cuda.synchronize()
        assert torch.equal(f.view(torch.int32), s.view(torch.int32))
        assert int((f[11].view(torch.int32) == 4).sum()) > rays.shape[1] // 10  # hits (what == intersect)


def test_cost_ordered_dispatch_keeps_the_bits(bzr, cfg2_lens):
    """k_trace's cost-ordered dispatch: a context's repeated fused calls of one size run
    their tiles longest-first from the previous calls' wave durations (the order is built on the first call of
    a size and rebuilt every 16 calls).  Calls 1..40 of one size, with calls of another size and an intersect
    call interleaved (size switches drop the order), must all equal the brute-force scan bit for bit."""
    import torch

    ctx = bzr.Context(0)  # a fresh context: no order yet
    dm = bzr.DeviceMesh(ctx, cfg2_lens)
    rays = torch.from_numpy(grid_rays(CONFIGS["cfg2"], side=512)).cuda()      # 4096 tiles (> 2048: ordered)
    other = torch.from_numpy(grid_rays(CONFIGS["cfg2"], side=384)).cuda()     # 2304 tiles
    want = [t.cpu().numpy() for t in bzr.trace_chain(ctx, [dm], [1.3], rays, mode=bzr.ACCEL_NONE)]
    want_o = [t.cpu().numpy() for t in bzr.trace_chain(ctx, [dm], [1.3], other, mode=bzr.ACCEL_NONE)]
    want_h = bzr.intersect(ctx, dm, rays, mode=bzr.ACCEL_NONE).cpu().numpy()
    for k in range(40):
        got = bzr.trace_chain(ctx, [dm], [1.3], rays, mode=bzr.PIPELINE_FUSED)
        for g, w in zip(got, want):
            assert np.array_equal(u32(g.cpu().numpy()), u32(w)), k
        if k in (5, 22):
            got = bzr.trace_chain(ctx, [dm], [1.3], other, mode=bzr.PIPELINE_FUSED)
            for g, w in zip(got, want_o):
                assert np.array_equal(u32(g.cpu().numpy()), u32(w)), ("other size", k)
        if k == 30:
            h = bzr.intersect(ctx, dm, rays, mode=bzr.PIPELINE_FUSED).cpu().numpy()
            assert np.array_equal(u32(h), u32(want_h))
