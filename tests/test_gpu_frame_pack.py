"""bzr_pack_frame (csrc/device/frame_pack.hip) against the torch packers of bzr_amd/frame.py -- the
gather layouts the multi-GPU frame loop sends to rank 0.  Bit-identical in every column
the reader (frame.assemble / unpack_compact) looks at; integer/byte work, so exact."""
import numpy as np
import pytest
import torch

from bzr_amd import frame

pytestmark = pytest.mark.gpu


def frame_outputs(n, seed, p_survive=0.65):
    """Synthetic chain outputs: status 0..2, segments 0..4 (survivors: segments >= 2 or status != 0)."""
    g = np.random.default_rng(seed)
    seg = g.integers(0, 5, n).astype(np.int32)
    st = np.where(g.random(n) < p_survive, g.integers(1, 3, n), 0).astype(np.int32)
    st[seg == 0] = 0
    rays = g.standard_normal((6, n)).astype(np.float32)
    dev = torch.device("cuda", 0)
    return torch.from_numpy(rays).to(dev), torch.from_numpy(st).to(dev), torch.from_numpy(seg).to(dev)


@pytest.mark.parametrize("n,npad", [(4096, 4096), (5000, 8192), (1, 4096), (3 * 1024 * 1024 + 77, 3 * 1024 * 1024 + 4096)])
@pytest.mark.parametrize("layout", ["image", "rays"])
def test_pack_words_match_torch(bzr, ctx, n, npad, layout):
    rays, st, sg = frame_outputs(n, n)
    rows = frame.IMAGE_ROWS if layout == "image" else frame.PACKED_ROWS
    want = torch.zeros((rows, npad), dtype=torch.float32, device="cuda")
    got = torch.full((rows, npad), 7.0, dtype=torch.float32, device="cuda")
    frame.pack(rays if layout == "rays" else None, st, sg, want)
    bzr.pack_frame(ctx, layout, rays if layout == "rays" else None, st, sg, got, npad)
    torch.cuda.synchronize()
    assert torch.equal(got[:, :n].view(torch.int32), want[:, :n].view(torch.int32))
    assert bool((got[:, n:] == 7.0).all())  # the padding columns are not written


@pytest.mark.parametrize("n,npad,cap_delta", [(4096, 4096, 64), (5000, 8192, 0), (1, 4096, 1),
                                               (2 * 1024 * 1024 + 333, 2 * 1024 * 1024 + 4096, 100),
                                               (5000, 8192, -700)])
def test_pack_compact_matches_torch(bzr, ctx, n, npad, cap_delta):
    """Survivors in ray order at the same positions as frame.pack_compact's cumsum; the count word; the
    bytes.  cap_delta < 0: more survivors than the capacity -- both write the first cap, count says more."""
    rays, st, sg = frame_outputs(n, 17 + n)
    count = int(frame.survivors(st, sg).sum())
    cap = max(1, min(npad, count + cap_delta))
    size = frame.compact_size(npad, cap)
    want = torch.zeros(size, dtype=torch.float32, device="cuda")
    got = torch.zeros(size, dtype=torch.float32, device="cuda")
    frame.pack_compact(st, sg, rays, want, npad, cap)
    bzr.pack_frame(ctx, "compact", rays, st, sg, got, npad, cap)
    torch.cuda.synchronize()
    nw = frame.compact_words(npad)
    assert torch.equal(got[:nw].view(torch.uint8)[:n], want[:nw].view(torch.uint8)[:n])
    assert int(got[nw:nw + 1].view(torch.int32)) == count == int(want[nw:nw + 1].view(torch.int32))
    k = min(count, cap)
    g6, w6 = got[nw + 1:].view(6, cap + 1), want[nw + 1:].view(6, cap + 1)
    assert torch.equal(g6[:, :k].view(torch.int32), w6[:, :k].view(torch.int32))
    if count <= cap:  # the reader's round trip (unpack_compact checks count <= cap)
        prim = np.zeros((6, n), np.float32)
        r, s, g = frame.unpack_compact(got.cpu(), n, npad, cap, prim)
        alive = frame.survivors(st, sg).cpu().numpy()
        assert np.array_equal(r[:, alive], rays.cpu().numpy()[:, alive])
        assert np.array_equal(s, (st.cpu().numpy() & 3).astype(np.uint32))
        assert np.array_equal(g, sg.cpu().numpy().astype(np.uint32))


def test_pack_compact_empty_frame(bzr, ctx):
    """n = 0: only the count word (0) is written."""
    e = torch.empty(0, dtype=torch.int32, device="cuda")
    got = torch.full((frame.compact_size(4096, 8),), 3.0, dtype=torch.float32, device="cuda")
    bzr.pack_frame(ctx, "compact", torch.empty((6, 0), device="cuda"), e, e, got, 4096, 8)
    torch.cuda.synchronize()
    nw = frame.compact_words(4096)
    assert int(got[nw:nw + 1].view(torch.int32)) == 0
    assert bool((got[:nw] == 3.0).all()) and bool((got[nw + 1:] == 3.0).all())


def test_frame_loop_with_device_packer_on_a_traced_frame(bzr, ctx):
    """The bench's loop shape on the device: a real cfg2 chain frame (256^2) packed by bzr_pack_frame through
    FrameLoop(pack_fn=...) equals the torch packers' buffers, in all three layouts."""
    from bzr_amd.configs import CONFIGS, build_lens

    cfg = CONFIGS["cfg2"]
    side = 256
    meshes = [bzr.DeviceMesh(ctx, build_lens(bzr.TriMesh, l).bezier_patches()) for l in cfg.lenses]
    ris = [l.ri for l in cfg.lenses]
    _, _, rays_np = frame.rank_rays(cfg, 0, 1, side, side)
    n = rays_np.shape[1]
    rays = torch.from_numpy(rays_np).cuda()
    outs = [(torch.empty((6, n), device="cuda"), torch.empty(n, dtype=torch.int32, device="cuda"),
             torch.empty(n, dtype=torch.int32, device="cuda"))]

    def trace(f, k):
        bzr.trace_chain(ctx, meshes, ris, rays, *outs[f], mode=bzr.MODE_PARITY)

    trace(0, 0)
    torch.cuda.synchronize()
    npad = frame.padded_count(1, side, side)
    cap = frame.compact_capacity(int(frame.survivors(outs[0][1], outs[0][2]).sum()), npad)
    for layout in frame.LAYOUTS:
        loops = [frame.FrameLoop(1, 0, n, npad, layout, trace, outs, cap=cap, device="cuda", pack_always=True,
                                 pack_fn=pf)
                 for pf in (None, lambda out, p, f, lay=layout: bzr.pack_frame(ctx, lay, *out, p, npad, cap))]
        for lp in loops:
            lp.step(1)
            lp.drain()
        torch.cuda.synchronize()
        want, got = loops[0].packed[0], loops[1].packed[0]
        if layout == "compact":
            nw = frame.compact_words(npad)
            count = int(want[nw:nw + 1].view(torch.int32))
            assert count <= cap
            assert torch.equal(got[:nw + 1].view(torch.int32), want[:nw + 1].view(torch.int32))
            assert torch.equal(got[nw + 1:].view(6, cap + 1)[:, :count], want[nw + 1:].view(6, cap + 1)[:, :count])
        else:
            assert torch.equal(got[:, :n].view(torch.int32), want[:, :n].view(torch.int32))
