"""Multi-rank path on CPU (gloo, world_size 2 and 3): shard the image, trace each rank's tiles, gather to
rank 0 and assemble -- the result must equal tracing the whole image in one process.  The per-rank
tracer here is the oracle (CPU); on GPUs bench.py runs the same frame logic with libbzr over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from bzr_amd import frame
from bzr_amd.configs import CONFIGS


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, world, port, width, height, patches, result_path, layout="rays"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import pyoracle

        cfg = CONFIGS["cfg2"]
        rows, cols, rays = frame.rank_rays(cfg, rank, world, width, height)
        o, s, g = pyoracle.trace_chain([patches], [1.3], rays, threads=2)
        rows_packed = frame.PACKED_ROWS if layout == "rays" else frame.IMAGE_ROWS
        packed = torch.zeros((rows_packed, frame.padded_count(world, width, height)), dtype=torch.float32)
        frame.pack(torch.from_numpy(o), torch.from_numpy(s.view(np.int32)), torch.from_numpy(g.view(np.int32)), packed)
        glist = [torch.empty_like(packed) for _ in range(world)] if rank == 0 else None
        parts = frame.gather(packed, world, rank, gather_list=glist)
        if rank == 0:
            r, st, sg = frame.assemble(parts, cfg, world, width, height)
            if r is None:
                np.savez(result_path, status=st, seg=sg)
            else:
                np.savez(result_path, rays=r, status=st, seg=sg)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,scaling", [(2, "weak"), (3, "weak"), (2, "strong"), (3, "strong")])
def test_sharded_frame_equals_single_process(bzr, orc, world, scaling, tmp_path):
    """weak: the image grows with the ranks (128 x 64*world); strong (bench.py's default): a fixed 128x128
    image dealt to the ranks -- at world 3 its 4 tiles split 2/1/1, so the gather buffers are padded."""
    cfg = CONFIGS["cfg2"]
    patches = bzr.TriMesh().make_ellipsoid(32, 16, (1, 4, 2)).translate((10, 0, 0)).standardize().bezier_patches()
    width, height = (128, 64 * world) if scaling == "weak" else (128, 128)
    out = tmp_path / "frame.npz"
    mp.start_processes(worker, args=(world, free_port(), width, height, patches, str(out)), nprocs=world,
                       join=True, start_method="spawn")
    got = np.load(out)
    rows, cols, rays = frame.rank_rays(cfg, 0, 1, width, height)
    o, s, g = orc.trace_chain([patches], [1.3], rays)
    flat = rows * width + cols
    assert np.array_equal(got["status"][flat], s) and np.array_equal(got["seg"][flat], g)
    assert np.array_equal(got["rays"][:, flat].view(np.uint32), o.view(np.uint32))
    assert got["seg"].sum() > width * height  # refracted segments were traced


@pytest.mark.parametrize("world,side", [(3, 128), (8, 256)])
def test_image_layout_gather(bzr, orc, tmp_path, world, side):
    """bench.py's default multi-GPU gather (--gather image): only the status/segment word per primary
    reaches rank 0 (4 B instead of 28 B); the assembled image equals the single-process trace's.  World 8
    is the driver's SCALE run's largest rank count (a 256^2 image: 16 tiles, 2 per rank)."""
    cfg = CONFIGS["cfg2"]
    patches = bzr.TriMesh().make_ellipsoid(32, 16, (1, 4, 2)).translate((10, 0, 0)).standardize().bezier_patches()
    width = height = side
    out = tmp_path / "image.npz"
    mp.start_processes(worker, args=(world, free_port(), width, height, patches, str(out), "image"), nprocs=world,
                       join=True, start_method="spawn")
    got = np.load(out)
    assert "rays" not in got.files
    rows, cols, rays = frame.rank_rays(cfg, 0, 1, width, height)
    o, s, g = orc.trace_chain([patches], [1.3], rays)
    flat = rows * width + cols
    assert np.array_equal(got["status"][flat], s) and np.array_equal(got["seg"][flat], g)
    assert (got["status"] != 0).any()


@pytest.mark.parametrize("world", [1, 3, 8])
def test_tile_deal_covers_the_image_centre_first(world):
    """configs.shard_pixels: the ranks' tiles partition the image (every pixel once), each rank's 64x64
    tiles listed nearest the image centre first, each tile in 8x8 wavefront blocks."""
    from bzr_amd.configs import shard_pixels

    cfg, side = CONFIGS["cfg4"], 512
    seen = np.zeros(side * side, np.int64)
    for r in range(world):
        rows, cols = shard_pixels(cfg, r, world, side=side)
        seen[rows * side + cols] += 1
        tr, tc = rows.reshape(-1, 4096).mean(axis=1) + 0.5, cols.reshape(-1, 4096).mean(axis=1) + 0.5  # tile centres
        dist2 = (tr - side / 2) ** 2 + (tc - side / 2) ** 2
        assert np.all(np.diff(dist2) >= -1e-9)
        w = rows.reshape(-1, 64)  # one wavefront: an 8x8 block
        assert np.all(w.max(axis=1) - w.min(axis=1) == 7)
    assert np.all(seen == 1)


def loop_worker(rank, world, port, width, height, patches, result_path, layout, inflight, frames):
    """bench.py's loop (frame.FrameLoop): `inflight` slots, double-buffered async gather, the oracle as
    each slot's tracer; frame k refracts with ri = 1.3 + 0.02 k so every frame's result differs and a
    frame gathered under the wrong index would be caught.  Rank 0 assembles every frame as it lands."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import pyoracle

        cfg = CONFIGS["cfg2"]
        rows, cols, rays = frame.rank_rays(cfg, rank, world, width, height)
        n = rays.shape[1]
        npad = frame.padded_count(world, width, height)
        outs = [(torch.zeros((6, n)), torch.zeros(n, dtype=torch.int32), torch.zeros(n, dtype=torch.int32))
                for _ in range(inflight)]

        def trace(slot, k):
            o, s, g = pyoracle.trace_chain([patches], [1.3 + 0.02 * k], rays, threads=2)
            outs[slot][0].copy_(torch.from_numpy(o))
            outs[slot][1].copy_(torch.from_numpy(s.view(np.int32)))
            outs[slot][2].copy_(torch.from_numpy(g.view(np.int32)))

        cap = 0
        if layout == "compact":  # capacity from a first frame's survivor count (max over ranks), as bench.py
            trace(0, 0)
            cnt = torch.tensor([int(frame.survivors(outs[0][1], outs[0][2]).sum())])
            dist.all_reduce(cnt, op=dist.ReduceOp.MAX)
            cap = frame.compact_capacity(int(cnt[0]), npad)
        got = {}

        def on_gathered(k, parts):
            got[k] = frame.assemble(parts, cfg, world, width, height, cap=cap)

        loop = frame.FrameLoop(world, rank, n, npad, layout, trace, outs, cap=cap, on_gathered=on_gathered)
        for _ in range(frames):
            loop.step(inflight)
        loop.drain()
        if rank == 0:
            np.savez(result_path, **{f"{name}{k}": a for k, v in got.items() for name, a in zip(("rays", "status", "seg"), v)
                                     if a is not None}, frames=np.array(sorted(got)), bytes=np.array(loop.bytes_per_rank))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("layout,inflight,frames", [("compact", 3, 5), ("rays", 3, 5), ("image", 3, 5), ("image", 6, 8)])
def test_frame_loop_inflight_async_gather(bzr, orc, tmp_path, layout, inflight, frames):
    """frame.FrameLoop at world size 2 with 3 frames in flight and 5 frames (and, in the image layout, bench.py's
    6 slots for small rank frames over 8 frames): every frame lands on rank 0 once, under its own index, equal to a
    single-process trace of that frame; the compact layout delivers every final ray in fewer bytes than the rays
    layout."""
    cfg = CONFIGS["cfg2"]
    patches = bzr.TriMesh().make_ellipsoid(32, 16, (1, 4, 2)).translate((10, 0, 0)).standardize().bezier_patches()
    width = height = 128
    world = 2
    out = tmp_path / "loop.npz"
    mp.start_processes(loop_worker, args=(world, free_port(), width, height, patches, str(out), layout, inflight, frames),
                       nprocs=world, join=True, start_method="spawn")
    got = np.load(out)
    assert list(got["frames"]) == list(range(frames))
    rows, cols, rays = frame.rank_rays(cfg, 0, 1, width, height)
    flat = rows * width + cols
    for k in range(frames):
        o, s, g = orc.trace_chain([patches], [1.3 + 0.02 * k], rays)
        assert np.array_equal(got[f"status{k}"][flat], s) and np.array_equal(got[f"seg{k}"][flat], g), k
        if layout != "image":
            assert np.array_equal(got[f"rays{k}"][:, flat].view(np.uint32), o.view(np.uint32)), k
    npad = frame.padded_count(world, width, height)
    if layout == "compact":
        assert int(got["bytes"]) < 0.8 * frame.PACKED_ROWS * 4 * npad


def test_compact_capacity_overflow_is_reported():
    """A frame with more survivors than the compact capacity is refused on rank 0, not truncated."""
    n = npad = 4096
    status = torch.zeros(n, dtype=torch.int32)
    seg = torch.full((n,), 2, dtype=torch.int32)
    seg[:100] = 1
    rays = torch.randn(6, n)
    cap = 1000
    packed = torch.zeros(frame.compact_size(npad, cap))
    frame.pack_compact(status, seg, rays, packed, npad, cap)
    with pytest.raises(RuntimeError, match="capacity"):
        frame.unpack_compact(packed, n, npad, cap, np.zeros((6, n), np.float32))
    cap = n
    packed = torch.zeros(frame.compact_size(npad, cap))
    frame.pack_compact(status, seg, rays, packed, npad, cap)
    r, st, sg = frame.unpack_compact(packed, n, npad, cap, np.zeros((6, n), np.float32))
    assert np.array_equal(r[:, 100:], rays.numpy()[:, 100:]) and (r[:, :100] == 0).all()
    assert np.array_equal(sg, seg.numpy().astype(np.uint32))


@pytest.mark.parametrize("layout", ["compact", "rays", "image"])
def test_verify_gathered_accepts_the_frame_and_rejects_a_corrupted_part(bzr, orc, layout):
    """bench.py's multi-rank check (frame.verify_gathered): rank 0 compares the gathered
    parts with the same frame traced in one process.  Two ranks' parts packed from the oracle's trace pass;
    one flipped bit in one part, or a compact count word that disagrees with the flagged survivors, fails."""
    import torch

    cfg = CONFIGS["cfg2"]
    patches = bzr.TriMesh().make_ellipsoid(32, 16, (1, 4, 2)).translate((10, 0, 0)).standardize().bezier_patches()
    world, width, height = 2, 128, 128
    npad = frame.padded_count(world, width, height)
    per_rank = []
    for r in range(world):
        _, _, rays = frame.rank_rays(cfg, r, world, width, height)
        per_rank.append(orc.trace_chain([patches], [1.3], rays, threads=2))
    cap = frame.compact_capacity(max(int(frame.survivors(s, g).sum()) for _, s, g in per_rank), npad)
    parts = []
    for o, s, g in per_rank:
        to = (torch.from_numpy(o), torch.from_numpy(s.view(np.int32)), torch.from_numpy(g.view(np.int32)))
        if layout == "compact":
            p = torch.zeros(frame.compact_size(npad, cap))
            frame.pack_compact(to[1], to[2], to[0], p, npad, cap)
        else:
            p = torch.zeros((frame.PACKED_ROWS if layout == "rays" else frame.IMAGE_ROWS, npad))
            frame.pack(*to, p)
        parts.append(p)
    rows, cols, rays = frame.rank_rays(cfg, 0, 1, width, height)
    o, s, g = orc.trace_chain([patches], [1.3], rays, threads=2)
    flat = rows * width + cols
    want = {"rays": np.zeros((6, width * height), np.float32), "status": np.zeros(width * height, np.uint32),
            "segments": np.zeros(width * height, np.uint32)}
    want["rays"][:, flat], want["status"][flat], want["segments"][flat] = o, s, g
    res = frame.verify_gathered(parts, layout, cfg, world, width, height, want, cap=cap)
    assert res["ok"] and res["mismatched_pixels"] == 0, res
    assert ("rays[6]" in res["compared"]) == (layout != "image")
    if layout == "compact":
        assert 0 < res["survivors_max"] <= cap
    bad = [p.clone() for p in parts]
    if layout == "image":  # a segment count off by one in rank 1's word row
        w = bad[1][0].view(torch.int32)
        w[5] += 1 << 8
    elif layout == "rays":
        bad[1][2, 7] = torch.nextafter(bad[1][2, 7], torch.tensor(1e30))
    else:  # a survivor's ray, then the count word
        nw = frame.compact_words(npad)
        bad[1][nw + 1 + 3] = torch.nextafter(bad[1][nw + 1 + 3], torch.tensor(1e30))
    res = frame.verify_gathered(bad, layout, cfg, world, width, height, want, cap=cap)
    assert not res["ok"] and res["mismatched_pixels"] == 1, res
    if layout == "compact":
        bad = [p.clone() for p in parts]
        bad[0][nw:nw + 1].view(torch.int32)[0] -= 1
        res = frame.verify_gathered(bad, layout, cfg, world, width, height, want, cap=cap)
        assert not res["ok"] and "not fully gathered" in res["error"]
