#!/usr/bin/env python3
"""A rank's k_trace time with its 64x64 tiles in dealing order vs centre-first (heavy tiles dispatched
first, so the frame's tail is made of short waves): rank 0's share of the fixed 4096^2 cfg4 image at
world sizes 1, 2, 4, 8, on one GPU."""
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "cuda-bezier-triangle-raytracer_amd"))
sys.path.insert(0, str(REPO))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bzr_amd  # noqa: E402
from bzr_amd.configs import CONFIGS, build_lens, rays_for, shard_pixels  # noqa: E402

K = 20
cfg = CONFIGS["cfg4"]
side = 4096
patches = [build_lens(bzr_amd.TriMesh, l).bezier_patches() for l in cfg.lenses]
slot_ctx = [bzr_amd.Context(0) for _ in range(3)]
slot_streams = [torch.cuda.Stream() for _ in range(3)]  # back to back: distinct hardware queues
for c, st in zip(slot_ctx, slot_streams):
    c.use_torch_stream(st)
ctx, stream = slot_ctx[0], slot_streams[0]
torch.cuda.set_stream(stream)
meshes = [bzr_amd.DeviceMesh(ctx, p) for p in patches]
ris = [l.ri for l in cfg.lenses]
mode = bzr_amd.MODE_PARITY | bzr_amd.PIPELINE_FUSED


def centre_first(rows, cols):
    t = 64 * 64
    r, c = rows.reshape(-1, t), cols.reshape(-1, t)
    cy, cx = r.mean(axis=1) - side / 2, c.mean(axis=1) - side / 2
    o = np.argsort(cy * cy + cx * cx, kind="stable")
    return r[o].reshape(-1), c[o].reshape(-1)


def by_cost(rows, cols, key):
    t = 64 * 64
    r, c = rows.reshape(-1, t), cols.reshape(-1, t)
    o = np.argsort(-key, kind="stable")
    return r[o].reshape(-1), c[o].reshape(-1)


def tile_segments(rows, cols):
    """Segments per 64x64 tile from one traced frame (the chain's per-ray segment count)."""
    rays = torch.from_numpy(rays_for(cfg, rows, cols, side)).cuda()
    n = rays.shape[1]
    out = torch.empty((6, n), dtype=torch.float32, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    sg = torch.empty(n, dtype=torch.int32, device="cuda")
    bzr_amd.trace_chain(ctx, meshes, ris, rays, out, st, sg, mode=mode)
    return sg.view(-1, 64 * 64).sum(dim=1).cpu().numpy()


def wave_cost(rows, cols):
    """Per 64x64 tile: the largest per-wave segment sum (the tile's slowest wave)."""
    rays = torch.from_numpy(rays_for(cfg, rows, cols, side)).cuda()
    n = rays.shape[1]
    out = torch.empty((6, n), dtype=torch.float32, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    sg = torch.empty(n, dtype=torch.int32, device="cuda")
    bzr_amd.trace_chain(ctx, meshes, ris, rays, out, st, sg, mode=mode)
    return sg.view(-1, 64, 64).sum(dim=2).max(dim=1).values.cpu().numpy()


for world in (1, 2, 4, 8):
    rows, cols = shard_pixels(cfg, 0, world, side=side, order="dealt")  # tiles k = rank, rank + world, ...
    res = {}
    seg = tile_segments(rows, cols)
    cy = rows.reshape(-1, 4096).mean(axis=1) - side / 2
    cx = cols.reshape(-1, 4096).mean(axis=1) - side / 2
    orders = (("dealt", (rows, cols)), ("centre_first", centre_first(rows, cols)))
    for name, (rr, cc) in orders:
        rays = torch.from_numpy(rays_for(cfg, rr, cc, side)).cuda()
        n = rays.shape[1]
        out = torch.empty((6, n), dtype=torch.float32, device="cuda")
        st = torch.empty(n, dtype=torch.int32, device="cuda")
        sg = torch.empty(n, dtype=torch.int32, device="cuda")
        times = []
        for rep in range(3):
            for _ in range(3):
                bzr_amd.trace_chain(ctx, meshes, ris, rays, out, st, sg, mode=mode)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(K):
                bzr_amd.trace_chain(ctx, meshes, ris, rays, out, st, sg, mode=mode)
            e1.record(stream)
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) / K)
        res[name] = round(float(np.median(times)), 4)
    # F frames in flight (own context, stream, outputs each), centre-first order
    rr, cc = centre_first(rows, cols)
    rays = torch.from_numpy(rays_for(cfg, rr, cc, side)).cuda()
    n = rays.shape[1]
    for F in (2, 3):
        bufs = [(torch.empty((6, n), dtype=torch.float32, device="cuda"), torch.empty(n, dtype=torch.int32, device="cuda"),
                 torch.empty(n, dtype=torch.int32, device="cuda")) for _ in range(F)]
        times = []
        for rep in range(3):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for st in slot_streams[1:F]:
                st.wait_event(e0)
            for k in range(K):
                c, st = slot_ctx[k % F], slot_streams[k % F]
                with torch.cuda.stream(st):
                    bzr_amd.trace_chain(c, meshes, ris, rays, *bufs[k % F], mode=mode)
            for st in slot_streams[1:F]:
                ev = torch.cuda.Event()
                ev.record(st)
                stream.wait_event(ev)
            e1.record(stream)
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) / K)
        res[f"centre_inflight{F}"] = round(float(np.median(times)), 4)
    print(json.dumps({"world": world, "rank0_rays": int(len(rows)), **res}), flush=True)
