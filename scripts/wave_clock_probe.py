#!/usr/bin/env python3
"""Per-wave start/duration of k_trace (bzr_debug_wave_clock) on rank 0's share of the cfg4 image at world
sizes 1 and 8: how long the slowest waves run, when they start, and what the frame's tail is made of."""
import ctypes
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

cfg = CONFIGS["cfg4"]
side = 4096
patches = [build_lens(bzr_amd.TriMesh, l).bezier_patches() for l in cfg.lenses]
ctx = bzr_amd.Context(0)
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
ctx.use_torch_stream(stream)
meshes = [bzr_amd.DeviceMesh(ctx, p) for p in patches]
ris = [l.ri for l in cfg.lenses]
mode = bzr_amd.MODE_PARITY | bzr_amd.PIPELINE_FUSED
L = bzr_amd.lib()


def centre_first(rows, cols):
    t = 64 * 64
    r, c = rows.reshape(-1, t), cols.reshape(-1, t)
    cy, cx = r.mean(axis=1) - side / 2, c.mean(axis=1) - side / 2
    o = np.argsort(cy * cy + cx * cx, kind="stable")
    return r[o].reshape(-1), c[o].reshape(-1)


for world in (1, 8):
    for order in ("dealt", "centre"):
        rows, cols = shard_pixels(cfg, 0, world, side=side)
        if order == "centre":
            rows, cols = centre_first(rows, cols)
        rays = torch.from_numpy(rays_for(cfg, rows, cols, side)).cuda()
        n = rays.shape[1]
        waves = n // 64
        clock = torch.zeros(2 * waves, dtype=torch.int64, device="cuda")
        out = torch.empty((6, n), dtype=torch.float32, device="cuda")
        st = torch.empty(n, dtype=torch.int32, device="cuda")
        sg = torch.empty(n, dtype=torch.int32, device="cuda")
        for _ in range(2):
            bzr_amd.trace_chain(ctx, meshes, ris, rays, out, st, sg, mode=mode)
        torch.cuda.synchronize()
        assert L.bzr_debug_wave_clock(ctx.handle, ctypes.c_void_p(clock.data_ptr()), waves) == 0
        bzr_amd.trace_chain(ctx, meshes, ris, rays, out, st, sg, mode=mode)
        torch.cuda.synchronize()
        assert L.bzr_debug_wave_clock(ctx.handle, None, 0) == 0
        c = clock.view(-1, 2).cpu().numpy().astype(np.float64)
        start, dur = c[:, 0] - c[:, 0].min(), c[:, 1]
        end = start + dur
        span = end.max()
        seg = sg.view(-1, 64).sum(dim=1).cpu().numpy()
        slow = np.argsort(-dur)[:20]
        q = lambda a, p: float(np.percentile(a, p))  # noqa: E731
        print(json.dumps({
            "world": world, "order": order, "waves": waves, "span_ticks": span,
            "dur_p50": q(dur, 50), "dur_p90": q(dur, 90), "dur_p99": q(dur, 99), "dur_max": float(dur.max()),
            "last_start": float(start.max()), "end_p99": q(end, 99), "end_p999": q(end, 99.9),
            "slowest": [{"wave": int(w), "start": float(start[w]), "dur": float(dur[w]), "segments": int(seg[w])} for w in slow[:8]],
            "dur_by_segments": {int(k): float(np.mean(dur[seg == k])) for k in np.unique(seg)[::16]},
        }), flush=True)
