#!/usr/bin/env python3
"""One rank's frame loop at the frame sizes of an N-rank strong-scaling run, on one GPU: rank 0's share of
the fixed cfg4 4096^2 image at N = 1, 2, 4, 8, traced by bench.py's loop (frame.FrameLoop, 3 frames in
flight) with each gather layout's packing on the device -- the torch packers of frame.py and bzr_pack_frame (bench.py's)
-- but no collective (pack_always; world 1).  Per
line: ms per frame (wall clock over K frames, synchronized at both ends) and the host's issue time per
frame (the loop alone, before the closing synchronize) -- a loop whose issue time approaches the frame time
would make an 8-GPU run host-bound.  The transport itself (RCCL over xGMI) is not in this probe.

usage: python scripts/rank_loop_probe.py [--frames 200] [--worlds 1,2,4,8] [--layouts none,image,compact]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

if not os.environ.get("GPU_MAX_HW_QUEUES", "").isdigit() or int(os.environ["GPU_MAX_HW_QUEUES"]) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"  # the frame slots need their own hardware queues (bench.py)
REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "cuda-bezier-triangle-raytracer_amd"), str(REPO)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--layouts", default="none,image,compact")
    ap.add_argument("--inflight", type=int, default=3)
    a = ap.parse_args()
    import torch

    import bzr_amd
    from bzr_amd import frame
    from bzr_amd.configs import CONFIGS, build_lens

    cfg = CONFIGS["cfg4"]
    side = cfg.side
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    F = a.inflight
    streams = [torch.cuda.Stream(dev) for _ in range(F)]
    ctxs = [bzr_amd.Context(0) for _ in range(F)]
    for c, st in zip(ctxs, streams):
        c.use_torch_stream(st)
    torch.cuda.set_stream(streams[0])
    meshes = [bzr_amd.DeviceMesh(ctxs[0], build_lens(bzr_amd.TriMesh, l).bezier_patches()) for l in cfg.lenses]
    ris = [l.ri for l in cfg.lenses]
    mode = bzr_amd.MODE_PARITY | bzr_amd.PIPELINE_FUSED
    for world in [int(w) for w in a.worlds.split(",")]:
        _, _, rays_np = frame.rank_rays(cfg, 0, world, side, side)
        n = rays_np.shape[1]
        npad = frame.padded_count(world, side, side)
        rays = torch.from_numpy(rays_np).to(dev)
        outs = [(torch.empty((6, n), dtype=torch.float32, device=dev), torch.empty(n, dtype=torch.int32, device=dev),
                 torch.empty(n, dtype=torch.int32, device=dev)) for _ in range(F)]

        def trace(f, k):
            bzr_amd.trace_chain(ctxs[f], meshes, ris, rays, *outs[f], mode=mode)

        trace(0, 0)
        torch.cuda.synchronize()
        cap = frame.compact_capacity(int(frame.survivors(outs[0][1], outs[0][2]).sum().item()), npad)
        runs = [(lay, pk) for lay in a.layouts.split(",") for pk in (("-",) if lay == "none" else ("torch", "hip"))]
        for layout, packer in runs:
            pack_fn = None
            if packer == "hip":  # bench.py's packer: bzr_pack_frame on the slot's context
                pack_fn = lambda out, p, f, lay=layout: bzr_amd.pack_frame(ctxs[f], lay, *out, p, npad, cap)  # noqa: E731
            loop = frame.FrameLoop(1, 0, n, npad, layout, trace, outs, stream_for=lambda f: torch.cuda.stream(streams[f]),
                                   cap=cap, device=dev, pack_always=True, pack_fn=pack_fn)
            for _ in range(3 * F):
                loop.step(F)
            loop.drain()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.frames):
                loop.step(F)
            t_issue = time.perf_counter() - t0
            loop.drain()
            torch.cuda.synchronize()
            t_all = time.perf_counter() - t0
            print(json.dumps({"world": world, "rank0_primaries": n, "layout": layout, "packer": packer, "frames": a.frames,
                              "ms_per_frame": round(t_all / a.frames * 1e3, 4),
                              "host_issue_ms_per_frame": round(t_issue / a.frames * 1e3, 4),
                              "packed_bytes": loop.bytes_per_rank}), flush=True)


if __name__ == "__main__":
    main()
