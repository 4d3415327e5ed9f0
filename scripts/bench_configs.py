#!/usr/bin/env python3
"""Throughput of the BASELINE.json configs on 1 GPU (bench.py measures cfg4): one JSON line each.

cfg3: robot.stl split x8 (28800 patches), 2048^2 primary rays, BezierMesh::intersect.
cfg4: two cfg2 lenses, 4096^2 rays, refraction chain (BASELINE quotes it on 8 GPUs; here 1 GPU's share
      would be 4096^2 / 8, so this is 8x one rank's work).
cfg5: 301056-patch ellipsoid, BezierMesh::intersect; 4096^2 of its 8192^2 grid (one quarter: the full
      grid is 8 GPUs' work, 2x one rank's share).
Inputs resident in HBM; K timed repetitions after one warm-up; Mrays/s counts BezierMesh::intersect calls.
usage: bench_configs.py [cfg2 cfg3 cfg4 cfg5] [--fast] [--pipeline fused|staged|auto]
"""
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "cuda-bezier-triangle-raytracer_amd"))
sys.path.insert(0, str(REPO))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bzr_amd  # noqa: E402
from bzr_amd.configs import CONFIGS, build_lens, grid_rays  # noqa: E402


def run(name, side, reps, mode=bzr_amd.MODE_PARITY):
    cfg = CONFIGS[name]
    t0 = time.perf_counter()
    patches = [build_lens(bzr_amd.TriMesh, l).bezier_patches() for l in cfg.lenses]
    prep = time.perf_counter() - t0
    ctx = bzr_amd.Context(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx.use_torch_stream(stream)
    t0 = time.perf_counter()
    meshes = [bzr_amd.DeviceMesh(ctx, p) for p in patches]
    upload = time.perf_counter() - t0
    rays = torch.from_numpy(grid_rays(cfg, side=side)).cuda()
    n = rays.shape[1]
    if cfg.op == "chain":
        o, s, g = (torch.empty((6, n), device="cuda"), torch.empty(n, dtype=torch.int32, device="cuda"),
                   torch.empty(n, dtype=torch.int32, device="cuda"))

        def step():
            bzr_amd.trace_chain(ctx, meshes, [l.ri for l in cfg.lenses], rays, o, s, g, mode=mode)
    else:
        hits = torch.empty((13, n), device="cuda")
        g = None

        def step():
            bzr_amd.intersect(ctx, meshes[0], rays, hits, mode=mode)
    step()
    torch.cuda.synchronize()
    segs = int(g.sum().item()) if g is not None else n
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    ctx.timing(True)  # per-kernel HIP-event times in a separate, untimed repetition
    ctx.timing_report()
    step()
    kern = {k: round(ms, 3) for k, (ms, calls) in ctx.timing_report().items()}
    ctx.timing(False)
    ctx.counters(True)
    ctx.counters_report()
    step()
    cnt = ctx.counters_report()
    ctx.counters(False)
    extra = {"kernels_ms": kern, "counters": cnt}
    if g is None:
        extra["hit_fraction"] = round(float((hits[11].view(torch.int32) == 4).float().mean().item()), 4)
    pipe = "fused" if mode & bzr_amd.PIPELINE_FUSED else "staged" if mode & bzr_amd.PIPELINE_STAGED else "auto"
    print(json.dumps({"config": name, "mode": "fast" if mode & bzr_amd.MODE_FAST else "parity", "pipeline": pipe,
                      "rays_side": side, "patches": int(sum(len(p) for p in patches)),
                      "segments_per_step": segs, "ms_per_step": round(dt * 1e3, 3),
                      "mrays_per_s": round(segs / dt / 1e6, 1), "preprocess_s": round(prep, 2),
                      "upload_bvh_s": round(upload, 2), **extra}), flush=True)
    del rays
    torch.cuda.empty_cache()


def main():
    args = sys.argv[1:]
    mode = bzr_amd.MODE_FAST if "--fast" in args else bzr_amd.MODE_PARITY
    pipeline = "auto"
    if "--pipeline" in args:
        pipeline = args[args.index("--pipeline") + 1]
        args.remove("--pipeline")
        args.remove(pipeline)
    mode |= {"fused": bzr_amd.PIPELINE_FUSED, "staged": bzr_amd.PIPELINE_STAGED, "auto": 0}[pipeline]
    which = [a for a in args if not a.startswith("--")] or ["cfg2", "cfg3", "cfg4", "cfg5"]
    plan = {"cfg2": (1024, 20), "cfg3": (2048, 10), "cfg4": (4096, 5), "cfg5": (8192, 3)}
    for name in which:
        run(name, *plan[name], mode=mode)


if __name__ == "__main__":
    main()
