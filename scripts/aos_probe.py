#!/usr/bin/env python3
"""The record-layout conversions on the device (BZR_RAYS_AOS, bzr_intersect_records) at the bench frame size, for
rocprofv3 --kernel-trace: cfg4's 4096^2 primaries as [n, 6] records on the device through bzr_trace_chain
(k_rays_aos_to_soa in, k_rays_soa_to_aos out) and lens 1's bzr_intersect_records (k_hits_to_records), 5 calls
each after a warm-up.  Prints the per-call wall times; the kernel durations come from the trace.
usage: rocprofv3 --kernel-trace --stats -d DIR -o run -- python3 scripts/aos_probe.py
"""
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "cuda-bezier-triangle-raytracer_amd"), str(REPO)]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bzr_amd as bzr  # noqa: E402
from bzr_amd.configs import CONFIGS, build_lens, grid_rays  # noqa: E402


def main():
    cfg = CONFIGS["cfg4"]
    ctx = bzr.Context(0)
    lenses = [bzr.DeviceMesh(ctx, build_lens(bzr.TriMesh, lens).bezier_patches()) for lens in cfg.lenses]
    ri = [lens.ri for lens in cfg.lenses]
    rows = grid_rays(cfg, side=4096)
    n = rows.shape[1]
    rec = torch.from_numpy(np.ascontiguousarray(rows.T)).cuda()
    out = (torch.empty((n, 6), device="cuda"), torch.empty(n, dtype=torch.int32, device="cuda"),
           torch.empty(n, dtype=torch.int32, device="cuda"))
    hits = torch.empty((n, 13), dtype=torch.int32, device="cuda")
    patch = torch.empty(n, dtype=torch.int32, device="cuda")
    for label, call in (("trace_chain RAYS_AOS", lambda: bzr.trace_chain(ctx, lenses, ri, rec, *out, mode=bzr.RAYS_AOS)),
                        ("intersect_records RAYS_AOS",
                         lambda: bzr.intersect_records(ctx, lenses[0], rec, hits, patch, mode=bzr.RAYS_AOS))):
        call()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            call()
        torch.cuda.synchronize()
        print(f"{label}: {(time.perf_counter() - t0) / 5 * 1e3:.3f} ms per call, {n} rays", flush=True)


if __name__ == "__main__":
    main()
