#!/usr/bin/env python3
"""Sustained-clock evidence for the headline number (MI355X_MICROARCH.md "DVFS give-back").

Runs the bench workload (cfg4, fused, parity, frames in flight like bench.py) back to back for --seconds,
reporting Mrays/s per window of --window frames (a synchronize closes each window), then stamps one more
frame with bzr_debug_wave_clock_rate: per wave, d(s_memtime) / d(s_memrealtime) x 100 MHz is the shader
clock that wave ran at.  Prints one JSON line.  The stamps go to their own device buffer; no output is
computed from them, and the timed windows run the normal kernel (stamping off).

usage: python scripts/sustained_clock.py [--seconds 3] [--window 50] [--inflight 3]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys
import time
from pathlib import Path

if not os.environ.get("GPU_MAX_HW_QUEUES", "").isdigit() or int(os.environ["GPU_MAX_HW_QUEUES"]) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"  # the frame slots need their own hardware queues (bench.py)
REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "cuda-bezier-triangle-raytracer_amd"), str(REPO)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--window", type=int, default=50)
    ap.add_argument("--inflight", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch

    import bzr_amd
    from bzr_amd import frame
    from bzr_amd.configs import CONFIGS, build_lens

    cfg = CONFIGS["cfg4"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    patches = [build_lens(bzr_amd.TriMesh, l).bezier_patches() for l in cfg.lenses]
    ris = [l.ri for l in cfg.lenses]
    F = a.inflight
    streams = [torch.cuda.Stream(dev) for _ in range(F)]
    ctxs = [bzr_amd.Context(0) for _ in range(F)]
    for c, st in zip(ctxs, streams):
        c.use_torch_stream(st)
    meshes = [bzr_amd.DeviceMesh(ctxs[0], p) for p in patches]
    _, _, rays_np = frame.rank_rays(cfg, 0, 1, cfg.side, cfg.side)
    n = rays_np.shape[1]
    rays = torch.from_numpy(rays_np).to(dev)
    outs = [(torch.empty((6, n), dtype=torch.float32, device=dev), torch.empty(n, dtype=torch.int32, device=dev),
             torch.empty(n, dtype=torch.int32, device=dev)) for _ in range(F)]
    mode = bzr_amd.MODE_PARITY | bzr_amd.PIPELINE_FUSED
    k = [0]

    def step():
        f = k[0] % F
        with torch.cuda.stream(streams[f]):
            bzr_amd.trace_chain(ctxs[f], meshes, ris, rays, *outs[f], mode=mode)
        k[0] += 1

    step()
    torch.cuda.synchronize()
    segs = int(outs[0][2].sum().item())
    windows = []
    t_all = time.perf_counter()
    while time.perf_counter() - t_all < a.seconds:
        t0 = time.perf_counter()
        for _ in range(a.window):
            step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        windows.append(round(segs * a.window / dt / 1e6, 1))
    total_s = time.perf_counter() - t_all
    # one stamped frame right after the sustained run (slot 0's context, its own stream)
    waves = (n + 63) // 64
    clock = torch.zeros(4 * waves, dtype=torch.int64, device=dev)
    L = bzr_amd.lib()
    assert L.bzr_debug_wave_clock_rate(ctxs[0].handle, ctypes.c_void_p(clock.data_ptr()), waves) == 0
    k[0] = 0
    step()
    torch.cuda.synchronize()
    assert L.bzr_debug_wave_clock_rate(ctxs[0].handle, None, 0) == 0
    c = clock.view(-1, 4).cpu().numpy().astype(np.float64)
    ok = c[:, 3] > 100  # waves of >= 1 us (100 MHz ticks): the ratio's resolution
    ghz = c[ok, 1] / c[ok, 3] * 0.1
    line = {
        "workload": "cfg4 4096^2 two-lens chain, fused, parity",
        "frames_in_flight": F,
        "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"),
        "segments_per_frame": segs,
        "sustained_s": round(total_s, 3),
        "frames": a.window * len(windows),
        "window_frames": a.window,
        "mrays_per_s_windows": windows,
        "mrays_per_s_first_last_median": [windows[0], windows[-1], statistics.median(windows)],
        "last_vs_first": round(windows[-1] / windows[0], 4),
        "in_kernel_clock_ghz": {"median": round(float(np.median(ghz)), 4), "p10": round(float(np.percentile(ghz, 10)), 4),
                                "p90": round(float(np.percentile(ghz, 90)), 4), "waves": int(ok.sum()),
                                "method": "per wave d(s_memtime)/d(s_memrealtime) x 100 MHz, one stamped frame "
                                          "right after the sustained run (bzr_debug_wave_clock_rate)"},
    }
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
