#!/usr/bin/env python3
"""Why does the BZR_TRACE_BUNDLE build count 4096 overflow rays where 1026 origins are far?

Runs tests/test_gpu_fused.py::test_far_origins_take_the_inline_full_scan's rays (robot.stl, 25 % of the
origins beyond s_max) through k_trace on the library named by BZR_LIBRARY, plus two controls: the same
rays with every origin near, and coherent rays.  Prints the device counters of each as one JSON line.
usage: BZR_LIBRARY=.../lib/tracebundle/libbzr.so python scripts/bundle_overflow_probe.py
"""
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "cuda-bezier-triangle-raytracer_amd"), str(REPO)]

import bzr_amd as bzr  # noqa: E402
from bzr_amd.configs import CONFIGS, build_lens  # noqa: E402


def rays_of(far_frac, seed=11, n=4096, spread=20.0):
    rng = np.random.default_rng(seed)
    o = rng.uniform(-30, 30, (3, n)).astype(np.float32)
    far = rng.random(n) < far_frac
    o[0, far] = np.float32(-5e4)
    tgt = rng.uniform(-spread, spread, (3, n)).astype(np.float32)
    d = tgt - o
    d /= np.sqrt((d * d).sum(axis=0, keepdims=True)).astype(np.float32)
    return np.concatenate([o, d.astype(np.float32)]).astype(np.float32), int(far.sum())


def main():
    ctx = bzr.Context(0)
    lens = build_lens(bzr.TriMesh, CONFIGS["cfg3"].lenses[0].__class__("stl", split=1)).bezier_patches()
    dm = bzr.DeviceMesh(ctx, lens)
    out = {"library": str(bzr.LIB_PATH)}
    for name, (rays, nfar) in {"mixed_25pct_far": rays_of(0.25), "all_near": rays_of(0.0),
                               "all_far": rays_of(1.0)}.items():
        ctx.counters(True)
        ctx.counters_report()
        got = bzr.intersect(ctx, dm, rays, mode=bzr.PIPELINE_FUSED)
        cnt = ctx.counters_report()
        ctx.counters(False)
        ref = bzr.intersect(ctx, dm, rays, mode=bzr.ACCEL_NONE)
        out[name] = dict(cnt, far=nfar, equal_bruteforce=bool(np.array_equal(got.view(np.uint32), ref.view(np.uint32))))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
