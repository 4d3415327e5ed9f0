#!/usr/bin/env python3
"""In-process A/B of libbzr.so builds (lib/<variant>/libbzr.so): interleaved rounds on one device.

usage: python scripts/ab.py [--config cfg2] [--rounds 7] [--steps 10] variant [variant ...]
       variant "base" = lib/libbzr.so.  Prints, per variant, the median / min chain time, the per-kernel
       averages and whether its outputs are bit-identical to the first variant's.
"""
import argparse
import ctypes
import json
import statistics
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
PKG = REPO / "cuda-bezier-triangle-raytracer_amd"
sys.path.insert(0, str(PKG))
sys.path.insert(0, str(REPO))


def bind(path):
    import bzr_amd
    h = ctypes.CDLL(str(path))
    for name, args in bzr_amd._SIGS.items():
        if not hasattr(h, name):  # (an older build, e.g. a previous round's library: its debug hooks differ)
            continue
        f = getattr(h, name)
        f.argtypes = args
        f.restype = bzr_amd._RET.get(name, ctypes.c_int32)
    return h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--side", type=int, default=0, help="rays per image side (0 = the config's own)")
    ap.add_argument("--pipeline", default="fused", choices=["fused", "staged", "auto"])
    ap.add_argument("--wave", default="8x8", help="rows x cols of image pixels per 64-ray wave (ray order)")
    a = ap.parse_args()
    import torch

    import bzr_amd
    from bzr_amd.configs import CONFIGS, build_lens, grid_rays

    cfg = CONFIGS[a.config]
    pflag = {"fused": bzr_amd.PIPELINE_FUSED, "staged": bzr_amd.PIPELINE_STAGED, "auto": 0}[a.pipeline]
    patches = [build_lens(bzr_amd.TriMesh, l).bezier_patches() for l in cfg.lenses]
    ris = (ctypes.c_float * len(patches))(*[l.ri for l in cfg.lenses])
    wave = tuple(int(x) for x in a.wave.split("x"))
    rays = torch.from_numpy(grid_rays(cfg, side=a.side or None, wave=wave)).cuda()
    n = rays.shape[1]
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    runs = []
    for v in a.variants:
        path = PKG / "lib" / "libbzr.so" if v == "base" else PKG / "lib" / v / "libbzr.so"
        h = bind(path)
        ctx = ctypes.c_void_p()
        assert h.bzr_ctx_create(0, ctypes.byref(ctx)) == 0, h.bzr_last_error()
        h.bzr_ctx_set_stream(ctx, ctypes.c_void_p(stream.cuda_stream))
        meshes = []
        for p in patches:
            m = ctypes.c_void_p()
            pa = np.ascontiguousarray(p, dtype=np.float32)
            assert h.bzr_mesh_create(ctx, pa.ctypes.data, len(pa), 264, ctypes.byref(m)) == 0, h.bzr_last_error()
            meshes.append(m)
        marr = (ctypes.c_void_p * len(meshes))(*[m.value for m in meshes])
        if cfg.op == "chain":
            out = torch.empty((6, n), dtype=torch.float32, device="cuda")
            st = torch.empty(n, dtype=torch.int32, device="cuda")
            sg = torch.empty(n, dtype=torch.int32, device="cuda")

            def step(h=h, ctx=ctx, marr=marr, out=out, st=st, sg=sg):
                r = h.bzr_trace_chain(ctx, marr, ris, len(patches), ctypes.c_void_p(rays.data_ptr()), n,
                                      ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(st.data_ptr()),
                                      ctypes.c_void_p(sg.data_ptr()), bzr_amd.DEVICE_PTRS | pflag)
                assert r == 0, h.bzr_last_error()
        else:  # BezierMesh::intersect configs (cfg3, cfg5): one segment per ray
            out = torch.empty((13, n), dtype=torch.float32, device="cuda")
            st = torch.zeros(1, dtype=torch.int32, device="cuda")
            sg = torch.ones(n, dtype=torch.int32, device="cuda")

            def step(h=h, ctx=ctx, m=meshes[0], out=out):
                r = h.bzr_intersect(ctx, m, ctypes.c_void_p(rays.data_ptr()), n, ctypes.c_void_p(out.data_ptr()),
                                    bzr_amd.DEVICE_PTRS | pflag)
                assert r == 0, h.bzr_last_error()
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        runs.append(dict(name=v, h=h, ctx=ctx, step=step, out=out, st=st, sg=sg, times=[], kern={}))
    ref = runs[0]
    for r in runs:
        same = torch.equal(r["out"].view(torch.int32), ref["out"].view(torch.int32)) and torch.equal(r["st"], ref["st"]) \
            and torch.equal(r["sg"], ref["sg"])
        r["same"] = bool(same)
    for _ in range(a.rounds):
        for r in runs:
            h, ctx = r["h"], r["ctx"]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(stream)
            for _ in range(a.steps):
                r["step"]()
            e1.record(stream)
            torch.cuda.synchronize()
            r["times"].append(e0.elapsed_time(e1) / a.steps)
            # per-kernel event timing in a separate pass (the events perturb the chain time)
            h.bzr_ctx_timing(ctx, 1)
            ms = (ctypes.c_float * 16)()
            calls = (ctypes.c_uint32 * 16)()
            h.bzr_ctx_timing_report(ctx, ms, calls)
            for _ in range(a.steps):
                r["step"]()
            h.bzr_ctx_timing_report(ctx, ms, calls)
            h.bzr_ctx_timing(ctx, 0)
            for k, name in enumerate(bzr_amd.KERNELS):
                if calls[k]:
                    r["kern"].setdefault(name, []).append(ms[k] / a.steps)
    segs = int(ref["sg"].sum().item())
    for r in runs:  # work counters of one frame
        h, ctx = r["h"], r["ctx"]
        cnt = (ctypes.c_uint64 * 16)()
        h.bzr_ctx_counters(ctx, 1)
        h.bzr_ctx_counters_report(ctx, cnt)
        r["step"]()
        h.bzr_ctx_counters_report(ctx, cnt)
        h.bzr_ctx_counters(ctx, 0)
        r["counters"] = {k: int(cnt[i]) for i, k in enumerate(bzr_amd.COUNTERS)}
    for r in runs:
        med = statistics.median(r["times"])
        print(json.dumps({"variant": r["name"], "same_as_first": r["same"], "ms_median": round(med, 4),
                          "ms_min": round(min(r["times"]), 4), "mrays_s": round(segs / med / 1e3, 1),
                          "kernels_ms_per_step": {k: round(statistics.median(v), 4) for k, v in r["kern"].items()},
                          "counters": r["counters"]}),
              flush=True)


if __name__ == "__main__":
    main()
