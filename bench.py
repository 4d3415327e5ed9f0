#!/usr/bin/env python3
"""Throughput benchmark: Mrays/s (primary + refracted) of the Bezier-lens refraction chain.

Workload (BASELINE.json configs[1]): makeEllipsoid(32,16,(1,4,2)) lens at x=10,
refractive index 1.3, 1024x1024 primary rays along +x from the plane x=0 over y in [-4.2,4.2],
z in [-2.1,2.1]; each ray runs refract(INSIDE) then refract(OUTSIDE) (reference/test.cpp:376-401).
"Rays" counts every BezierMesh::intersect call (primary + refracted segments).  --config cfg4 runs
the two-lens 4096x4096 chain instead.

A step = one frame: the whole chain over this rank's primary rays, inputs already resident in HBM,
results bit-identical to the reference restatement (tests/test_gpu_parity.py).  N GPUs = N processes
(torch.distributed over RCCL): weak scaling -- the image grows to side x (side*N) pixels, 64x64
tiles dealt round-robin, side^2 rays per rank, and each frame's results (28 B per primary) are gathered to
rank 0 over RCCL inside the timed region (--gather step, the default), double-buffered so frame k's
gather overlaps frame k+1's tracing.

Prints ONE JSON line on rank 0; fields are described in DESIGN.md (Measurement).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "cuda-bezier-triangle-raytracer_amd"))
sys.path.insert(0, str(REPO))

VALU_PEAK_TFLOPS = 157.3      # MI355X FP32 vector peak (MI355X_MICROARCH.md, chip parameters)
HBM_PEAK_GBS = 8000.0         # MI355X HBM3E peak (spec)
FLOPS_PLANAR = 33.0           # algorithmic flops per (segment, patch) planar test
FLOPS_NEWTON = 1750.0         # algorithmic flops per Newton candidate: bracket + 4 iterations + tail
FLOPS_REFRACT = 30.0          # Snell step per segment
BYTES_PER_PRIMARY = 24 + 32   # ray in; ray + status + segment count out


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default="cfg2", choices=["cfg2", "cfg4"])
    p.add_argument("--side", type=int, default=0, help="override rays per image side (per rank)")
    p.add_argument("--gather", default="step", choices=["step", "none"])
    p.add_argument("--accel", default="bvh", choices=["bvh", "none"], help="none = brute-force scan (A/B)")
    p.add_argument("--mode", default="parity", choices=["parity", "fast"],
                   help="fast = BZR_MODE_FAST Newton stage (contracted FMA, approximate div/sqrt; not bit-exact)")
    p.add_argument("--cpu-baseline", default="on", choices=["on", "off"])
    p.add_argument("--cpu-sample-stride", type=int, default=2, help="oracle sample: every k-th row and column")
    return p.parse_args()


def cpu_baseline(cfg, side, patches, ris, stride):
    """The oracle (CPU restatement, test infrastructure) on a strided sample of the same workload;
    also returns its work counters (planar tests, Newton runs) used for the algorithmic flop count."""
    from bzr_amd.configs import pixel_coords, rays_for
    from oracle import pyoracle

    r, c = pixel_coords(cfg, side=side, order="rows")
    keep = (r % stride == 0) & (c % stride == 0)
    rays = rays_for(cfg, r[keep], c[keep], side=side)
    threads = min(16, os.cpu_count() or 1)
    pyoracle.counters_reset()
    t0 = time.perf_counter()
    _, _, seg = pyoracle.trace_chain(patches, ris, rays, threads=threads)
    dt = time.perf_counter() - t0
    cnt = pyoracle.counters()
    return {
        "value": round(float(seg.sum()) / dt / 1e6, 4),
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{rays.shape[1]} primaries (every {stride}th row and column of the {side}^2 grid), "
                  f"{int(seg.sum())} segments, {dt:.2f} s wall; oracle/bzr_oracle.c -O2, OpenMP {threads} threads",
    }, cnt


def pmc_traffic(kernel, workload, same_workload):
    """HBM bytes per launch of `kernel` ("a+b" sums the parts) from the committed PMC profile of this
    workload (profiles/pmc_traffic.json, written by scripts/prof_summary.py from rocprofv3 FETCH_SIZE x2
    + WRITE_SIZE passes over bench.py).  PMC counters cannot be read from inside the timed process."""
    path = REPO / "profiles" / "pmc_traffic.json"
    if not same_workload or not path.exists():
        return None, None
    d = json.loads(path.read_text())
    if d.get("workload") != workload:
        return None, None
    parts = kernel.split("+")
    if not all(p in d["kernels"] for p in parts):
        return None, None
    total = sum(d["kernels"][p].get("read", 0.0) + d["kernels"][p].get("write", 0.0) for p in parts)
    return round(total), f"{d['source']} ({d['method']})"


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    import bzr_amd
    from bzr_amd import frame
    from bzr_amd.configs import CONFIGS, build_lens

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # BZR_BENCH_DEVICE: pin every rank to one device index (multi-rank rehearsal on a 1-GPU box only)
    local = int(os.environ.get("BZR_BENCH_DEVICE", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world > 1:
        backend = os.environ.get("BZR_BENCH_BACKEND", "nccl")  # "gloo": rehearsal on a 1-GPU box only
        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)

    cfg = CONFIGS[a.config]
    side = a.side or cfg.side
    t0 = time.perf_counter()
    patches = [build_lens(bzr_amd.TriMesh, lens).bezier_patches() for lens in cfg.lenses]
    ris = [lens.ri for lens in cfg.lenses]
    prep_s = time.perf_counter() - t0
    n_patch = sum(len(p) for p in patches)

    ctx = bzr_amd.Context(local)
    t0 = time.perf_counter()
    meshes = [bzr_amd.DeviceMesh(ctx, p) for p in patches]  # upload + BVH build
    upload_s = time.perf_counter() - t0
    stream = torch.cuda.Stream(dev)   # one stream for the kernels, torch ops and the timing events
    torch.cuda.set_stream(stream)
    ctx.use_torch_stream(stream)
    mode = bzr_amd.ACCEL_NONE if a.accel == "none" else bzr_amd.MODE_PARITY
    if a.mode == "fast":
        mode |= bzr_amd.MODE_FAST

    _, _, rays_np = frame.rank_rays(cfg, rank, world, side, side * world)
    n = rays_np.shape[1]
    rays = torch.from_numpy(rays_np).to(dev)
    out_rays = torch.empty((6, n), dtype=torch.float32, device=dev)
    out_status = torch.empty(n, dtype=torch.int32, device=dev)
    out_seg = torch.empty(n, dtype=torch.int32, device=dev)
    # double-buffered frame gather: frame k's packed results travel to rank 0 (RCCL, its own stream)
    # while frame k+1 is traced; a buffer is refilled only after its previous gather completed
    packed = [torch.empty((frame.PACKED_ROWS, n), dtype=torch.float32, device=dev) for _ in range(2)]
    gather_lists = [[torch.empty_like(packed[0]) for _ in range(world)] if (world > 1 and rank == 0) else None
                    for _ in range(2)]
    pending = [None, None]
    frames = [0]

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        bzr_amd.trace_chain(ctx, meshes, ris, rays, out_rays, out_status, out_seg, mode=mode)
        if ev is not None:
            ev[1].record(stream)
        if world > 1 and a.gather == "step":
            slot = frames[0] % 2
            if pending[slot] is not None:
                pending[slot].wait()
            frame.pack(out_rays, out_status, out_seg, packed[slot])
            pending[slot] = frame.gather(packed[slot], world, rank, gather_list=gather_lists[slot], async_op=True)
        frames[0] += 1

    def drain():
        for k in range(2):
            if pending[k] is not None:
                pending[k].wait()
                pending[k] = None

    for _ in range(a.warmup):
        step()
    drain()
    torch.cuda.synchronize()
    # work counters of one frame (device-side; measured here, outside the timed region)
    ctx.counters(True)
    ctx.counters_report()
    step()
    drain()
    work_cnt = ctx.counters_report()
    ctx.counters(False)
    seg_local = int(out_seg.sum().item())
    seg_total = torch.tensor([seg_local], dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(seg_total)
    seg_total = int(seg_total.item())

    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(a.steps):
        step(events[k])
    drain()  # the last frames' gathers complete inside the timed region
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    chain_ms = float(np.mean([s.elapsed_time(e) for s, e in events]))
    # per-kernel HIP-event timing on the kernels' stream, in a separate untimed pass of the same
    # K steps (the per-launch events would otherwise sit inside the timed region)
    ctx.timing(True)
    ctx.timing_report()  # reset
    for k in range(a.steps):
        step()
    drain()
    kernels = ctx.timing_report()
    ctx.timing(False)
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t[0])

    if rank == 0:
        ms_per_step = elapsed / a.steps * 1e3
        value = seg_total * a.steps / elapsed / 1e6
        base, cnt = (None, None)
        if a.cpu_baseline == "on" and world == 1:
            base, cnt = cpu_baseline(cfg, side, patches, ris, a.cpu_sample_stride)
        # measured on the GPU (bzr_ctx_counters, rank 0's frame); the brute-force-equivalent planar
        # test count per segment is N_b (every patch), as SURVEY.md 8d prices it
        segs = max(work_cnt["segments"], 1)
        newton_per_seg = work_cnt["pairs"] / segs
        follow_per_seg = work_cnt["follows"] / segs
        tests_per_seg = float(n_patch) / len(patches)
        if cnt and cnt["segments"]:  # cross-check with the oracle's counts on its sample
            oracle_rates = {"newton": cnt["newton"] / cnt["segments"], "follow": cnt["follow"] / cnt["segments"]}
        else:
            oracle_rates = None
        # algorithmic work per step on rank 0: F_seg = 33 N_b + 1750 (N_cand + N_follow)
        seg_r0 = seg_local
        work = {
            "k_traverse": (seg_r0 * FLOPS_PLANAR * tests_per_seg,
                           "brute-force-equivalent planar tests 33 N_b per segment (culling skips most of them)"),
            "k_newton": (seg_r0 * FLOPS_NEWTON * newton_per_seg, "Newton stage 1750 flops per candidate pair"),
            "k_follow": (seg_r0 * FLOPS_NEWTON * follow_per_seg,
                         "k_resolve: Newton stage 1750 flops per follow-side retry (+ overflow rays' full scans)"),
            "k_finish": (seg_r0 * FLOPS_REFRACT, "Snell step 30 flops per segment"),
        }
        all_flops = sum(f for f, _ in work.values())
        # the Newton stage runs as k_newton (patch-uniform chunks) + k_newton_lane (fragmented chunks):
        # priced and reported together, every Newton pair once
        if "k_newton_lane" in kernels and "k_newton" in kernels:
            (m1, c1), (m2, c2) = kernels.pop("k_newton"), kernels.pop("k_newton_lane")
            kernels["k_newton+k_newton_lane"] = (m1 + m2, c1)
            work["k_newton+k_newton_lane"] = (work.pop("k_newton")[0],
                                              "Newton stage 1750 flops per candidate pair (both kernels)")
        per_kernel = {}
        for name, (ms, calls) in kernels.items():
            per_step = ms / a.steps
            fl, what = work.get(name, (all_flops, "brute-force segment work F_seg"))
            if name in ("bucket", "k_overflow"):
                fl, what = 0.0, "bookkeeping (prefix sum + scatter) / overflow rays' full scan"
            per_kernel[name] = {"ms_per_step": round(per_step, 4), "launches_per_step": calls / a.steps,
                                "avg_launch_ms": round(ms / calls, 4),
                                "alg_tflops": round(fl / (per_step * 1e-3) / 1e12, 3), "work": what}
        # roofline kernel: the arithmetic stage (Newton), whose algorithmic flops are well defined.  The
        # longer-running k_traverse is priced brute-force-equivalent, which culling
        # beats by >1x, so its fraction says nothing about the kernel's efficiency.
        dom_time = max(per_kernel, key=lambda k: per_kernel[k]["ms_per_step"])
        dom = "k_newton+k_newton_lane" if "k_newton+k_newton_lane" in per_kernel else dom_time
        d = per_kernel[dom]
        achieved = d["alg_tflops"]
        alg_bytes = n * BYTES_PER_PRIMARY
        traffic, traffic_src = pmc_traffic(dom, cfg.name, side == cfg.side and world == 1 and a.mode == "parity")
        line = {
            "metric": "Mrays/sec (primary+refracted) at 1/2/4/8 MI355X; % of HBM-read roofline",
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (deterministic ray grid; lens built by the reference's preprocessing recipe)",
            "config": {
                "workload": f"{cfg.name}: {cfg.note}",
                "rays_per_gpu_side": side,
                "primaries_per_gpu": n,
                "segments_per_step": seg_total,
                "patches": n_patch,
                "parallelism": f"image tiles x{world}" + (", RCCL gather of every frame to rank 0 (overlapped with the next frame)"
                                                          if world > 1 and a.gather == "step" else ""),
                "scan": "BVH-culled (bit-identical to brute force)" if a.accel == "bvh" else "brute force",
                "numerics": "parity: bit-identical to the CPU oracle" if a.mode == "parity" else
                            "fast: exact planar gate, Newton stage with FMA + approximate div/sqrt (SURVEY 8c fast gates)",
                "preprocess_s": round(prep_s, 3),
                "upload_and_bvh_s": round(upload_s, 3),
            },
            "roofline": {
                "bound": "valu",
                "kernel": dom,
                "longest_kernel": dom_time,
                "achieved": achieved,
                "peak": VALU_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(achieved / VALU_PEAK_TFLOPS, 4),
                "traffic": traffic,
                "traffic_unit": "HBM bytes per launch",
                "traffic_source": traffic_src,
                "avg_launch_ms": d["avg_launch_ms"],
                "work": d["work"],
                "per_kernel": per_kernel,
                "chain_ms_hip_events": round(chain_ms, 4),
                "hbm_alg_bytes_per_step": alg_bytes,
                "hbm_achieved_GBps": round(alg_bytes / (chain_ms * 1e-3) / 1e9, 3),
                "hbm_frac": round(alg_bytes / (chain_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 6),
                "work_per_segment": {"planar_tests": round(tests_per_seg, 2), "newton": round(newton_per_seg, 4),
                                     "follow": round(follow_per_seg, 4),
                                     "overflow_rays_per_frame": work_cnt["overflow_rays"],
                                     "source": "GPU counters (bzr_ctx_counters)",
                                     "oracle_sample_rates": oracle_rates},
            },
            "cpu_baseline": base,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
