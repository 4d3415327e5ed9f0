#!/usr/bin/env python3
"""Throughput benchmark: Mrays/s (primary + refracted) of the Bezier-lens refraction chain.

Workload (default, BASELINE.json north_star / configs[3]): two stacked
makeEllipsoid(32,16,(1,4,2)) lenses at x=10 and x=13, refractive index 1.3 each, 4096x4096 primary rays
along +x from the plane x=0 over y in [-4.2,4.2], z in [-2.1,2.1]; per lens refract(INSIDE) then
refract(OUTSIDE), a miss ends the ray (reference/test.cpp:376-401).  "Rays" counts every
BezierMesh::intersect call (primary + refracted segments).  --config cfg2 (one lens, 1024^2), cfg3 and
cfg5 (BezierMesh::intersect configs) are available for A/B; the driver's line is cfg4.

A step = one frame: the whole chain over this rank's primary rays, inputs already resident in HBM,
results bit-identical to the reference restatement (tests/test_gpu_parity.py).  N GPUs = N processes
(torch.distributed over RCCL).  --scaling strong (default): the fixed side x side image is dealt to the
ranks as 64x64 tiles round-robin (the north-star's 1->8 GPU scaling on a fixed 4096^2 grid); --scaling
weak: the image grows to side x (side*N).  Each frame's results are gathered to rank 0 over RCCL inside
the timed region, double-buffered so frame k's gather overlaps frame k+1's tracing (bzr_amd/frame.py layouts):
--gather image (the default, "auto") the frame's result image on rank 0: the per-primary status + segment-count
word (4 B per primary; for the intersect configs the hit's `what` row), the final rays / hits staying in each
rank's HBM -- at N = 8 on cfg4 ~0.12 ms of xGMI per frame against a 0.58 ms rank frame (DESIGN.md (e) byte
budget), so the gather never bounds the strong-scaling line; --gather compact every final ray on rank 0 in
~17.6 B per primary (a status/segment byte per primary plus the final rays of the primaries that refracted;
rank 0 regenerates the others from their pixels), ~0.49-0.58 ms per frame at N = 8, i.e. as long as the frame
itself; --gather rays the 6 final-ray floats + the word (28 B per primary; longer than the N = 8 frame);
--gather none nothing (tracing alone).  The line reports gather_only_ms_per_frame and its ratio to ms_per_step.

--gpus N: N ranks, one process per GPU.  Run bare (no WORLD_SIZE in the environment) with N > 1, bench.py
starts the N rank processes itself (bzr_amd/launch.py: children with RANK / LOCAL_RANK / WORLD_SIZE and a
127.0.0.1 rendezvous; the parent touches no GPU and exits with the ranks' status).  Under an external
launcher (torch.distributed.run) WORLD_SIZE must equal N, else bench.py exits with status 2.  The line
reports the process group's own world size, the RCCL version and each rank's tile count.
--inflight F (default: 6 for a rank frame of at most 4 M primaries, else 3 for the fused pipeline and 2 for the
staged one): frame k runs on slot k % F (its own context, stream and output buffers), so the next frames' waves
fill the GPU while a frame's slowest waves finish; every frame is traced in full.

Prints ONE JSON line on rank 0; fields are described in DESIGN.md (d).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

import numpy as np

# Frames in flight (--inflight) need their slot streams on distinct hardware queues.  HIP shares its
# GPU_MAX_HW_QUEUES (default 4) queues among all streams of the process, and which streams end up sharing
# depends on the creation / first-use order (torch's pool, the contexts' own streams, RCCL's): with 4, a
# probe that created its streams in another order saw two slots land on one queue and lose the overlap
# entirely.  16 queues give every stream here its own.  Set before HIP initialises (torch is imported
# in main()).  set_hw_queues() keeps a caller's value that is large enough (or any value given through
# BZR_BENCH_HW_QUEUES) and reports the effective one in config.hw_queues.
HWQ_WANT = 16
HWQ_MAX = 32  # the GPU pool refuses a GPU_MAX_HW_QUEUES above 32


def set_hw_queues(frames_in_flight: int, world: int) -> str:
    """GPU_MAX_HW_QUEUES for this run (before HIP initialises): the slots need distinct queues, and HIP's
    default of 4 (which the GPU pool exports) let two slots share one in a probe.  Capped at HWQ_MAX (a
    larger --inflight then warns).  Returns the source.  The value is what this process *requested*: under a
    profiler that preloads HIP (rocprofv3) the runtime has read the variable before this runs."""
    explicit = os.environ.get("BZR_BENCH_HW_QUEUES")
    if explicit:
        if explicit.isdigit() and int(explicit) > HWQ_MAX:
            print(f"bench.py: warning: BZR_BENCH_HW_QUEUES={explicit} capped at {HWQ_MAX}", file=sys.stderr, flush=True)
            explicit = str(HWQ_MAX)
        os.environ["GPU_MAX_HW_QUEUES"] = explicit
        return "BZR_BENCH_HW_QUEUES"
    have = os.environ.get("GPU_MAX_HW_QUEUES", "")
    need = max(HWQ_WANT, frames_in_flight + (1 if world > 1 else 0))
    if need > HWQ_MAX:
        print(f"bench.py: warning: {frames_in_flight} frames in flight want {need} hardware queues; capped at "
              f"{HWQ_MAX}, so some frame slots will share a queue", file=sys.stderr, flush=True)
        need = HWQ_MAX
    if have.isdigit() and int(have) >= need:
        return "caller"
    os.environ["GPU_MAX_HW_QUEUES"] = str(need)
    return f"bench.py (raised from {have or 'unset'}: the frame slots need their own queues)"

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "cuda-bezier-triangle-raytracer_amd"))
sys.path.insert(0, str(REPO))

VALU_PEAK_TFLOPS = 157.3      # MI355X FP32 vector peak (MI355X_MICROARCH.md, chip parameters)
PEAK_CLOCK_GHZ = 2.4          # the clock the peaks above are quoted at
SIMDS, CUS = 1024, 256        # 256 CUs x 4 SIMDs
VALU_ISSUE_PEAK = SIMDS * PEAK_CLOCK_GHZ / 2.0  # G wave64 VALU instructions/s (one per 2 cycles per SIMD)
SALU_ISSUE_PEAK = CUS * PEAK_CLOCK_GHZ          # G scalar instructions/s (one scalar unit per CU)
HBM_PEAK_GBS = 8000.0         # MI355X HBM3E peak (spec)
FLOPS_PLANAR = 33.0           # algorithmic flops per (segment, patch) planar gate
FLOPS_NEWTON = 1750.0         # algorithmic flops per Newton run: bracket + 4 iterations + tail
FLOPS_REFRACT = 30.0          # Snell step per segment
BYTES_CHAIN = 24 + 32         # per primary: ray in; ray + status + segment count out
BYTES_INTERSECT = 24 + 52     # per ray: ray in; BezierIntersection (13 words) out


SMALL_FRAME_RAYS = 1 << 22   # a rank's frame at or below this many primaries gets SMALL_FRAME_INFLIGHT slots
SMALL_FRAME_INFLIGHT = 6


def default_inflight(a, world: int) -> int:
    """--inflight 0: frames in flight from the rank's frame size and the pipeline.  Small frames
    (cfg2 1024², cfg3 2048², the strong-scaling shares of cfg4 from N = 4) end in short kernels and tails that
    further frames fill: 6 slots measured +3 % on cfg2 fused and +8 % on cfg3 staged against 3 / 2, and the same
    on cfg4's N = 4 and N = 8 shares (`profiles/r06_inflight_sweep.jsonl`).  Large frames keep 3 (fused) / 2
    (staged): cfg4 4096² measures the same at 3 and 6, and the staged pipeline's multi-chunk frames contend
    beyond two (cfg5 2 against 3, 4, 6)."""
    from bzr_amd.configs import CONFIGS
    side = a.side or CONFIGS[a.config].side
    rays = side * side if a.scaling == "weak" else side * side // max(world, 1)
    if rays <= SMALL_FRAME_RAYS:
        return SMALL_FRAME_INFLIGHT
    return 3 if (a.accel == "bvh" and a.pipeline == "fused") else 2


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--prewarm-s", type=float, default=4.0,
                   help="seconds of back-to-back frames before the warmup steps (clock ramp), 0 = off")
    p.add_argument("--config", default="cfg4", choices=["cfg2", "cfg3", "cfg4", "cfg5"])
    p.add_argument("--side", type=int, default=0, help="override rays per image side")
    p.add_argument("--scaling", default="strong", choices=["strong", "weak"])
    p.add_argument("--gather", default="auto", choices=["auto", "image", "rays", "compact", "none"],
                   help="what each frame sends to rank 0 when N > 1 (frame.py layouts, DESIGN.md (e) byte budget); "
                        "auto = image (the result image, 4 B per primary: its gather stays under a fifth of the "
                        "N = 8 frame); compact = every final ray on rank 0 (~17.6 B per primary, as long as the "
                        "N = 8 frame)")
    p.add_argument("--accel", default="bvh", choices=["bvh", "none"], help="none = brute-force scan (A/B)")
    p.add_argument("--pipeline", default="fused", choices=["fused", "staged", "auto"],
                   help="culled-path pipeline (include/bzr.h BZR_PIPELINE_*; same output bits): fused = one k_trace "
                        "kernel per frame (default), staged = the multi-kernel path, auto = the library's choice")
    p.add_argument("--inflight", type=int, default=0,
                   help="frames in flight (each on its own context, stream and output buffers); "
                        "0 = 6 for a rank frame of at most 4 M primaries, else 3 for the fused pipeline and 2 "
                        "for the staged one (scripts/inflight_sweep.sh)")
    p.add_argument("--mode", default="parity", choices=["parity", "fast"],
                   help="fast = BZR_MODE_FAST Newton stage (contracted FMA, approximate div/sqrt; not bit-exact)")
    p.add_argument("--cpu-baseline", default="on", choices=["on", "off"])
    p.add_argument("--cpu-sample-stride", type=int, default=0,
                   help="oracle sample: every k-th row and column (0 = per-config default)")
    p.add_argument("--cpu-runs", type=int, default=5)
    return p.parse_args()


def cpu_model() -> str:
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.lower().startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads() -> tuple[int, str]:
    """Host threads for the CPU baseline: every CPU this process may run on, capped by OMP_NUM_THREADS
    when the environment sets it (the GPU pool allots a fixed CPU share per GPU and says so there)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and 0 < int(env) < aff:
        return int(env), f"OMP_NUM_THREADS={env} (the host's CPU share for this process; affinity {aff})"
    return aff, f"all {aff} CPUs in this process's affinity mask"


def cpu_baseline(cfg, side, patches, ris, stride, runs):
    """The oracle (CPU restatement, test infrastructure) on a strided sample of the same workload, timed as
    BASELINE.md 2 prescribes: OpenMP over the host's threads, -O2 (reference/CMakeLists.txt:8) and
    -O3 -march=native builds, median of `runs` runs each.  Returns the line plus the oracle's work counters."""
    from bzr_amd.configs import pixel_coords, rays_for
    from oracle import pyoracle

    r, c = pixel_coords(cfg, side=side, order="rows")
    keep = (r % stride == 0) & (c % stride == 0)
    rays = rays_for(cfg, r[keep], c[keep], side=side)
    threads, why = cpu_threads()
    builds = {"-O2": pyoracle.lib()}
    try:
        builds["-O3 -march=native"] = pyoracle.load_variant("-O3 -march=native", "native")
    except Exception as e:  # noqa: BLE001 -- reported, the -O2 number still stands
        builds["-O3 -march=native"] = None
        native_err = str(e)[:200]
    results, cnt = {}, None
    for flags, L in builds.items():
        if L is None:
            results[flags] = {"error": native_err}
            continue
        times, segs = [], 0
        for k in range(runs):
            if flags == "-O2" and k == 0:
                pyoracle.counters_reset()
            t0 = time.perf_counter()
            if cfg.op == "chain":
                _, _, seg = pyoracle.trace_chain(patches, ris, rays, threads=threads, L=L)
                segs = int(seg.sum())
            else:
                pyoracle.intersect(patches[0], rays, threads=threads, L=L)
                segs = rays.shape[1]
            times.append(time.perf_counter() - t0)
            if flags == "-O2" and k == 0:
                cnt = pyoracle.counters()
        med = statistics.median(times)
        results[flags] = {"median_s": round(med, 4), "runs_s": [round(t, 4) for t in times],
                          "mrays_per_s": round(segs / med / 1e6, 4)}
    frac = rays.shape[1] / float(side * side)
    line = {
        "value": results["-O2"]["mrays_per_s"],
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "nproc": os.cpu_count(),
        "threads_reason": why,
        "cpu_model": cpu_model(),
        "builds": results,
        "sample": f"{rays.shape[1]} primaries = every {stride}th row and column of the {side}^2 grid "
                  f"(fraction {frac:.5f}); oracle/bzr_oracle.c (CPU restatement of the reference hot path), "
                  f"OpenMP schedule(dynamic) over {threads} threads; value = -O2 median of {runs} runs",
    }
    return line, cnt


def pmc_issue(kernel, workload):
    """Issue counts per launch of `kernel` (SQ_INSTS_VALU / _SALU / _SMEM, SQ_WAVES) from the committed PMC
    profile of this workload (profiles/pmc_traffic.json), or None."""
    path = REPO / "profiles" / "pmc_traffic.json"
    if not path.exists():
        return None
    d = json.loads(path.read_text()).get("workloads", {}).get(workload)
    k = d and d["kernels"].get(kernel)
    if not k or "valu_insts" not in k:
        return None
    return dict(k, source=d["source"])


def pmc_traffic(kernel, workload):
    """HBM bytes per launch of `kernel` from the committed PMC profile of this workload
    (profiles/pmc_traffic.json, written by scripts/prof_summary.py from rocprofv3 FETCH_SIZE (x2, gfx950
    correction) and WRITE_SIZE passes over bench.py).  PMC counters cannot be read inside the timed process."""
    path = REPO / "profiles" / "pmc_traffic.json"
    if not path.exists():
        return None, None
    d = json.loads(path.read_text()).get("workloads", {}).get(workload)
    if not d:
        return None, None
    parts = kernel.split("+")
    if not all(p in d["kernels"] for p in parts):
        return None, None
    total = sum(d["kernels"][p].get("read", 0.0) + d["kernels"][p].get("write", 0.0) for p in parts)
    return round(total), f"{d['source']} ({d['method']})"


GOLDEN = REPO / "tests" / "golden"


def oracle_digests(cfg, side, rays_img, status_img, seg_img):
    """The whole frame (row-major full-image arrays) against the committed oracle digests of this workload
    (tests/golden/d_<cfg>_<side>.npz: one SHA-256 per 64x64 tile, made by tests/golden/make_digests.py from the
    CPU oracle -- data, not the oracle).  None when no digests exist for it."""
    import importlib.util

    path = GOLDEN / f"d_{cfg.name}_{side}.npz"
    if not path.exists() or cfg.op != "chain":
        return None
    spec = importlib.util.spec_from_file_location("tile_digest", GOLDEN / "tile_digest.py")
    td = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(td)
    g = np.load(path)
    rows, cols = td.tile_pixels(cfg, side, g["tiles"])
    flat = rows * side + cols
    got = td.chain_digests(rays_img[:, flat], status_img[flat], seg_img[flat])
    match = int((got == g["digests"]).all(axis=1).sum())
    return {"tiles_matching": match, "tiles": int(len(g["tiles"])), "ok": match == len(g["tiles"]),
            "source": str(path.relative_to(REPO))}


def verify_frame(a, cfg, chain, world, rank, side, height, ctx, meshes, ris, mode, dev, gather, loop, last, own_out, cap):
    """Untimed checks of what the timed frames delivered.  Returns {"gather": {...} (N > 1), "frame": {...}}.
    N > 1: rank 0 traces the whole image itself and compares the last gathered frame with it bit for bit
    (frame.verify_gathered), then that frame with the oracle digests; all ranks time the gather alone.
    N = 1: the last frame's own outputs against the oracle digests."""
    import torch
    import torch.distributed as dist

    from bzr_amd import frame
    import bzr_amd

    out = {"gather": {}, "frame": None}
    total = side * height
    host_bytes = total * (32 if chain else 52) * 3  # reference image + assembled image + temporaries
    if rank == 0:
        if host_bytes > 6e9:
            msg = f"skipped: {total} pixels ({host_bytes / 1e9:.0f} GB of host arrays)"
            out["frame"] = {"skipped": msg}
            if gather:
                out["gather"]["gather_verified"] = None
                out["gather"]["gather_verify"] = {"skipped": msg}
        elif world == 1:
            if chain:
                rows, cols, _ = frame.rank_rays(cfg, 0, 1, side, height)
                flat = rows * side + cols
                r, s_, g_ = (t.cpu().numpy() for t in own_out)
                img = np.zeros((6, total), np.float32), np.zeros(total, np.uint32), np.zeros(total, np.uint32)
                img[0][:, flat], img[1][flat], img[2][flat] = r, s_.view(np.uint32), g_.view(np.uint32)
                out["frame"] = {"oracle_digests": oracle_digests(cfg, side, *img), "what": "the last timed frame"}
        else:
            rows, cols, rays_all = frame.rank_rays(cfg, 0, 1, side, height)  # every tile, in one process
            flat = rows * side + cols
            rt = torch.from_numpy(rays_all).to(dev)
            m = rays_all.shape[1]
            if chain:
                o = (torch.empty((6, m), dtype=torch.float32, device=dev), torch.empty(m, dtype=torch.int32, device=dev),
                     torch.empty(m, dtype=torch.int32, device=dev))
                bzr_amd.trace_chain(ctx, meshes, ris, rt, *o, mode=mode)
                torch.cuda.synchronize()
                want = {"rays": np.zeros((6, total), np.float32), "status": np.zeros(total, np.uint32),
                        "segments": np.zeros(total, np.uint32)}
                want["rays"][:, flat] = o[0].cpu().numpy()
                want["status"][flat] = o[1].cpu().numpy().view(np.uint32)
                want["segments"][flat] = o[2].cpu().numpy().view(np.uint32)
            else:
                h = torch.empty((13, m), dtype=torch.float32, device=dev)
                bzr_amd.intersect(ctx, meshes[0], rt, h, mode=mode)
                torch.cuda.synchronize()
                want = {"hits": np.zeros((13, total), np.float32)}
                want["hits"][:, flat] = h.cpu().numpy()
            del rt
            if gather and "parts" in last:
                res = frame.verify_gathered(last["parts"], a.gather, cfg, world, side, height, want, cap=cap)
                out["gather"]["gather_verified"] = res["ok"]
                out["gather"]["gather_verify"] = dict(res, frame_index=last["frame"],
                                                      against="the same frame traced by rank 0 in one process")
            if chain:
                out["frame"] = {"oracle_digests": oracle_digests(cfg, side, want["rays"], want["status"], want["segments"]),
                                "what": "rank 0's single-process trace of the whole image (the gathered frame's reference)"}
    if gather:  # the gather alone: K gathers of the packed buffers back to back (no tracing), max over ranks
        kk = max(5, min(a.steps, 20))
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(kk):
            w = frame.gather(loop.packed[k % 2], world, rank, gather_list=loop.lists[k % 2], async_op=True)
            w.wait()
        torch.cuda.synchronize()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        out["gather"]["gather_only_ms_per_frame"] = round(float(t[0]) / kk * 1e3, 4)
        out["gather"]["gather_only_frames"] = kk
    return out


def main():
    a = parse()
    from bzr_amd import launch  # no torch, no HIP: safe in the launching parent

    if launch.check_world(a.gpus) == "spawn":  # bare `bench.py --gpus N`: start the N rank processes here
        raise SystemExit(launch.spawn([sys.executable, str(Path(__file__).resolve())] + sys.argv[1:], a.gpus))
    if a.inflight <= 0:
        a.inflight = default_inflight(a, int(os.environ.get("WORLD_SIZE", str(a.gpus))))
    hwq_source = set_hw_queues(a.inflight, int(os.environ.get("WORLD_SIZE", "1")))
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
    chain = cfg.op == "chain"
    if a.gather == "auto":  # the frame's result image on rank 0 (the gather that keeps N = 8 margin)
        a.gather = "image"
    side = a.side or cfg.side
    height = side * world if a.scaling == "weak" else side
    t0 = time.perf_counter()
    patches = [build_lens(bzr_amd.TriMesh, lens).bezier_patches() for lens in cfg.lenses]
    ris = [lens.ri for lens in cfg.lenses]
    prep_s = time.perf_counter() - t0
    n_patch = sum(len(p) for p in patches)

    ctx = bzr_amd.Context(local)
    t0 = time.perf_counter()
    meshes = [bzr_amd.DeviceMesh(ctx, p) for p in patches]  # upload + BVH build
    upload_s = time.perf_counter() - t0
    # one stream per frame slot (--inflight); GPU_MAX_HW_QUEUES (top of this file) gives each its own
    # hardware queue, so the slots' frames overlap
    # BZR_BENCH_SLOT_PRIO (A/B knob, default off): "lead" puts slot 0's stream at the device's highest stream
    # priority, so the other slots' frames fill the tails of slot 0's kernels instead of contending with them
    slot_prio = os.environ.get("BZR_BENCH_SLOT_PRIO", "")
    top_prio = torch.cuda.Stream.priority_range()[1] if slot_prio == "lead" else 0
    streams = [torch.cuda.Stream(dev, priority=top_prio if i == 0 else 0) for i in range(max(1, a.inflight))]
    hwq = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    if hwq < len(streams) + (1 if world > 1 else 0) and rank == 0:
        print(f"bench.py: warning: GPU_MAX_HW_QUEUES={hwq} < {len(streams)} frame streams"
              f"{' + the RCCL stream' if world > 1 else ''}: slots may share a hardware queue and lose the overlap",
              file=sys.stderr, flush=True)
    stream = streams[0]  # slot 0: the kernels, torch ops and the timing events
    torch.cuda.set_stream(stream)
    ctx.use_torch_stream(stream)
    mode = bzr_amd.ACCEL_NONE if a.accel == "none" else bzr_amd.MODE_PARITY
    if a.mode == "fast":
        mode |= bzr_amd.MODE_FAST
    if a.accel == "bvh":
        mode |= {"fused": bzr_amd.PIPELINE_FUSED, "staged": bzr_amd.PIPELINE_STAGED, "auto": 0}[a.pipeline]

    _, _, rays_np = frame.rank_rays(cfg, rank, world, side, height)
    n = rays_np.shape[1]
    # what actually runs: the process group's own size and every rank's share, as each rank counted it
    pg_world = dist.get_world_size() if world > 1 else 1
    if pg_world != a.gpus:
        raise SystemExit(f"bench.py: process group has {pg_world} ranks, --gpus {a.gpus}")
    shares = torch.tensor([n // (frame.TILE * frame.TILE)], dtype=torch.int64,
                          device=dev if (world > 1 and dist.get_backend() == "nccl") else "cpu")
    if world > 1:
        parts = [torch.zeros_like(shares) for _ in range(world)]
        dist.all_gather(parts, shares)
        tiles_per_rank = [int(p.item()) for p in parts]
    else:
        tiles_per_rank = [int(shares.item())]
    rccl = None
    if world > 1 and dist.get_backend() == "nccl":
        v = torch.cuda.nccl.version()
        rccl = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    rays = torch.from_numpy(rays_np).to(dev)
    # Frames in flight: frame k runs on slot k % F -- its own context, stream and output buffers -- so the
    # next frame's waves fill the GPU while this frame's slowest waves finish (a frame's last waves run
    # up to ~6x the median wave; with one frame in flight their tail idles most of the chip).
    F = max(1, a.inflight)
    ctxs = [ctx] + [bzr_amd.Context(local) for _ in range(F - 1)]
    for c, st in zip(ctxs[1:], streams[1:]):
        c.use_torch_stream(st)
    if chain:
        outs = [(torch.empty((6, n), dtype=torch.float32, device=dev), torch.empty(n, dtype=torch.int32, device=dev),
                 torch.empty(n, dtype=torch.int32, device=dev)) for _ in range(F)]
        out_rays, out_status, out_seg = outs[0]
    else:
        outs = [torch.empty((13, n), dtype=torch.float32, device=dev) for _ in range(F)]
        hits = outs[0]
    gather = world > 1 and a.gather != "none"
    npad = frame.padded_count(world, side, height)

    def trace(f, k):  # frame k on slot f: its context, stream (the loop's stream_for) and outputs
        if chain:
            bzr_amd.trace_chain(ctxs[f], meshes, ris, rays, *outs[f], mode=mode)
        else:
            bzr_amd.intersect(ctxs[f], meshes[0], rays, outs[f], mode=mode)

    # work counters of one frame (device-side; measured here, outside the timed region)
    ctx.counters(True)
    ctx.counters_report()
    with torch.cuda.stream(streams[0]):
        trace(0, 0)
    torch.cuda.synchronize()
    work_cnt = ctx.counters_report()
    ctx.counters(False)
    seg_local = int(out_seg.sum().item()) if chain else n
    seg_total = torch.tensor([seg_local], dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(seg_total)
    seg_total = int(seg_total.item())
    # compact gather (frame.py): survivor capacity from this frame's largest rank share
    cap = 0
    if a.gather == "compact":
        if not chain:
            raise SystemExit("--gather compact applies to the refraction-chain configs (cfg2, cfg4)")
        cnt = frame.survivors(out_status, out_seg).sum().reshape(1).to(torch.int64)
        if world > 1:
            dist.all_reduce(cnt, op=dist.ReduceOp.MAX)
        cap = frame.compact_capacity(int(cnt.item()), npad)
    # The frame loop (frame.FrameLoop): frames in flight, and with N > 1 a double-buffered asynchronous gather
    # -- frame k's packed results travel to rank 0 (RCCL, its own stream) while frame k+1 is traced; a
    # buffer is refilled only after its previous gather completed.  Buffers hold the largest rank's share
    # (strong scaling may deal one tile fewer to some ranks).  Layouts: rays (chain: 6 ray rows + the
    # status/segment word; intersect: the 13 hit rows), compact (every final ray, survivors only), image
    # (one word per primary; intersect: the hit's `what` row).
    # chain frames are packed on the device by bzr_pack_frame (one kernel; three for compact) on the slot's context
    if chain:
        pack_fn = lambda out, p, f: bzr_amd.pack_frame(ctxs[f], a.gather, *out, p, npad, cap)  # noqa: E731
    else:
        pack_fn = ((lambda out, p, f: p[0, :n].copy_(out[11])) if a.gather == "image" else
                   (lambda out, p, f: p[:, :n].copy_(out)))
    last_gathered = {}  # rank 0: the latest frame's gathered parts (kept by reference; checked after the timed region)
    loop = frame.FrameLoop(world, rank, n, npad, a.gather, trace, outs, stream_for=lambda f: torch.cuda.stream(streams[f]),
                           cap=cap, device=dev, pack_fn=pack_fn, rows=0 if chain else 13,
                           on_gathered=lambda k, parts: last_gathered.update(frame=k, parts=parts))

    def step(inflight=F):
        loop.step(inflight)

    def join_streams():  # stream 0 waits for the other slots' queued frames
        for st in streams[1:]:
            ev = torch.cuda.Event()
            ev.record(st)
            streams[0].wait_event(ev)

    drain = loop.drain

    # time-based pre-warm (--prewarm-s): frames until the GPU has run back to back that long, so the timed
    # steps start at the clock the chip holds under this load (scripts/sustained_clock.py: the first
    # ~0.2 s of frames run ~3 % slower); then the W warmup steps, right before the timed ones (no host
    # round trip in between)
    # (tracing only: no gather, so ranks may run different frame counts without a collective mismatch)
    if a.prewarm_s > 0:
        t_pw, k_pw = time.perf_counter(), 0
        while True:
            for _ in range(8):
                with torch.cuda.stream(streams[k_pw % F]):
                    trace(k_pw % F, k_pw)
                k_pw += 1
            torch.cuda.synchronize()
            if time.perf_counter() - t_pw >= a.prewarm_s:
                break
        if world > 1:
            dist.barrier()
    for _ in range(a.warmup):
        step()
    drain()

    # one HIP event pair around the K steps (no timing markers between the frames)
    events = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    events[0].record(stream)
    for st in streams[1:]:
        st.wait_event(events[0])
    for k in range(a.steps):
        step()
    join_streams()
    events[1].record(stream)
    drain()  # the last frames' gathers complete inside the timed region
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    chain_ms = events[0].elapsed_time(events[1]) / a.steps
    last_slot = (loop.frames - 1) % F  # the slot of the last timed frame (its outputs are still in place)
    # What the timed frames delivered (untimed): rank 0 checks the last gathered frame
    # against the same frame traced in one process, and (cfg4 4096^2) that frame against the committed oracle
    # digests; at N = 1 the last frame's own outputs against the digests.  Then the gather alone, timed.
    verify = verify_frame(a, cfg, chain, world, rank, side, height, ctx, meshes, ris, mode, dev, gather, loop,
                          last_gathered, outs[last_slot], cap)
    # per-kernel HIP-event timing on the kernels' stream, in a separate untimed pass of the same
    # K steps (the per-launch events would otherwise sit inside the timed region)
    ctx.timing(True)
    ctx.timing_report()  # reset
    for k in range(a.steps):
        step(inflight=1)  # slot 0's context only: kernel durations without a neighbouring frame
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
            stride = a.cpu_sample_stride or {"cfg2": 4, "cfg3": 32, "cfg4": 8, "cfg5": 256}[cfg.name]
            base, cnt = cpu_baseline(cfg, side, patches, ris, stride, a.cpu_runs)
        segs = max(work_cnt["segments"], 1)
        # algorithmic work of one frame on rank 0, from the GPU's own counters (bzr_ctx_counters): every
        # planar gate the culled walk evaluated (33 flops), every Newton run (1750: cThis pairs + follow-side
        # retries) and the Snell step per segment (30).  SURVEY.md 8d's brute-force-equivalent count
        # (33 N_b per segment instead of the gates evaluated) is reported beside it, labelled as such.
        newton_runs = work_cnt["pairs"] + work_cnt["follows"]
        exec_flops = FLOPS_NEWTON * newton_runs + FLOPS_PLANAR * work_cnt["gate_tests"] + FLOPS_REFRACT * segs
        bf_flops = FLOPS_PLANAR * n_patch / len(patches) * segs + FLOPS_NEWTON * newton_runs + FLOPS_REFRACT * segs
        fused_kernel = "k_trace" in kernels
        if "k_newton_lane" in kernels and "k_newton" in kernels:
            (m1, c1), (m2, _) = kernels.pop("k_newton"), kernels.pop("k_newton_lane")
            kernels["k_newton+k_newton_lane"] = (m1 + m2, c1)
        work = {
            "k_trace": (exec_flops, "culled algorithmic flops: 1750 per Newton run + 33 per planar gate evaluated "
                                    "+ 30 per segment (GPU counters)"),
            "k_newton+k_newton_lane": (FLOPS_NEWTON * work_cnt["pairs"], "Newton stage 1750 flops per candidate pair"),
            "k_follow": (FLOPS_NEWTON * work_cnt["follows"], "follow-side retries, 1750 flops each"),
            "k_finish": (FLOPS_REFRACT * segs, "Snell step 30 flops per segment"),
        }
        per_kernel = {}
        for name, (ms, calls) in kernels.items():
            per_step = ms / a.steps
            fl, what = work.get(name, (None, "no flop model (bookkeeping / traversal without counters)"))
            per_kernel[name] = {"ms_per_step": round(per_step, 4), "launches_per_step": calls / a.steps,
                                "avg_launch_ms": round(ms / calls, 4), "work": what,
                                "alg_tflops": None if fl is None else round(fl / (per_step * 1e-3) / 1e12, 3)}
        # roofline kernel: the one that runs longest per step
        dom = max(per_kernel, key=lambda k: per_kernel[k]["ms_per_step"])
        d = per_kernel[dom]
        achieved = d["alg_tflops"]
        alg_bytes = n * (BYTES_CHAIN if chain else BYTES_INTERSECT)
        workload_key = f"{cfg.name}/{a.pipeline}/{a.mode}/{side}"
        traffic, traffic_src = pmc_traffic(dom, workload_key) if world == 1 else (None, None)
        launches = d["launches_per_step"]
        roof = {"bound": "valu", "kernel": dom, "achieved": achieved, "peak": VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": None if achieved is None else round(achieved / VALU_PEAK_TFLOPS, 4)}
        iss = pmc_issue(dom, workload_key) if (achieved is None and world == 1) else None
        if iss is not None:
            # no flop model (the BVH walk: bookkeeping, slab tests, scalar loads): an issue roof instead --
            # the kernel's VALU and SALU instructions per launch (committed PMC) over its HIP-event launch
            # time, against one wave64 VALU instruction per 2 cycles per SIMD and one SALU instruction per
            # cycle per CU at the 2.4 GHz peak clock; the busier unit is the bound
            sec = d["avg_launch_ms"] * 1e-3
            v_rate, s_rate = iss["valu_insts"] / sec / 1e9, iss["salu_insts"] / sec / 1e9
            vf, sf = v_rate / VALU_ISSUE_PEAK, s_rate / SALU_ISSUE_PEAK
            roof = {"bound": "valu-issue" if vf >= sf else "salu-issue", "kernel": dom,
                    "achieved": round(v_rate if vf >= sf else s_rate, 3),
                    "peak": VALU_ISSUE_PEAK if vf >= sf else SALU_ISSUE_PEAK, "unit": "G instructions/s",
                    "frac": round(max(vf, sf), 4),
                    "issue": {"valu_frac": round(vf, 4), "salu_frac": round(sf, 4),
                              "valu_insts_per_launch": iss["valu_insts"], "salu_insts_per_launch": iss["salu_insts"],
                              "smem_insts_per_launch": iss.get("smem_insts"), "waves_per_launch": iss.get("waves"),
                              "source": iss["source"],
                              "node_visits_per_wave_segment": round(work_cnt["node_visits"] * 64 / segs, 3),
                              "leaf_fetches_per_wave_segment": round(work_cnt["leaf_fetches"] * 64 / segs, 3)}}
        # VALU issue over the frame interval with frames in flight: the committed PMC instruction count of
        # the dominant kernel per launch x launches per step, one wave64 VALU instruction per 2 cycles per
        # SIMD at the 2.4 GHz peak clock, over ms_per_step (the serialized per-launch view above idles
        # through each frame's tail; this is what the overlapped frames keep the SIMDs busy with)
        iss_all = pmc_issue(dom, workload_key) if world == 1 else None
        if iss_all is not None:
            roof["valu_issue_in_flight"] = {
                "frac": round(iss_all["valu_insts"] * launches * 2.0 / (SIMDS * PEAK_CLOCK_GHZ * 1e9 * ms_per_step * 1e-3), 4),
                "valu_insts_per_step": round(iss_all["valu_insts"] * launches), "source": iss_all["source"],
                "note": "VALU instructions per step (PMC) x 2 cycles / (1024 SIMDs x 2.4 GHz x ms_per_step)"}
        line = {
            "metric": "Mrays/sec (primary+refracted) at 1/2/4/8 MI355X; % of HBM-read roofline",
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": pg_world,
            "steps": a.steps,
            "warmup": a.warmup,
            "prewarm_s": a.prewarm_s,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": a.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (deterministic ray grid; lenses built by the reference's preprocessing recipe)",
            "config": {
                "workload": f"{cfg.name}: {cfg.note}" + (f" (side {side})" if side != cfg.side else ""),
                "image": f"{side}x{height}",
                "primaries_per_gpu": n,
                "ranks": {"world_size": pg_world, "backend": dist.get_backend() if world > 1 else None,
                          "rccl_version": rccl, "launcher": os.environ.get(launch.LAUNCHED_BY) or
                          ("external (WORLD_SIZE set)" if world > 1 else "single process"),
                          "tiles_per_rank": tiles_per_rank, "tile": f"{frame.TILE}x{frame.TILE}"},
                "segments_per_step": seg_total,
                "patches": n_patch,
                "parallelism": f"64x64 image tiles round-robin over {world} rank(s), {a.scaling} scaling"
                               + (f", RCCL gather of every frame to rank 0 (overlapped with the next frames): "
                                  f"{loop.bytes_per_rank / npad:.2f} B per primary ({a.gather})" if gather else ""),
                "gather": ({"layout": a.gather, "bytes_per_rank_per_frame": loop.bytes_per_rank,
                            "bytes_per_primary": round(loop.bytes_per_rank / npad, 3), "compact_capacity": cap or None,
                            **verify["gather"],
                            # the gather's rate against the frame's: below 1 it never stalls the tracing
                            "gather_only_over_ms_per_step": (round(verify["gather"]["gather_only_ms_per_frame"] / ms_per_step, 4)
                                                             if verify["gather"].get("gather_only_ms_per_frame") else None)}
                           if gather else None),
                "frame_verified": verify["frame"],
                "pipeline": a.pipeline,
                "frames_in_flight": F,
                **({"slot_priority": {"mode": slot_prio, "slot0": top_prio}} if slot_prio else {}),
                "hw_queues": {"GPU_MAX_HW_QUEUES_requested": hwq, "source": hwq_source,
                              "streams": len(streams) + (1 if gather else 0),
                              "ok": hwq >= len(streams) + (1 if gather else 0)},
                "scan": "BVH-culled (bit-identical to brute force)" if a.accel == "bvh" else "brute force",
                "numerics": "parity: bit-identical to the CPU oracle" if a.mode == "parity" else
                            "fast: exact planar gate, Newton stage with FMA + approximate div/sqrt (SURVEY 8c fast gates)",
                "preprocess_s": round(prep_s, 3),
                "upload_and_bvh_s": round(upload_s, 3),
            },
            "roofline": {
                **roof,
                "traffic": traffic,
                "traffic_unit": "HBM bytes per launch (PMC)",
                "traffic_source": traffic_src,
                "traffic_workload": workload_key,
                "avg_launch_ms": d["avg_launch_ms"],
                "work": d["work"],
                "alg_bytes_per_launch": round(alg_bytes / launches),
                "per_kernel": per_kernel,
                "chain_ms_hip_events": round(chain_ms, 4),
                "hbm_alg_bytes_per_step": alg_bytes,
                "hbm_achieved_GBps": round(alg_bytes / (chain_ms * 1e-3) / 1e9, 3),
                "hbm_frac": round(alg_bytes / (chain_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 6),
                "brute_force_equiv_tflops": round(bf_flops / (chain_ms * 1e-3) / 1e12, 3),
                "work_per_segment": {
                    "newton_pairs": round(work_cnt["pairs"] / segs, 4),
                    "follows": round(work_cnt["follows"] / segs, 4),
                    "gate_tests": round(work_cnt["gate_tests"] / segs, 4),
                    "node_visits_per_wave_segment": round(work_cnt["node_visits"] * 64 / segs, 3),
                    "leaf_fetches_per_wave_segment": round(work_cnt["leaf_fetches"] * 64 / segs, 3),
                    # fused: every Newton run (cThis pairs + follow-side retries) happens in k_trace's patch-uniform
                    # passes; staged: the passes are k_newton's / k_newton_lane's 64-pair chunks, which hold the
                    # candidate pairs only (the retries run per lane in k_resolve), so pairs / (64 x chunks)
                    "newton_lane_utilisation": round((newton_runs if fused_kernel else work_cnt["pairs"])
                                                     / max(1, 64 * work_cnt["newton_rounds"]), 4)
                    if work_cnt["newton_rounds"] else None,
                    "newton_lane_utilisation_def": ("(pairs + follow retries) / (64 x k_trace passes)" if fused_kernel
                                                    else "pairs / (64 x k_newton + k_newton_lane chunks)"),
                    # the fused chain per surface: even segments refract(INSIDE) (a lens's front), odd ones
                    # refract(OUTSIDE) (its back)
                    "newton_lane_utilisation_by_surface": ({
                        "front": round((newton_runs - work_cnt["runs_odd"])
                                       / max(1, 64 * (work_cnt["newton_rounds"] - work_cnt["rounds_odd"])), 4),
                        "back": round(work_cnt["runs_odd"] / max(1, 64 * work_cnt["rounds_odd"]), 4),
                        "passes_front": work_cnt["newton_rounds"] - work_cnt["rounds_odd"],
                        "passes_back": work_cnt["rounds_odd"]}
                        if fused_kernel and chain and work_cnt.get("rounds_odd") else None),
                    "overflow_rays_per_frame": work_cnt["overflow_rays"],
                    "source": "GPU counters (bzr_ctx_counters), rank 0, one frame",
                    "oracle_sample_rates": ({"newton": round(cnt["newton"] / cnt["segments"], 4),
                                             "follow": round(cnt["follow"] / cnt["segments"], 4)}
                                            if cnt and cnt["segments"] else None),
                },
            },
            "cpu_baseline": base,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
