#!/usr/bin/env python3
"""Throughput of the illumination pipeline (bzr_illuminate: emit -> sphere cull -> chain -> target counts)
on the cfg2 lens, emitter just behind it (inside the lens's bounding sphere, so nothing is culled and
every ray is traced).  Prints one JSON line: emitted rays / s and the landed fraction."""
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "cuda-bezier-triangle-raytracer_amd"))
sys.path.insert(0, str(REPO))

import bzr_amd  # noqa: E402
from bzr_amd.configs import CONFIGS, build_lens  # noqa: E402


def main():
    total = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 24
    ctx = bzr_amd.Context(0)
    dm = bzr_amd.DeviceMesh(ctx, build_lens(bzr_amd.TriMesh, CONFIGS["cfg2"].lenses[0]).bezier_patches())
    em = bzr_amd.Emitter(origin=(0.0, -0.5, -0.5), edge_u=(0.0, 1.0, 0.0), edge_v=(0.0, 0.0, 1.0), parts_u=4,
                         parts_v=4, points_per_part=1024, rays_per_point=1024, belts=16, seed=1)
    tg = bzr_amd.Target(origin=(25.0, -12.0, -12.0), axis_u=(0.0, 1.0, 0.0), axis_v=(0.0, 0.0, 1.0), size_u=24.0,
                        size_v=24.0, bins_u=512, bins_v=512)
    bzr_amd.illuminate(ctx, [dm], [1.3], em, 1 << 20, tg)  # warm-up
    t0 = time.perf_counter()
    hist, stats = bzr_amd.illuminate(ctx, [dm], [1.3], em, total, tg)
    dt = time.perf_counter() - t0
    print(json.dumps({"workload": "illuminate cfg2 lens, emitter at x=0 (no cull), 512^2 target",
                      "rays": total, "seconds": round(dt, 4), "mrays_per_s": round(total / dt / 1e6, 1),
                      "stats": stats, "landed_fraction": round(stats["landed"] / total, 5)}))


if __name__ == "__main__":
    main()
