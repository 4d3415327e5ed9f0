#!/usr/bin/env python3
"""Host simulation: fused-kernel Newton passes if a wave's sparse entries (patches fewer than T of its lanes
pass) ran as per-lane rounds (each lane evaluating its own patch, record per lane) instead of one
patch-uniform pass each.  Same sampling as scripts/bucket_sim.py (cfg4 chain, oracle planar gates, retries
left out).  Per wave:  dense passes = entries with >= T lanes;  sparse rounds = the largest number of sparse
entries any one lane is in.  cost(c) = dense + c * rounds, c = a per-lane round's cost in passes.
usage: python scripts/sparse_sim.py [--blocks 80] [--side 4096]
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "cuda-bezier-triangle-raytracer_amd"), str(REPO), str(REPO / "scripts")]

from bzr_amd.configs import CONFIGS, build_lens, rays_for  # noqa: E402
from oracle import pyoracle as po  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=80)
    ap.add_argument("--side", type=int, default=4096)
    ap.add_argument("--config", default="cfg4")
    ap.add_argument("--seed", type=int, default=9)
    a = ap.parse_args()
    cfg = CONFIGS[a.config]
    lenses = [build_lens(po.OMesh, l).bezier_patches() for l in cfg.lenses]
    rng = np.random.default_rng(a.seed)
    nb = a.side // 32
    by, bx = np.divmod(np.arange(nb * nb), nb)
    y = cfg.y[0] + (cfg.y[1] - cfg.y[0]) * (bx + 0.5) / nb
    z = cfg.z[0] + (cfg.z[1] - cfg.z[0]) * (by + 0.5) / nb
    inside = np.nonzero((y / 4.0) ** 2 + (z / 2.0) ** 2 < 1.0)[0]
    blocks = rng.choice(inside, min(a.blocks, len(inside)), replace=False)
    rows, cols = [], []
    for b in blocks:
        r0, c0 = (b // nb) * 32, (b % nb) * 32
        for w in range(16):
            q, k = divmod(w, 4)
            wr, wc = r0 + 16 * (q // 2) + 8 * (k // 2), c0 + 16 * (q % 2) + 8 * (k % 2)
            rr, cc = np.meshgrid(np.arange(8) + wr, np.arange(8) + wc, indexing="ij")
            rows.append(rr.reshape(-1))
            cols.append(cc.reshape(-1))
    rays = rays_for(cfg, np.concatenate(rows), np.concatenate(cols), side=a.side)
    alive = np.ones(rays.shape[1], bool)
    Ts = (2, 4, 8, 12, 16, 24, 32)
    cs = (1.5, 2.0, 3.0)
    nw = rays.shape[1] // 64
    wave_passes = np.zeros(nw)
    wave_cost = {(T, c): np.zeros(nw) for T in Ts for c in cs}
    for seg in range(2 * len(lenses)):
        lens = lenses[seg // 2]
        gate = po.planar_gate(lens, rays, threads=8) & alive[:, None]
        g = gate.reshape(-1, 64, gate.shape[1])          # [waves, lanes, patches]
        lanes_per = g.sum(axis=1)                         # [waves, patches]
        wave_passes += (lanes_per > 0).sum(axis=1)
        for T in Ts:
            sparse = (lanes_per > 0) & (lanes_per < T)    # [waves, patches]
            dense = ((lanes_per >= T)).sum(axis=1)
            per_lane = (g & sparse[:, None, :]).sum(axis=2)  # [waves, lanes] sparse entries per lane
            rounds = per_lane.max(axis=1)
            for c in cs:
                wave_cost[(T, c)] += dense + c * rounds
        o, st = po.refract(lens, cfg.lenses[seg // 2].ri, rays, np.full(rays.shape[1], 1 + seg % 2, np.uint32),
                           threads=8)
        alive &= st != 0
        rays = o
    base = wave_passes.sum()
    print({"config": a.config, "waves": nw, "passes": int(base), "p99_wave": float(np.percentile(wave_passes, 99)),
           "max_wave": float(wave_passes.max())})
    for T in Ts:
        print({"T": T, **{f"c={c}": f"{100 * (wave_cost[(T, c)].sum() / base - 1):+.1f} % (max wave {wave_cost[(T, c)].max():.0f})"
                          for c in cs}}, flush=True)


if __name__ == "__main__":
    main()
