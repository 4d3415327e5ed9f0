#!/usr/bin/env python3
"""Host simulation of the fused kernel's Newton-pass count ("lane utilisation"): how many
patch-uniform passes a wave needs for its rays' gate-passing patches, and how many a group of G waves
would need if it pooled its (ray, patch) pairs by patch (cross-wave bucketing).  CPU only (the oracle's
planar gate, reference/bezierTriangle.cpp:124-131); follow-side retries are left out (the kernel folds
almost all of them into existing passes).

For each segment of the cfg4 chain (primaries at the first lens's inside surface, then the rays the
oracle refracts there at its outside surface, ...), sampled 32x32-pixel blocks of 16 waves (8x8 each,
bench.py's layout; pools of 2 and 4 waves are 16x8 / 16x16 sub-blocks) are simulated:
  per-wave passes      = sum over waves of the distinct gate-passing patches of its live rays
  pooled(G) passes     = sum over groups of G waves of sum over patches of ceil(pairs / 64)
usage: python scripts/bucket_sim.py [--blocks 80] [--side 4096]
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "cuda-bezier-triangle-raytracer_amd"), str(REPO)]

from bzr_amd.configs import CONFIGS, build_lens, rays_for  # noqa: E402
from oracle import pyoracle as po  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=80)
    ap.add_argument("--side", type=int, default=4096)
    ap.add_argument("--seed", type=int, default=9)
    a = ap.parse_args()
    cfg = CONFIGS["cfg4"]
    lenses = [build_lens(po.OMesh, l).bezier_patches() for l in cfg.lenses]
    rng = np.random.default_rng(a.seed)
    # 32x32-pixel blocks whose centre lies inside the lens outline (the only ones with work), 16 waves each,
    # ordered so that consecutive pools of 2 / 4 / 16 waves are 16x8 / 16x16 / 32x32 pixels
    nb = a.side // 32
    by, bx = np.divmod(np.arange(nb * nb), nb)
    y = cfg.y[0] + (cfg.y[1] - cfg.y[0]) * (bx + 0.5) / nb
    z = cfg.z[0] + (cfg.z[1] - cfg.z[0]) * (by + 0.5) / nb
    inside = np.nonzero((y / 4.0) ** 2 + (z / 2.0) ** 2 < 1.0)[0]
    blocks = rng.choice(inside, a.blocks, replace=False)
    rows, cols = [], []
    for b in blocks:
        r0, c0 = (b // nb) * 32, (b % nb) * 32
        for w in range(16):  # 16 waves of 8x8 pixels: quadrants of 2x2 waves
            q, k = divmod(w, 4)
            wr, wc = r0 + 16 * (q // 2) + 8 * (k // 2), c0 + 16 * (q % 2) + 8 * (k % 2)
            rr, cc = np.meshgrid(np.arange(8) + wr, np.arange(8) + wc, indexing="ij")
            rows.append(rr.reshape(-1))
            cols.append(cc.reshape(-1))
    rays = rays_for(cfg, np.concatenate(rows), np.concatenate(cols), side=a.side)
    alive = np.ones(rays.shape[1], bool)
    tot = {"wave": 0, 2: 0, 4: 0, 16: 0}
    pairs_total = 0
    for seg in range(4):
        lens = lenses[seg // 2]
        gate = po.planar_gate(lens, rays, threads=8) & alive[:, None]  # [rays, patches]
        g = gate.reshape(-1, 64, gate.shape[1])  # waves
        pairs = int(gate.sum())
        pairs_total += pairs
        per_wave = int(g.any(axis=1).sum())
        line = {"segment": seg, "live_rays": int(alive.sum()), "pairs": pairs, "passes_per_wave_model": per_wave,
                "lane_utilisation": round(pairs / max(1, 64 * per_wave), 4)}
        tot["wave"] += per_wave
        for G in (2, 4, 16):
            cnt = g.reshape(-1, G * 64, gate.shape[1]).sum(axis=1)  # pairs per (group, patch)
            passes = int(np.ceil(cnt / 64.0).sum())
            line[f"pooled_{G}_waves"] = passes
            tot[G] += passes
        print(line, flush=True)
        # next segment's rays: the oracle's refraction at this surface (inside, then outside)
        o, st = po.refract(lens, lens_ri(cfg, seg), rays, np.full(rays.shape[1], 1 + seg % 2, np.uint32), threads=8)
        alive &= st != 0
        rays = o
    print({"passes_per_wave": tot["wave"], "utilisation": round(pairs_total / (64 * tot["wave"]), 4),
           **{f"pooled_{G}": f"{tot[G]} ({100 * (1 - tot[G] / tot['wave']):.1f} % fewer)" for G in (2, 4, 16)}})


def lens_ri(cfg, seg):
    return cfg.lenses[seg // 2].ri


if __name__ == "__main__":
    main()
