#!/usr/bin/env python3
"""Host simulation for an intersect-only hybrid of the two pipelines.

A wave (8x8 pixels, bench ray order) walks the tree as k_traverse does and meets a set of entries: patches
whose exact planar gate (oracle) passes for some of its lanes.  With threshold T, entries with >= T lanes
would run in the walking wave as one patch-uniform Newton pass (k_trace's site); entries below T go to the
staged buckets as 8-byte pairs (k_newton, ~0.95 lane utilisation).  Printed per T: the share of pairs that
stay in-wave, the in-wave passes per wave and their lane utilisation, and the pairs left to the buckets.
Waves are sampled uniformly over the whole image (misses included) so the shares are frame totals.
usage: python scripts/hybrid_sim.py [--config cfg5] [--waves 1024]
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
    ap.add_argument("--config", default="cfg5")
    ap.add_argument("--waves", type=int, default=1024)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16, help="waves per gate batch")
    a = ap.parse_args()
    cfg = CONFIGS[a.config]
    patches = build_lens(po.OMesh, cfg.lenses[0]).bezier_patches()
    side = cfg.side
    nbw = side // 8
    rng = np.random.default_rng(a.seed)
    waves = rng.choice(nbw * nbw, a.waves, replace=False)
    hist = np.zeros(65, np.int64)  # entries by lane count
    hit_waves = 0
    for b0 in range(0, len(waves), a.batch):
        rows, cols = [], []
        for w in waves[b0:b0 + a.batch]:
            r0, c0 = (w // nbw) * 8, (w % nbw) * 8
            rr, cc = np.meshgrid(np.arange(8) + r0, np.arange(8) + c0, indexing="ij")
            rows.append(rr.reshape(-1))
            cols.append(cc.reshape(-1))
        rays = rays_for(cfg, np.concatenate(rows), np.concatenate(cols), side=side)
        gate = po.planar_gate(patches, rays, threads=8)  # [rays, patches]
        g = gate.reshape(-1, 64, gate.shape[1])
        lanes = g.sum(axis=1)  # [waves, patches]
        hit_waves += int((lanes.sum(axis=1) > 0).sum())
        hist += np.bincount(lanes[lanes > 0].ravel(), minlength=65)
    pairs = (hist * np.arange(65)).sum()
    entries = hist.sum()
    print({"config": a.config, "waves": a.waves, "waves_with_entries": hit_waves,
           "pairs_per_ray": round(pairs / (64 * a.waves), 4), "entries_per_wave": round(entries / a.waves, 3),
           "fused_utilisation": round(pairs / (64 * entries), 4)})
    for T in (1, 8, 16, 24, 32, 40, 48, 56):
        d = np.arange(65) >= T
        dp, de = (hist * np.arange(65))[d].sum(), hist[d].sum()
        print({"T": T, "in_wave_pair_share": round(dp / pairs, 4), "in_wave_passes_per_wave": round(de / a.waves, 3),
               "in_wave_utilisation": round(dp / max(1, 64 * de), 4),
               "bucket_pairs_per_ray": round((pairs - dp) / (64 * a.waves), 4)}, flush=True)
    print({"lanes_hist": {int(k): int(v) for k, v in enumerate(hist) if v}})


if __name__ == "__main__":
    main()
