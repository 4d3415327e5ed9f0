#!/usr/bin/env python3
"""Host bound for VERDICT r04 item 5 (two-wave k_trace blocks that lend lanes across waves): how many of the
fused kernel's patch-uniform Newton passes two neighbouring waves could share, and how unevenly their work is
split.  CPU only (the oracle's planar gate, reference/bezierTriangle.cpp:124-131); follow-side retries are left
out (the kernel folds almost all of them into existing passes).

The proposal: the waves of a two-wave block exchange their collected-entry lists in LDS; a patch both waves
need runs once, in the wave holding more of its lanes, and the other wave's lanes join (their rays through
LDS) when both waves' lane counts for that patch are below 32 ("both < 32"), or more generally whenever the
lanes fit into one wave ("a + b <= 64").  Saved passes per block = patches shared under the rule.  Any real
implementation only shares patches that sit in both waves' current 16-entry batches at the same time, so this
is an upper bound on the saving.

The cost side: the two waves must meet at every batch to exchange lists, so each waits for the other; the
imbalance of the two waves' pass counts, E|pA - pB| / E[pA + pB], is the fraction of pass time one of them
would spend waiting (lower bound: walk lengths differ too).

For each segment of the cfg4 chain (primaries at the first lens's inside surface, then the rays the oracle
refracts there at its outside surface, ...), sampled 16x8-pixel blocks (two 8x8 waves side by side, bench.py's
layout) inside the lens outline.
usage: python scripts/pair_sim.py [--blocks 400] [--side 4096]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "cuda-bezier-triangle-raytracer_amd"), str(REPO)]

from bzr_amd.configs import CONFIGS, build_lens, rays_for  # noqa: E402
from oracle import pyoracle as po  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=400)
    ap.add_argument("--side", type=int, default=4096)
    ap.add_argument("--seed", type=int, default=5)
    a = ap.parse_args()
    cfg = CONFIGS["cfg4"]
    lenses = [build_lens(po.OMesh, l).bezier_patches() for l in cfg.lenses]
    rng = np.random.default_rng(a.seed)
    nbx, nby = a.side // 16, a.side // 8  # 16 x 8 pixel blocks
    by, bx = np.divmod(np.arange(nbx * nby), nbx)
    y = cfg.y[0] + (cfg.y[1] - cfg.y[0]) * (bx * 16 + 8) / a.side
    z = cfg.z[0] + (cfg.z[1] - cfg.z[0]) * (by * 8 + 4) / a.side
    inside = np.nonzero((y / 4.0) ** 2 + (z / 2.0) ** 2 < 1.0)[0]
    blocks = rng.choice(inside, a.blocks, replace=False)
    rows, cols = [], []
    for b in blocks:
        r0, c0 = (b // nbx) * 8, (b % nbx) * 16
        for w in range(2):
            rr, cc = np.meshgrid(np.arange(8) + r0, np.arange(8) + c0 + 8 * w, indexing="ij")
            rows.append(rr.reshape(-1))
            cols.append(cc.reshape(-1))
    rays = rays_for(cfg, np.concatenate(rows), np.concatenate(cols), side=a.side)
    alive = np.ones(rays.shape[1], bool)
    tot = dict(passes=0, pairs=0, save_fit=0, save_32=0, imb=0)
    for seg in range(4):
        lens = lenses[seg // 2]
        gate = po.planar_gate(lens, rays, threads=8) & alive[:, None]  # [rays, patches]
        lanes = gate.reshape(-1, 2, 64, gate.shape[1]).sum(axis=2)      # [block, wave, patch] lane counts
        A, B = lanes[:, 0, :], lanes[:, 1, :]
        passes = int((A > 0).sum() + (B > 0).sum())
        shared = (A > 0) & (B > 0)
        save_fit = int((shared & (A + B <= 64)).sum())
        save_32 = int((shared & (A < 32) & (B < 32)).sum())
        pa, pb = (A > 0).sum(axis=1), (B > 0).sum(axis=1)
        imb = int(np.abs(pa - pb).sum())
        pairs = int(gate.sum())
        for k, v in dict(passes=passes, pairs=pairs, save_fit=save_fit, save_32=save_32, imb=imb).items():
            tot[k] += v
        print(json.dumps({"segment": seg, "live_rays": int(alive.sum()), "pairs": pairs, "passes": passes,
                          "utilisation": round(pairs / max(1, 64 * passes), 4),
                          "shared_fit_saved": save_fit, "shared_both_below_32_saved": save_32,
                          "pass_imbalance": round(imb / max(1, passes), 4)}), flush=True)
        o, st = po.refract(lens, cfg.lenses[seg // 2].ri, rays, np.full(rays.shape[1], 1 + seg % 2, np.uint32),
                           threads=8)
        alive &= st != 0
        rays = o
    P = tot["passes"]
    print(json.dumps({
        "blocks": a.blocks, "passes": P, "utilisation": round(tot["pairs"] / (64 * P), 4),
        "saved_fit_pct": round(100 * tot["save_fit"] / P, 2),
        "saved_both_below_32_pct": round(100 * tot["save_32"] / P, 2),
        "utilisation_if_saved_fit": round(tot["pairs"] / (64 * (P - tot["save_fit"])), 4),
        "utilisation_if_saved_both_below_32": round(tot["pairs"] / (64 * (P - tot["save_32"])), 4),
        "pass_imbalance_pct": round(100 * tot["imb"] / P, 2),
        "note": "saved = passes two side-by-side waves share under the rule (upper bound); imbalance = "
                "sum |passes(A) - passes(B)| / sum passes: the pass time a wave waits for its partner at a "
                "per-batch exchange (walk-length differences come on top)"}))


if __name__ == "__main__":
    main()
