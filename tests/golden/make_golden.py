#!/usr/bin/env python3
"""Generate the golden fixtures F1-F4 of SURVEY.md 8(c) from the oracle (oracle/bzr_oracle.c, the C
restatement of the reference; see oracle/README in DESIGN.md "Oracle").  F5, the seven
measureApproximation KATs, lives in tests/test_oracle_kats.py as published constants.

  f1_cfg1.npz         cfg1 patches (126), 64x64 primary grid, BezierMesh::intersect hits [13, n]
  f2_cfg2.npz         cfg2 patches (3072), 64x64 primary grid, hits
  f3_cfg2_chain.npz   cfg2 64x64 grid: refract(INSIDE) -> refract(OUTSIDE) per stage, and trace_chain
  f4_random.npz       4096 seeded rays (splitmix64, seed 0x5EED): origins jittered on x = 0 over the cfg2
                      window, directions in a +-15 degree cone around +x; hits against the cfg2 lens at
                      the origin and at x = 10

Every array is data (float32 / uint32), loadable with numpy.load(allow_pickle=False).  Rerun with
`python tests/golden/make_golden.py`; tests/test_golden.py checks the oracle still reproduces them.
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
sys.path[:0] = [str(REPO), str(REPO / "cuda-bezier-triangle-raytracer_amd")]

from bzr_amd.configs import CONFIGS, Lens, build_lens, grid_rays  # noqa: E402
from oracle import pyoracle as po  # noqa: E402

SIDE = 64
SEED = 0x5EED
N_RANDOM = 4096


def splitmix64(seed: int, n: int) -> np.ndarray:
    """n uint64 outputs of splitmix64 (Vigna) from `seed`."""
    out = np.empty(n, np.uint64)
    x = seed & 0xFFFFFFFFFFFFFFFF
    for k in range(n):
        x = (x + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = x
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        out[k] = z ^ (z >> 31)
    return out


def random_rays(n: int = N_RANDOM, seed: int = SEED) -> np.ndarray:
    u = (splitmix64(seed, 4 * n) >> np.uint64(11)).astype(np.float64) / float(1 << 53)  # [0, 1)
    u = u.reshape(4, n)
    cfg = CONFIGS["cfg2"]
    y = cfg.y[0] + (cfg.y[1] - cfg.y[0]) * u[0]
    z = cfg.z[0] + (cfg.z[1] - cfg.z[0]) * u[1]
    theta = np.radians(15.0) * np.sqrt(u[2])  # uniform over the cone's cap
    phi = 2.0 * np.pi * u[3]
    d = np.stack([np.cos(theta), np.sin(theta) * np.cos(phi), np.sin(theta) * np.sin(phi)]).astype(np.float32)
    # Ray's constructor normalizes in float (reference/3dGeomUtil.h:176-178): v / sqrt(x*x + (y*y + z*z))
    zz = d[0] * d[0] + (d[1] * d[1] + d[2] * d[2])
    d = d / np.sqrt(zz)
    o = np.stack([np.zeros(n), y, z]).astype(np.float32)
    return np.ascontiguousarray(np.concatenate([o, d.astype(np.float32)]))


def main():
    cfg1, cfg2 = CONFIGS["cfg1"], CONFIGS["cfg2"]
    p1 = build_lens(po.OMesh, cfg1.lenses[0]).bezier_patches()
    r1 = grid_rays(cfg1, side=SIDE)
    np.savez_compressed(HERE / "f1_cfg1.npz", patches=p1, rays=r1, hits=po.intersect(p1, r1))

    p2 = build_lens(po.OMesh, cfg2.lenses[0]).bezier_patches()
    r2 = grid_rays(cfg2, side=SIDE)
    np.savez_compressed(HERE / "f2_cfg2.npz", patches=p2, rays=r2, hits=po.intersect(p2, r2))

    o1, s1 = po.refract(p2, 1.3, r2, np.full(r2.shape[1], 1, np.uint32))
    alive = s1 != 0
    o2, s2 = po.refract(p2, 1.3, o1, np.full(r2.shape[1], 2, np.uint32))
    s2 = np.where(alive, s2, 0).astype(np.uint32)
    co, cs, cg = po.trace_chain([p2], [1.3], r2)
    np.savez_compressed(HERE / "f3_cfg2_chain.npz", rays=r2, stage1_rays=o1, stage1_status=s1, stage2_rays=o2,
                        stage2_status=s2, chain_rays=co, chain_status=cs, chain_segments=cg)

    at_origin = Lens("ellipsoid", 32, 16, (1.0, 4.0, 2.0), (0.0, 0.0, 0.0))
    p0 = build_lens(po.OMesh, at_origin).bezier_patches()
    r4 = random_rays()
    np.savez_compressed(HERE / "f4_random.npz", rays=r4, hits_origin=po.intersect(p0, r4),
                        hits_x10=po.intersect(p2, r4))
    for f in sorted(HERE.glob("f*.npz")):
        print(f.name, f.stat().st_size)


if __name__ == "__main__":
    main()
