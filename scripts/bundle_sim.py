#!/usr/bin/env python3
"""Host replay of a wave-bundle BVH walk (bzr_debug_traverse_bundle) against the per-lane walk.

Waves are 8x8-pixel tiles sampled from the lens region; the rays of every chain segment come from the
oracle (cfg2/cfg4: refract inside / outside per lens; cfg3/cfg5: primaries only).  Prints, per segment:
batches of up to 16 nodes per wave, leaves admitted by the bundle test vs by the per-lane slab tests,
per-lane node visits, and leaves the bundle test missed (must be 0: the bundle test is conservative).
usage: python scripts/bundle_sim.py [--config cfg4] [--waves 400] [--seed 1]
"""
import argparse
import ctypes
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "cuda-bezier-triangle-raytracer_amd"))
sys.path.insert(0, str(REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg4")
    ap.add_argument("--waves", type=int, default=400)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--spread", type=float, default=float("inf"), help="direction spread above which a wave walks per lane")
    a = ap.parse_args()
    import bzr_amd
    from bzr_amd.configs import CONFIGS, build_lens, pixel_coords, rays_for
    from oracle import pyoracle

    cfg = CONFIGS[a.config]
    lenses = [build_lens(bzr_amd.TriMesh, l).bezier_patches() for l in cfg.lenses]
    rng = np.random.default_rng(a.seed)
    side = cfg.side
    ntile = side // 8
    # sample tiles whose centre ray hits the first lens's bounding box in y/z (the lens region)
    tiles = []
    while len(tiles) < a.waves:
        t = int(rng.integers(0, ntile * ntile))
        r, c = (t // ntile) * 8 + 4, (t % ntile) * 8 + 4
        ray = rays_for(cfg, np.array([r]), np.array([c]))
        if a.config in ("cfg3",) or (abs(ray[1, 0]) < 4.0 and abs(ray[2, 0]) < 2.0):
            tiles.append(t)
    tiles = np.array(tiles)
    sub_r, sub_c = pixel_coords(cfg, 8, "tiles")
    rows = ((tiles // ntile)[:, None] * 8 + sub_r[None, :]).reshape(-1)
    cols = ((tiles % ntile)[:, None] * 8 + sub_c[None, :]).reshape(-1)
    rays = rays_for(cfg, rows, cols)
    L = bzr_amd.lib()
    fn = L.bzr_debug_traverse_bundle
    fn.restype = ctypes.c_int32
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_float,
                   ctypes.c_void_p]
    segs = []
    if cfg.op == "chain":
        alive = np.ones(rays.shape[1], bool)
        cur = rays
        for li, p in enumerate(lenses):
            for exp in (1, 2):  # BZR_RR_INSIDE, BZR_RR_OUTSIDE
                segs.append((f"lens{li}-{'in' if exp == 1 else 'out'}", li, cur.copy(), alive.copy()))
                o, s = pyoracle.refract(p, cfg.lenses[li].ri, cur, np.full(cur.shape[1], exp, np.uint32))
                alive &= s == exp
                cur = np.where(alive[None, :], o, cur).astype(np.float32)
    else:
        segs.append(("primary", 0, rays, np.ones(rays.shape[1], bool)))
    tot = np.zeros(12, np.uint64)
    for name, li, r, al in segs:
        r = r.copy()
        r[:, ~al] = np.float32(0.0)  # dead lanes: zero direction -> inactive in the replay
        r = np.ascontiguousarray(r, np.float32)
        p = np.ascontiguousarray(lenses[li], np.float32)
        st = (ctypes.c_uint64 * 12)()
        assert fn(p.ctypes.data, len(p), 264, r.ctypes.data, r.shape[1], a.spread, st) == 0
        s = np.array(st[:], np.uint64)
        tot += s
        w = max(int(s[0]), 1)
        print(f"{a.config} {name:10s} waves {int(s[0]):5d}  bundle batches/wave {s[1]/w:6.2f}  leaves/wave bundle "
              f"{s[2]/w:6.2f} lane {s[4]/w:6.2f}  lane node visits/wave {s[3]/w:6.2f}  slots/wave {s[6]/w:6.1f}  "
              f"max stack {int(s[7])}  missed {int(s[5])}  per-lane waves {int(s[8])}  overflowing batches {int(s[9])}  "
              f"pre-test keeps {s[10]/w:6.2f}/wave (wrongly rejected {int(s[11])})")
    w = max(int(tot[0]), 1)
    print(f"{a.config} all        waves {int(tot[0]):5d}  bundle batches/wave {tot[1]/w:6.2f}  leaves/wave bundle "
          f"{tot[2]/w:6.2f} lane {tot[4]/w:6.2f}  lane node visits/wave {tot[3]/w:6.2f}  missed {int(tot[5])}  "
          f"per-lane waves {int(tot[8])}  overflowing batches {int(tot[9])}  pre-test keeps {tot[10]/w:6.2f}/wave "
          f"(wrongly rejected {int(tot[11])})")


if __name__ == "__main__":
    main()
