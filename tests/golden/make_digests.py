#!/usr/bin/env python3
"""Full-frame oracle digests (test infrastructure): run the CPU oracle (oracle/bzr_oracle.c, the C
restatement of reference/bezierMesh.cpp:206-227, bezierTriangle.cpp:123-195, bezierLens.cpp:4-34 and the
chain driver reference/test.cpp:376-401) over whole benchmark frames and commit one SHA-256 per 64x64 tile
(layout: tests/golden/tile_digest.py).  tests/test_gpu_fullsize.py traces the same frames through libbzr
and compares tile by tile, so the bench configs' full-size output is pinned to the oracle bit for bit.

  d_cfg4_4096.npz   cfg4 (BASELINE configs[3], the bench workload): two lenses, refraction chain, the
                    whole 4096x4096 frame (4096 tiles)
  d_cfg3_2048.npz   cfg3 (configs[2]): robot.stl x8 split, BezierMesh::intersect, whole 2048x2048 frame
  d_cfg5_8192.npz   cfg5 (configs[4]): 301 056 patches, BezierMesh::intersect, 24 of the 16 384 tiles of
                    the 8192x8192 frame (8 inside the lens outline, 12 on its rim, 4 outside; seeded) --
                    the whole frame is ~30 h of oracle time

Meshes are built by the oracle's own preprocessing (OMesh), not by the product.  Each file also holds
the SHA-256 of the patch records, the tile indices and per-tile hit counts (to tell a preprocessing
difference from a tracing one).  Every array is plain data (numpy.load(allow_pickle=False)).

usage: python tests/golden/make_digests.py [cfg4 cfg3 cfg5] [--threads N]
(about 4 + 3 + 4 minutes on 8 cores)
"""
from __future__ import annotations

import argparse
import hashlib
import sys
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
sys.path[:0] = [str(REPO), str(REPO / "cuda-bezier-triangle-raytracer_amd"), str(HERE)]

from bzr_amd.configs import CONFIGS, build_lens, rays_for  # noqa: E402
from oracle import pyoracle as po  # noqa: E402
from tile_digest import TILE, chain_digests, hits_digests, tile_pixels  # noqa: E402

CHUNK_TILES = 128  # tiles per oracle call (524 288 rays)


def cfg5_tiles(side: int = 8192, seed: int = 0xC5) -> np.ndarray:
    """24 tiles of the cfg5 frame: 8 well inside the lens outline, 12 straddling its rim, 4 outside."""
    cfg = CONFIGS["cfg5"]
    nb = side // TILE
    k = np.arange(nb * nb)
    # tile centre in world (y, z); the lens outline is the ellipse (y/4)^2 + (z/2)^2 = 1
    y = cfg.y[0] + (cfg.y[1] - cfg.y[0]) * ((k % nb) + 0.5) / nb
    z = cfg.z[0] + (cfg.z[1] - cfg.z[0]) * ((k // nb) + 0.5) / nb
    rho = np.sqrt((y / 4.0) ** 2 + (z / 2.0) ** 2)
    half = 0.5 * (cfg.y[1] - cfg.y[0]) / nb / 4.0  # half a tile in rho units (y direction)
    rng = np.random.default_rng(seed)
    inside = rng.choice(k[rho < 0.9], 8, replace=False)
    rim = rng.choice(k[np.abs(rho - 1.0) < 1.5 * half], 12, replace=False)
    outside = rng.choice(k[(rho > 1.05) & (rho < 1.2)], 4, replace=False)
    return np.sort(np.concatenate([inside, rim, outside]))


def run(name: str, threads: int) -> None:
    cfg = CONFIGS[name]
    side = cfg.side
    patches = [build_lens(po.OMesh, lens).bezier_patches() for lens in cfg.lenses]
    ris = [lens.ri for lens in cfg.lenses]
    tiles = cfg5_tiles(side) if name == "cfg5" else np.arange((side // TILE) ** 2)
    digests, hits = [], []
    t0 = time.time()
    for c0 in range(0, len(tiles), CHUNK_TILES):
        tk = tiles[c0:c0 + CHUNK_TILES]
        r, c = tile_pixels(cfg, side, tk)
        rays = rays_for(cfg, r, c, side=side)
        if cfg.op == "chain":
            o, s, g = po.trace_chain(patches, ris, rays, threads=threads)
            digests.append(chain_digests(o, s, g))
            hits.append((s.reshape(-1, TILE * TILE) != 0).sum(1))
        else:
            h = po.intersect(patches[0], rays, threads=threads)
            digests.append(hits_digests(h))
            hits.append((h.view(np.uint32)[11].reshape(-1, TILE * TILE) == 4).sum(1))
        done = c0 + len(tk)
        print(f"{name}: {done}/{len(tiles)} tiles, {time.time() - t0:.0f} s", flush=True)
    ph = hashlib.sha256(b"".join(np.ascontiguousarray(p).tobytes() for p in patches)).digest()
    out = HERE / f"d_{name}_{side}.npz"
    np.savez_compressed(out, digests=np.concatenate(digests), tiles=tiles.astype(np.int32),
                        hits=np.concatenate(hits).astype(np.uint16),
                        patch_sha256=np.frombuffer(ph, np.uint8), side=np.int32(side))
    print(f"wrote {out} ({len(tiles)} tiles, {time.time() - t0:.0f} s)", flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["cfg4", "cfg3", "cfg5"])
    ap.add_argument("--threads", type=int, default=0, help="OpenMP threads (0: all)")
    a = ap.parse_args()
    for name in a.configs:
        run(name, a.threads)


if __name__ == "__main__":
    main()
