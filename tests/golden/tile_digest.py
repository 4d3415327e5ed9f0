"""Per-tile SHA-256 digests of a whole frame's results (test infrastructure, shared by
tests/golden/make_digests.py, which runs the CPU oracle, and the GPU tests, which run libbzr).

Layout (fixed; the committed digests depend on it):
  - the side x side image is cut into 64 x 64 tiles, tile k = ty * (side / 64) + tx;
  - inside a tile the 4096 pixels are walked in 8 x 8 sub-tiles (configs.pixel_coords(.., 64, "tiles")),
    which is the order both the generator and the GPU test trace them in;
  - a tile's digest is SHA-256 over, in this order:
      chain configs:     out rays [6][4096] (float32 bits, row-major), status [4096] u32, segments [4096] u32
      intersect configs: hits [13][4096] (BezierIntersection SoA, float32 / u32 bits, row-major).
"""
from __future__ import annotations

import hashlib

import numpy as np

TILE = 64


def tile_pixels(cfg, side: int, tiles: np.ndarray | None = None):
    """(rows, cols) of the given tiles (default: all, in tile order), each tile in 8x8 sub-tile order."""
    from bzr_amd.configs import pixel_coords

    nbx = side // TILE
    if tiles is None:
        tiles = np.arange(nbx * nbx)
    sub_r, sub_c = pixel_coords(cfg, TILE, "tiles")
    rows = ((tiles // nbx)[:, None] * TILE + sub_r[None, :]).reshape(-1)
    cols = ((tiles % nbx)[:, None] * TILE + sub_c[None, :]).reshape(-1)
    return rows, cols


def _u32(a) -> np.ndarray:
    a = np.ascontiguousarray(a)
    return a.view(np.uint32) if a.dtype.itemsize == 4 else a.astype(np.uint32)


def chain_digests(out_rays: np.ndarray, status: np.ndarray, segments: np.ndarray) -> np.ndarray:
    """uint8 [ntiles, 32] for results laid out tile after tile (4096 rays each)."""
    n = status.shape[0]
    assert n % (TILE * TILE) == 0 and out_rays.shape == (6, n)
    k = n // (TILE * TILE)
    r = _u32(out_rays).reshape(6, k, TILE * TILE).transpose(1, 0, 2)
    s = _u32(status).reshape(k, TILE * TILE)
    g = _u32(segments).reshape(k, TILE * TILE)
    out = np.empty((k, 32), np.uint8)
    for t in range(k):
        h = hashlib.sha256(np.ascontiguousarray(r[t]).tobytes())
        h.update(s[t].tobytes())
        h.update(g[t].tobytes())
        out[t] = np.frombuffer(h.digest(), np.uint8)
    return out


def hits_digests(hits: np.ndarray) -> np.ndarray:
    """uint8 [ntiles, 32] for BezierIntersection SoA results [13, n] laid out tile after tile."""
    n = hits.shape[1]
    assert n % (TILE * TILE) == 0 and hits.shape[0] == 13
    k = n // (TILE * TILE)
    u = _u32(hits).reshape(13, k, TILE * TILE).transpose(1, 0, 2)
    out = np.empty((k, 32), np.uint8)
    for t in range(k):
        out[t] = np.frombuffer(hashlib.sha256(np.ascontiguousarray(u[t]).tobytes()).digest(), np.uint8)
    return out
