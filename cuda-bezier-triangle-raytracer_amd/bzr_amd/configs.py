"""Workload recipes of BASELINE.json's five configs.

A recipe builds the lens / object meshes with any Mesh-like builder (the
product's TriMesh or the oracle's OMesh: same method names) and defines the
primary-ray grid.  Rays start on an axis-aligned plane and travel along +x,
pixel centres at (k + 0.5) / size, exactly as SURVEY.md section 8d specifies.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from pathlib import Path

import numpy as np

# package data: copy of reference/robot.stl (150 binary STL triangles), the input mesh of cfg3
ROBOT_STL = Path(__file__).resolve().parent / "data" / "robot.stl"


@dataclass(frozen=True)
class Lens:
    kind: str                   # "ellipsoid" | "stl"
    sectors: int = 0
    belts: int = 0
    size: tuple = (1.0, 1.0, 1.0)
    offset: tuple = (0.0, 0.0, 0.0)
    split: int = 1              # Mesh::splitTriangles(divisor) before standardizing
    ri: float = 1.3             # refractive index (reference/test.cpp:375)


@dataclass(frozen=True)
class Config:
    name: str
    lenses: tuple
    side: int                   # rays per image side
    origin_x: float
    y: tuple
    z: tuple
    op: str                     # "intersect" (primary hits) | "chain" (refraction chain)
    note: str = ""
    extra: dict = field(default_factory=dict)


CONFIGS = {
    "cfg1": Config("cfg1", (Lens("ellipsoid", 3, 7),), 256, -5.0, (-1.2, 1.2), (-1.2, 1.2), "intersect",
                   "makeUnitSphere(3,7) Bezier mesh, 256x256 primary rays (CPU plumbing config)"),
    "cfg2": Config("cfg2", (Lens("ellipsoid", 32, 16, (1.0, 4.0, 2.0), (10.0, 0.0, 0.0)),), 1024, 0.0,
                   (-4.2, 4.2), (-2.1, 2.1), "chain",
                   "makeEllipsoid(32,16,(1,4,2)) lens at x=10, ri 1.3, 1024x1024 rays, refract(inside)+refract(outside)"),
    "cfg3": Config("cfg3", (Lens("stl", split=8),), 2048, -100.0, (-25.0, 25.0), (-25.0, 25.0), "intersect",
                   "robot.stl (150 tris) split x8 -> 9600 tris -> 28800 patches, 2048x2048 primary rays"),
    "cfg4": Config("cfg4", (Lens("ellipsoid", 32, 16, (1.0, 4.0, 2.0), (10.0, 0.0, 0.0)),
                            Lens("ellipsoid", 32, 16, (1.0, 4.0, 2.0), (13.0, 0.0, 0.0))), 4096, 0.0,
                   (-4.2, 4.2), (-2.1, 2.1), "chain", "two stacked cfg2 lenses at x=10 and x=13, 4096x4096 rays"),
    "cfg5": Config("cfg5", (Lens("ellipsoid", 224, 224, (1.0, 4.0, 2.0), (10.0, 0.0, 0.0)),), 8192, 0.0,
                   (-4.2, 4.2), (-2.1, 2.1), "intersect",
                   "makeEllipsoid(224,224,(1,4,2)) at x=10 (100352 tris -> 301056 patches), 8192x8192 rays"),
}


def build_lens(builder_cls, lens: Lens):
    """Run the reference's preprocessing recipe with `builder_cls` (TriMesh or OMesh); returns the mesh."""
    m = builder_cls()
    if lens.kind == "ellipsoid":
        m.make_ellipsoid(lens.sectors, lens.belts, lens.size)
    elif lens.kind == "stl":
        m.read_stl(ROBOT_STL)
    else:
        raise ValueError(lens.kind)
    if lens.split > 1:
        m.split(lens.split)
    if any(lens.offset):
        m.translate(lens.offset)
    m.standardize()
    return m


def build_patches(builder_cls, cfg: Config):
    return [build_lens(builder_cls, lens).bezier_patches() for lens in cfg.lenses]


def pixel_coords(cfg: Config, side: int | None = None, order: str = "tiles", tile: int = 8, wave=None):
    """Pixel (row, col) index arrays for a side x side grid.

    order "rows": row-major.  order "tiles": tile x tile blocks (one 64-ray wavefront
    per 8x8 block) so the rays of a wavefront are spatially coherent.  wave=(wr, wc) (order "tiles", wr x wc
    = the rays per block): blocks of wr rows x wc columns instead (A/B of ray-to-wave mappings)."""
    s = cfg.side if side is None else side
    wr, wc = (tile, tile) if wave is None else wave
    k = np.arange(s * s, dtype=np.int64)
    if order == "rows" or s % wr or s % wc:
        return k // s, k % s
    t, w = k // (wr * wc), k % (wr * wc)
    tiles_per_row = s // wc
    return (t // tiles_per_row) * wr + w // wc, (t % tiles_per_row) * wc + w % wc


def rays_for(cfg: Config, rows: np.ndarray, cols: np.ndarray, side: int | None = None,
             height: int | None = None) -> np.ndarray:
    """SoA rays [6, n] float32 for the given pixels of a side-wide, height-tall image (height defaults
    to side) over the config's window; direction +x (already unit length)."""
    s = cfg.side if side is None else side
    h = s if height is None else height
    n = len(rows)
    f = np.float32
    y0, y1 = f(cfg.y[0]), f(cfg.y[1])
    z0, z1 = f(cfg.z[0]), f(cfg.z[1])
    out = np.zeros((6, n), dtype=np.float32)
    out[0] = f(cfg.origin_x)
    out[1] = y0 + (y1 - y0) * ((cols.astype(np.float32) + f(0.5)) / f(s))
    out[2] = z0 + (z1 - z0) * ((rows.astype(np.float32) + f(0.5)) / f(h))
    out[3] = f(1.0)
    return out


def grid_rays(cfg: Config, side: int | None = None, order: str = "tiles", wave=None) -> np.ndarray:
    r, c = pixel_coords(cfg, side, order, wave=wave)
    return rays_for(cfg, r, c, side)


def shard_pixels(cfg: Config, rank: int, world: int, side: int | None = None, height: int | None = None,
                 block: int = 64, order: str = "centre"):
    """Image-plane sharding for multi-GPU runs over a side-wide, height-tall image: block x block pixel
    tiles dealt round-robin (tile k -> rank k % world), each tile walked in 8x8 sub-tiles (one 64-ray
    wavefront each).  A rank's tiles are listed nearest the image centre first: the lens-hitting tiles,
    whose waves run longest, are dispatched first and the frame ends on short missing waves (cfg4, one
    frame in flight, scripts/tile_order_probe.py).  order="dealt" keeps the plain dealing order (the probe's
    baseline).  Returns (rows, cols) of this rank's pixels."""
    s = cfg.side if side is None else side
    h = s if height is None else height
    if s % block or h % block:
        raise ValueError("image sides must be multiples of the tile size")
    nbx, nby = s // block, h // block
    tiles = np.arange(nbx * nby)[rank::world]
    dy = (tiles // nbx + 0.5) * block - h / 2
    dx = (tiles % nbx + 0.5) * block - s / 2
    if order == "centre":
        tiles = tiles[np.argsort(dy * dy + dx * dx, kind="stable")]
    elif order != "dealt":
        raise ValueError(f"order {order!r}")
    sub_r, sub_c = pixel_coords(cfg, block, "tiles")
    rows = ((tiles // nbx)[:, None] * block + sub_r[None, :]).reshape(-1)
    cols = ((tiles % nbx)[:, None] * block + sub_c[None, :]).reshape(-1)
    return rows, cols
