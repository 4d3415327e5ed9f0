"""Multi-GPU frames: image-plane tiles sharded over ranks, traced independently, gathered to rank 0.

One process per GPU (torch.distributed; "nccl" = RCCL over xGMI on MI355X, "gloo" on CPU for tests).
Rays are independent, so the only exchange is the final gather.  The image is
`width` x `height` pixels; 64x64 tiles are dealt round-robin to ranks (configs.shard_pixels) so
every rank gets a similar mix of lens-hitting and missing rays.  Strong scaling keeps the image fixed as
ranks are added (bench.py's default); weak scaling grows it with the rank count.  A rank's result for one
frame is packed into a float32 tensor whose last row holds one raw 32-bit word per ray: the status (bits
0-7) and the segment count (bits 8-15).  Two layouts cross xGMI:
  rays   [7, n]: the 6 final-ray rows + the word (28 B per primary) -- every ray result on rank 0;
  image  [1, n]: the word only (4 B per primary) -- the frame's status/segment image on rank 0, the final
         rays staying in each rank's HBM.
"""
from __future__ import annotations

import numpy as np

from .configs import Config, rays_for, shard_pixels

PACKED_ROWS = 7
IMAGE_ROWS = 1
TILE = 64  # pixels per tile side


def rank_rays(cfg: Config, rank: int, world: int, width: int, height: int):
    """(rows, cols, rays [6, n]) of this rank's tiles."""
    rows, cols = shard_pixels(cfg, rank, world, side=width, height=height, block=TILE)
    return rows, cols, rays_for(cfg, rows, cols, side=width, height=height)


def padded_count(world: int, width: int, height: int) -> int:
    """Pixels per rank in the gather buffers: the largest rank's share (tiles are dealt round-robin, so a
    fixed image whose tile count is not a multiple of `world` leaves some ranks one tile short)."""
    tiles = (width // TILE) * (height // TILE)
    return -(-tiles // world) * TILE * TILE


def pack(out_rays, out_status, out_segments, packed):
    """Write one frame's results into the first n columns of `packed` (torch tensors, same device):
    [7, >= n] (rays layout) or [1, >= n] (image layout; out_rays is not read and may be None).  The
    columns past n are padding (padded_count) and are not read by assemble()."""
    import torch

    n = out_status.shape[0]
    if packed.shape[0] == PACKED_ROWS:
        packed[:6, :n].copy_(out_rays)
    word = out_status.to(torch.int32) | (out_segments.to(torch.int32) << 8)
    packed[-1, :n].copy_(word.view(torch.float32))
    return packed


def gather(packed, world: int, rank: int, dst: int = 0, gather_list=None, async_op: bool = False):
    """Gather every rank's packed frame on `dst` (collective; all ranks call it).  With async_op the
    collective's work handle is returned instead: the caller waits on it before reusing `packed`."""
    import torch.distributed as dist

    if world == 1:
        return None if async_op else [packed]
    work = dist.gather(packed, gather_list if rank == dst else None, dst=dst, async_op=async_op)
    if async_op:
        return work
    return gather_list if rank == dst else None


def assemble(parts, cfg: Config, world: int, width: int, height: int):
    """Rank 0: scatter the gathered per-rank results into full-image arrays (rays [6, height*width]
    float32 -- None for the image layout --, status and segments [height*width] uint32), row-major pixels."""
    rays = None
    status = np.zeros(height * width, np.uint32)
    seg = np.zeros(height * width, np.uint32)
    for r, part in enumerate(parts):
        p = part.cpu().numpy() if hasattr(part, "cpu") else np.asarray(part)
        rows, cols = shard_pixels(cfg, r, world, side=width, height=height, block=TILE)
        flat = rows * width + cols
        p = p[:, :len(flat)]  # drop the padding
        if p.shape[0] == PACKED_ROWS:
            if rays is None:
                rays = np.zeros((6, height * width), np.float32)
            rays[:, flat] = p[:6]
        word = np.ascontiguousarray(p[-1]).view(np.uint32)
        status[flat] = word & 0xFF
        seg[flat] = (word >> 8) & 0xFF
    return rays, status, seg
