"""Multi-GPU frames: image-plane tiles sharded over ranks, traced independently, gathered to rank 0.

One process per GPU (torch.distributed; "nccl" = RCCL over xGMI on MI355X, "gloo" on CPU for tests).
Rays are independent, so the only exchange is the final gather.  The image is
`width` x `height` pixels; 64x64 tiles are dealt round-robin to ranks (configs.shard_pixels) so
every rank gets a similar mix of lens-hitting and missing rays.  A rank's result for one frame is a
packed [8, n] float32 tensor: the 6 ray rows, then status and segment counts as raw 32-bit words.
"""
from __future__ import annotations

import numpy as np

from .configs import Config, rays_for, shard_pixels

PACKED_ROWS = 8


def rank_rays(cfg: Config, rank: int, world: int, width: int, height: int):
    """(rows, cols, rays [6, n]) of this rank's tiles."""
    rows, cols = shard_pixels(cfg, rank, world, side=width, height=height)
    return rows, cols, rays_for(cfg, rows, cols, side=width, height=height)


def pack(out_rays, out_status, out_segments, packed):
    """Write one frame's results into `packed` [8, n] (torch tensors, same device)."""
    import torch

    packed[:6].copy_(out_rays)
    packed[6].copy_(out_status.view(torch.float32))
    packed[7].copy_(out_segments.view(torch.float32))
    return packed


def gather(packed, world: int, rank: int, dst: int = 0, gather_list=None):
    """Gather every rank's packed frame on `dst` (collective; all ranks call it)."""
    import torch.distributed as dist

    if world == 1:
        return [packed]
    dist.gather(packed, gather_list if rank == dst else None, dst=dst)
    return gather_list if rank == dst else None


def assemble(parts, cfg: Config, world: int, width: int, height: int):
    """Rank 0: scatter the gathered per-rank results into full-image arrays
    (rays [6, height*width] float32, status and segments [height*width] uint32), row-major pixels."""
    rays = np.zeros((6, height * width), np.float32)
    status = np.zeros(height * width, np.uint32)
    seg = np.zeros(height * width, np.uint32)
    for r, part in enumerate(parts):
        p = part.cpu().numpy() if hasattr(part, "cpu") else np.asarray(part)
        rows, cols = shard_pixels(cfg, r, world, side=width, height=height)
        flat = rows * width + cols
        rays[:, flat] = p[:6]
        status[flat] = p[6].view(np.uint32)
        seg[flat] = p[7].view(np.uint32)
    return rays, status, seg
