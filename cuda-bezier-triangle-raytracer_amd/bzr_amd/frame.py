"""Multi-GPU frames: image-plane tiles sharded over ranks, traced independently, gathered to rank 0.

One process per GPU (torch.distributed; "nccl" = RCCL over xGMI on MI355X, "gloo" on CPU for tests).
Rays are independent, so the only exchange is the final gather.  The image is
`width` x `height` pixels; 64x64 tiles are dealt round-robin to ranks (configs.shard_pixels) so
every rank gets a similar mix of lens-hitting and missing rays.  Strong scaling keeps the image fixed as
ranks are added (bench.py's default); weak scaling grows it with the rank count.  A rank's result for one
frame is packed into a float32 tensor whose last row holds one raw 32-bit word per ray: the status (bits
0-7) and the segment count (bits 8-15).  Three layouts cross xGMI:
  rays     [7, n]: the 6 final-ray rows + the word (28 B per primary) -- every ray result on rank 0;
  compact  every ray result on rank 0 in ~16.5 B per primary (cfg4): one byte per primary (status | segments
           << 2), a survivor count, and the final rays of the survivors only -- the primaries that refracted
           at least once (64.7 % on cfg4); a ray that missed its first lens leaves the chain unchanged, so
           rank 0 regenerates it from the pixel (configs.rays_for).  Survivors are packed on the device
           (prefix sum + scatter, no host sync) into a fixed capacity per rank (compact_capacity); a frame
           with more survivors than that is reported by assemble(), never truncated silently;
  image    [1, n]: the word only (4 B per primary) -- the frame's status/segment image on rank 0, the final
           rays staying in each rank's HBM.
FrameLoop is the frames-in-flight x double-buffered asynchronous gather loop bench.py runs (and
tests/test_distributed.py drives on CPU with gloo and the oracle as the tracer).
"""
from __future__ import annotations

import numpy as np

from .configs import Config, rays_for, shard_pixels

PACKED_ROWS = 7
IMAGE_ROWS = 1
TILE = 64  # pixels per tile side
LAYOUTS = ("image", "rays", "compact")


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


def assemble(parts, cfg: Config, world: int, width: int, height: int, cap: int = 0):
    """Rank 0: scatter the gathered per-rank results into full-image arrays (rays [6, height*width]
    float32 -- None for the image layout --, status and segments [height*width] uint32), row-major pixels.
    Compact-layout parts (1-D) need the capacity `cap` they were packed with."""
    rays = None
    status = np.zeros(height * width, np.uint32)
    seg = np.zeros(height * width, np.uint32)
    for r, part in enumerate(parts):
        p = part.cpu().numpy() if hasattr(part, "cpu") else np.asarray(part)
        rows, cols = shard_pixels(cfg, r, world, side=width, height=height, block=TILE)
        flat = rows * width + cols
        if p.ndim == 1:  # compact layout
            prim = rays_for(cfg, rows, cols, side=width, height=height)
            rr, st, sg = unpack_compact(p, len(flat), padded_count(world, width, height), cap, prim)
            if rays is None:
                rays = np.zeros((6, height * width), np.float32)
            rays[:, flat], status[flat], seg[flat] = rr, st, sg
            continue
        p = p[:, :len(flat)]  # drop the padding
        if p.shape[0] == PACKED_ROWS:
            if rays is None:
                rays = np.zeros((6, height * width), np.float32)
            rays[:, flat] = p[:6]
        word = np.ascontiguousarray(p[-1]).view(np.uint32)
        status[flat] = word & 0xFF
        seg[flat] = (word >> 8) & 0xFF
    return rays, status, seg


def assemble_hits(parts, cfg: Config, world: int, width: int, height: int):
    """Rank 0, intersect configs: the gathered parts -> the full image's BezierIntersection rows, row-major
    pixels: hits [13, height*width] (the rays layout, 13 rows per rank) or, for the image layout (one row: the
    hit's `what` word), what [height*width] uint32."""
    out = None
    for r, part in enumerate(parts):
        p = part.cpu().numpy() if hasattr(part, "cpu") else np.asarray(part)
        rows, cols = shard_pixels(cfg, r, world, side=width, height=height, block=TILE)
        flat = rows * width + cols
        p = np.ascontiguousarray(p[:, :len(flat)]).view(np.uint32)
        if out is None:
            out = np.zeros((p.shape[0], height * width), np.uint32)
        out[:, flat] = p
    return out if out.shape[0] > 1 else out[0]


def verify_gathered(parts, layout: str, cfg: Config, world: int, width: int, height: int, want: dict, cap: int = 0):
    """Rank 0: one gathered frame against `want`, the same frame traced in one process (full-image arrays in
    row-major pixel order: chain configs "rays" [6, HW], "status", "segments"; intersect configs "hits"
    [13, HW]).  Bit-for-bit on every word the layout carries (the image layout: the status / segment word, or
    the hit's `what`; compact and rays: the final rays too).  Returns {"ok", "mismatched_pixels", "compared",
    "survivors_max" (compact: the largest rank's survivor count word), "cap", "error"}; a compact part whose
    survivors exceed the capacity or disagree with its count word fails with that error."""
    res = {"ok": False, "mismatched_pixels": None, "compared": None, "survivors_max": None,
           "cap": cap if layout == "compact" else None, "error": None}
    if layout == "compact":
        nw = compact_words(padded_count(world, width, height))
        res["survivors_max"] = max(int(np.ascontiguousarray((p.cpu().numpy() if hasattr(p, "cpu") else np.asarray(p))
                                                           [nw:nw + 1]).view(np.int32)[0]) for p in parts)
    bad = np.zeros(height * width, bool)
    try:
        if "hits" in want:
            got = assemble_hits(parts, cfg, world, width, height)
            ref = np.ascontiguousarray(want["hits"]).view(np.uint32)
            if got.ndim == 1:
                bad |= got != ref[11]
                res["compared"] = ["what"]
            else:
                bad |= (got != ref).any(axis=0)
                res["compared"] = ["hits[13]"]
        else:
            rays, status, seg = assemble(parts, cfg, world, width, height, cap=cap)
            bad |= status != np.asarray(want["status"], np.uint32)
            bad |= seg != np.asarray(want["segments"], np.uint32)
            res["compared"] = ["status", "segments"]
            if rays is not None:
                bad |= (rays.view(np.uint32) != np.ascontiguousarray(want["rays"]).view(np.uint32)).any(axis=0)
                res["compared"].append("rays[6]")
    except RuntimeError as e:  # compact capacity / count mismatch (unpack_compact)
        res["error"] = str(e)
        return res
    res["mismatched_pixels"] = int(bad.sum())
    res["ok"] = res["mismatched_pixels"] == 0
    return res


# ------------------------------------------------------------------ compact layout
def compact_words(npad: int) -> int:
    """int32 words holding one status/segments byte per primary (npad is a multiple of 4096)."""
    return npad // 4


def compact_size(npad: int, cap: int) -> int:
    """float32 elements of one rank's compact buffer: byte words, the survivor count, 6 x (cap + 1) ray
    floats (column cap is the scatter's dump column for rays that are not survivors)."""
    return compact_words(npad) + 1 + 6 * (cap + 1)


def survivors(status, segments):
    """Primaries whose final ray differs from the primary ray: refracted at least once."""
    return (segments >= 2) | (status != 0)


def compact_capacity(count: int, npad: int) -> int:
    """Survivor capacity per rank for a frame whose largest rank has `count` survivors: a little headroom
    (1/64 + 64 rays), at most the padded share."""
    return min(npad, count + count // 64 + 64)


def pack_compact(out_status, out_segments, out_rays, packed, npad: int, cap: int):
    """One frame into the 1-D compact buffer `packed` (torch, float32, compact_size(npad, cap) elements) on
    the device, without a host sync: bytes, count, then survivors in index order (prefix sum + scatter)."""
    import torch

    n = out_status.shape[0]
    nw = compact_words(npad)
    st = out_status.to(torch.int32)
    sg = out_segments.to(torch.int32)
    packed[:nw].view(torch.uint8)[:n].copy_(((st & 3) | (sg << 2)).to(torch.uint8))
    alive = survivors(st, sg)
    pos = torch.cumsum(alive.to(torch.int64), 0) - 1
    packed[nw:nw + 1].view(torch.int32).copy_(alive.sum().to(torch.int32).reshape(1))
    idx = torch.where(alive & (pos < cap), pos, torch.full_like(pos, cap))
    packed[nw + 1:].view(6, cap + 1).index_copy_(1, idx, out_rays)
    return packed


def unpack_compact(part, n: int, npad: int, cap: int, primaries):
    """Rank 0: one rank's compact buffer -> (rays [6, n], status [n], segments [n]); `primaries` [6, n]
    are that rank's primary rays (regenerated from the pixels).  Raises if the rank had more survivors
    than the capacity (its frame was not fully gathered)."""
    p = part.cpu().numpy() if hasattr(part, "cpu") else np.asarray(part)
    nw = compact_words(npad)
    b = np.ascontiguousarray(p[:nw]).view(np.uint8)[:n]
    status = (b & 3).astype(np.uint32)
    seg = (b >> 2).astype(np.uint32)
    count = int(np.ascontiguousarray(p[nw:nw + 1]).view(np.int32)[0])
    alive = survivors(status, seg)
    if count > cap or count != int(alive.sum()):
        raise RuntimeError(f"compact gather: {count} survivors for a capacity of {cap} "
                           f"({int(alive.sum())} flagged): the frame was not fully gathered")
    rays = np.array(primaries, dtype=np.float32, copy=True)
    rays[:, alive] = p[nw + 1:].reshape(6, cap + 1)[:, :count]
    return rays, status, seg


# ------------------------------------------------------------------ the frame loop
class FrameLoop:
    """Frames in flight x double-buffered asynchronous gather (bench.py's multi-rank loop).

    Frame k runs on slot k % inflight: trace(slot, k) fills outs[slot] = (rays [6, n], status [n],
    segments [n]) on that slot's stream (stream_for(slot) returns a context manager; nullcontext on
    CPU).  With a gather layout the frame is then packed into gather buffer k % 2 -- after that buffer's
    previous gather completed -- and gathered to rank 0 asynchronously, so frame k's gather overlaps
    frame k + 1's tracing.  on_gathered(frame, parts) (rank 0, optional) sees each frame's gathered
    buffers when its handle is waited for (the next use of the buffer, or drain()).  pack_fn(outs[slot], packed,
    slot), when given, packs instead of pack() / pack_compact() (bench.py: bzr_amd.pack_frame on the slot's
    context, one HIP kernel instead of a dozen torch ops; or the intersect configs' hit rows).  pack_always packs every
    frame even with world == 1 (no collective: scripts/rank_loop_probe.py times one rank's loop that way)."""

    def __init__(self, world: int, rank: int, n: int, npad: int, layout: str, trace, outs, stream_for=None,
                 cap: int = 0, device=None, on_gathered=None, pack_fn=None, rows: int = 0, pack_always: bool = False):
        import contextlib

        import torch

        if layout not in LAYOUTS + ("none",):
            raise ValueError(f"layout {layout!r}")
        self.world, self.rank, self.n, self.npad, self.layout = world, rank, n, npad, layout
        self.trace, self.outs = trace, outs
        self.stream_for = stream_for or (lambda f: contextlib.nullcontext())
        self.cap, self.on_gathered, self.pack_fn = cap, on_gathered, pack_fn
        self.gather_on = (world > 1 or pack_always) and layout != "none"
        self.frames = 0
        self.pending = [None, None]
        self.pending_frame = [-1, -1]
        if layout == "compact" and not 0 < cap <= npad:
            raise ValueError("compact layout needs 0 < cap <= npad")
        shape = {"image": (IMAGE_ROWS, npad), "rays": (rows or PACKED_ROWS, npad),
                 "compact": (compact_size(npad, cap),), "none": (1,)}[layout]
        self.packed = [torch.zeros(shape, dtype=torch.float32, device=device) for _ in range(2)] if self.gather_on else None
        self.lists = [[torch.empty_like(self.packed[0]) for _ in range(world)] if (self.gather_on and rank == 0) else None
                      for _ in range(2)]

    @property
    def bytes_per_rank(self) -> int:
        return 0 if not self.gather_on else self.packed[0].numel() * 4

    def _finish(self, slot):
        if self.pending[slot] is not None:
            self.pending[slot].wait()
            self.pending[slot] = None
            if self.on_gathered is not None and self.rank == 0:
                self.on_gathered(self.pending_frame[slot], self.lists[slot])

    def step(self, inflight: int):
        f = self.frames % inflight
        with self.stream_for(f):
            self.trace(f, self.frames)
            if self.gather_on:
                slot = self.frames % 2
                self._finish(slot)
                if self.pack_fn is not None:  # a device packer (bzr_amd.pack_frame) or other result shapes
                    self.pack_fn(self.outs[f], self.packed[slot], f)
                elif self.layout == "compact":
                    rays, status, seg = self.outs[f]
                    pack_compact(status, seg, rays, self.packed[slot], self.npad, self.cap)
                else:
                    pack(*self.outs[f], self.packed[slot])
                self.pending[slot] = gather(self.packed[slot], self.world, self.rank, gather_list=self.lists[slot],
                                            async_op=True)
                self.pending_frame[slot] = self.frames
        self.frames += 1

    def drain(self):
        for slot in sorted(range(2), key=lambda k: self.pending_frame[k]):
            self._finish(slot)
