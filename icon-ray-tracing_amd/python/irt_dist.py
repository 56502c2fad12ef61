"""irt_dist -- multi-GPU frame splitting for the ICON renderer (one process per GPU).

The reference is single-device; its CPU path already cuts a frame into 64x64 tiles pulled
by a thread pool (common/for_each.h:70-85, common/thread_pool.h:146-161).  Here the same
tiles are dealt to N ranks by estimated cost (irt_deal_tiles: a longest-processing-time
greedy deal -- tiles sorted by the estimated cost of their rays through the shell, longest
first, each given to the least-loaded rank, rank 0 preloaded with its unpack share -- so
every rank's share costs about the same; the plain round-robin t -> rank t mod N hands whole tile COLUMNS to each rank when N divides
the tile row, ~1.6x cost spread over a centred globe), every rank renders its tiles into a
packed buffer (irt_render_tile_list), and rank 0 gathers the RGBA8 tiles over RCCL
(torch.distributed, backend "nccl") and scatters them into the framebuffer
(irt_unpack_tile_table).  Pixel seeds
depend only on (accumID, W, H, x, y) (deviceCode.cu:288-289), so the assembled frame is
bit-identical to a single-GPU launch.  The accumulation buffer stays sharded: each rank
keeps the accum of its own tiles across frames (progressive rendering needs no exchange).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

TILE = 64
TILE_PIX = TILE * TILE
# irt_unpack_tile_table of a whole frame against one frame's render on one GPU: ~4.5 us vs
# 0.104 ms at C3, ~8.5 us vs 0.33 ms at C4 (profiles/r03b_dist/): rank 0's extra work per
# step, as a fraction of a frame's render cost
UNPACK_COST = 0.04


@dataclass(frozen=True, eq=False)
class TileSplit:
    """Which 64x64 tiles each rank renders.  `table` (world, max_tiles) from irt_deal_tiles
    (row r = rank r's tiles in render order, -1 padding); None: round-robin t mod world."""
    width: int
    height: int
    rank: int
    world: int
    table: np.ndarray | None = None

    @classmethod
    def dealt(cls, width: int, height: int, rank: int, world: int, lp, info,
              frames: int = 1) -> "TileSplit":
        """The cost-balanced deal for the camera lp over the volume `info` (every rank
        computes the same table: a deterministic function of its inputs).  With more than
        one rank, rank 0 also unpacks the gathered frame once per step of `frames` frames:
        UNPACK_COST of one frame's render cost, taken off its tiles."""
        import irt
        extra = UNPACK_COST / max(1, frames) if world > 1 else 0.0
        return cls(width, height, rank, world,
                   irt.deal_tiles(lp, info, width, height, world, extra))

    @property
    def tiles_x(self) -> int:
        return (self.width + TILE - 1) // TILE

    @property
    def num_tiles(self) -> int:
        return self.tiles_x * ((self.height + TILE - 1) // TILE)

    @property
    def max_tiles(self) -> int:
        if self.table is not None:
            return int(self.table.shape[1])
        return (self.num_tiles + self.world - 1) // self.world

    def tiles(self, rank: int | None = None) -> list[int]:
        r = self.rank if rank is None else rank
        if self.table is not None:
            return [int(t) for t in self.table[r] if t >= 0]
        return list(range(r, self.num_tiles, self.world))

    def render(self, ctx, lp, frames: int, buf_ptr: int, acc_ptr: int, stream: int = 0):
        """This rank's tiles of `frames` progressive frames (accumID = lp.accumID ...) into
        the packed buffer buf_ptr (accum tiles acc_ptr)."""
        if self.table is not None:
            ctx.render_tile_list(lp, self.width, self.height, self.tiles(), frames, buf_ptr,
                                 acc_ptr, stream)
        elif frames == 1:
            ctx.render_tiles(lp, self.width, self.height, self.rank, self.world, buf_ptr,
                             acc_ptr, stream)
        else:
            ctx.render_tiles_accumulate(lp, self.width, self.height, self.rank, self.world,
                                        frames, buf_ptr, acc_ptr, stream)

    def render_sequence(self, ctx, lps, buf_ptr: int, acc_ptr: int, stream: int = 0):
        """This rank's tiles of the views lps[0..] (a camera path, one launch) into the packed
        buffer buf_ptr (accum tiles acc_ptr)."""
        ctx.render_tile_list_sequence(lps, self.width, self.height, self.tiles(), buf_ptr, acc_ptr, stream)

    def unpack(self, ctx, gathered_ptr: int, fb_ptr: int, stream: int = 0):
        """Rank 0: every rank's packed tiles (gathered rank-major) into the framebuffer."""
        if self.table is not None:
            ctx.unpack_tile_table(gathered_ptr, self.table, self.width, self.height, fb_ptr,
                                  stream)
        else:
            ctx.unpack_tiles(gathered_ptr, self.world, self.max_tiles, self.width, self.height,
                             fb_ptr, stream)

    def tile_pixels(self, tile: int) -> np.ndarray:
        """(x, y) of the in-frame pixels of a tile, in packed (ly*64 + lx) order, with -1
        for pixels past the frame edge."""
        tx, ty = tile % self.tiles_x, tile // self.tiles_x
        ly, lx = np.mgrid[0:TILE, 0:TILE]
        x, y = tx * TILE + lx.ravel(), ty * TILE + ly.ravel()
        inside = (x < self.width) & (y < self.height)
        return np.stack([np.where(inside, x, -1), np.where(inside, y, -1)], 1)


def unpack_host(gathered: np.ndarray, split: TileSplit) -> np.ndarray:
    """Host twin of irt_unpack_tiles: rank-major packed tiles -> (H, W) framebuffer."""
    fb = np.zeros((split.height, split.width), dtype=gathered.dtype)
    g = gathered.reshape(split.world, split.max_tiles, TILE_PIX)
    for r in range(split.world):
        for k, t in enumerate(split.tiles(r)):
            xy = split.tile_pixels(t)
            ok = xy[:, 0] >= 0
            fb[xy[ok, 1], xy[ok, 0]] = g[r, k, ok]
    return fb


class FrameGather:
    """Per-frame RCCL gather of packed RGBA8 tiles to rank 0 (torch.distributed).

    Rank 0 receives straight into rank-major storage: the gather list is the per-rank rows
    of one preallocated (world, tiles) tensor (contiguous views, so the collective writes
    them in place and no concatenation copy follows).  `buffers` > 1 double-buffers the
    packed tiles so that the gather of frame s can run (async_op, on the collective's own
    stream) while frame s+1 renders into the other buffer: gather_async() returns a
    pending handle, finish() waits for it (making the current stream wait, not the host)
    and on rank 0 returns the rank-major frame."""

    def __init__(self, split: TileSplit, device, buffers: int = 1, stage_cpu: bool = False):
        import torch
        import torch.distributed as dist
        self.dist, self.torch, self.split = dist, torch, split
        self.stage_cpu = stage_cpu  # gloo rehearsal of the GPU path: collectives on host copies
        n = split.max_tiles * TILE_PIX
        cdev = "cpu" if stage_cpu else device
        self.bufs = [torch.zeros(n, dtype=torch.int32, device=device) for _ in range(buffers)]
        if split.rank == 0:
            self.gathered = [torch.zeros(split.world * n, dtype=torch.int32, device=device)
                             for _ in range(buffers)]
            recv = (self.gathered if not stage_cpu else
                    [torch.zeros(split.world * n, dtype=torch.int32, device=cdev)
                     for _ in range(buffers)])
            self.recv = recv
            self.parts = [list(r.view(split.world, n).unbind(0)) for r in recv]
        else:
            self.gathered = self.recv = self.parts = None
        self.tiles = self.bufs[0]

    def gather_async(self, b: int = 0):
        src = self.bufs[b].cpu() if self.stage_cpu else self.bufs[b]
        return self.dist.gather(src, self.parts[b] if self.parts else None, dst=0,
                                async_op=True)

    def finish(self, work, b: int = 0):
        work.wait()
        if self.split.rank != 0:
            return None
        if self.stage_cpu:  # host-staged rehearsal: one copy of the gathered frame to HBM
            self.gathered[b].copy_(self.recv[b])
        return self.gathered[b]

    def gather(self):
        """Collective: every rank calls it after rendering into self.tiles.  On rank 0
        returns the rank-major gathered tensor, elsewhere None."""
        return self.finish(self.gather_async(0), 0)


class FramePipeline:
    """The multi-rank step loop bench.py runs (and tests/test_gpu_distributed.py checks).
    Step s renders this rank's tiles into packed buffer b = s mod 2K on the current (render)
    stream and starts the RCCL gather of that buffer; K = `batch`.
      * Buffer reuse: the render into b must follow the gather that read b 2K steps earlier.
        Gathers of one process group run in order on one collective stream, so the render
        stream waits once per K steps, on the newest gather of the previous half-cycle,
        instead of once per step: each cross-queue wait costs the render stream ~20 us of
        idle time per step (profiles/r02j_dist/), more than the unpack it used to carry.
      * Rank 0 issues its gathers from a side stream, which also waits for each received
        frame and unpacks it into the framebuffer (in step order: the framebuffer ends with
        the newest frame), overlapping the renders; the next gather into a receive buffer
        follows that buffer's unpack on the same stream."""

    def __init__(self, ctx, fg: FrameGather, fb, batch: int = 4):
        import torch
        self.torch, self.ctx, self.fg, self.fb = torch, ctx, fg, fb
        self.split = fg.split
        self.k = max(1, batch)
        assert len(fg.bufs) == 2 * self.k, "FrameGather needs buffers = 2 * batch"
        self.works = {}    # step -> pending gather
        self.pending = []  # rank 0: steps gathered, not yet unpacked (oldest first)
        self.rank0 = self.split.rank == 0
        self.side = torch.cuda.Stream() if self.rank0 else None
        self.host_staged = fg.stage_cpu

    def _unpack_upto(self, last):
        """Rank 0, side stream: wait for and unpack the frames of steps <= last."""
        torch, sp = self.torch, self.split
        while self.pending and self.pending[0] <= last:
            t = self.pending.pop(0)
            b = t % len(self.fg.bufs)
            with torch.cuda.stream(self.side):
                g = self.fg.finish(self.works[t], b)
                sp.unpack(self.ctx, g.data_ptr(), self.fb.data_ptr(), self.side.cuda_stream)

    def _wait_reuse(self, t):
        """The render stream waits for the gather of step t (it read the buffers about to
        be rendered into again)."""
        self.works[t].wait()

    def step(self, s: int, render):
        """render(buf): this rank's tiles of step s into the packed buffer `buf`."""
        torch = self.torch
        nb = len(self.fg.bufs)
        b = s % nb
        if b % self.k == 0:  # buffers b .. b+K-1 were last read by the gathers s-2K .. s-K-1
            newest = s - self.k - 1
            for t in [t for t in self.works if t <= newest]:
                if t == newest or self.host_staged:
                    self._wait_reuse(t)  # the render stream (in-order collectives: one wait)
                if not self.rank0:
                    del self.works[t]
        if self.rank0:
            self._unpack_upto(s - 2)
            for t in [t for t in self.works if t <= s - 2 * self.k]:
                del self.works[t]
        render(self.fg.bufs[b])
        if self.rank0:  # ordered after this render and after earlier unpacks of gathered[b]
            self.side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self.side):
                self.works[s] = self.fg.gather_async(b)
            self.pending.append(s)
        else:
            self.works[s] = self.fg.gather_async(b)

    def drain(self):
        """Finish every gather in flight and unpack the frames still pending, oldest first."""
        torch = self.torch
        last = max(self.works) if self.works else -1
        if self.rank0:
            self._unpack_upto(last)
            torch.cuda.current_stream().wait_stream(self.side)
        for t in sorted(self.works):
            self.works[t].wait()
        self.works.clear()
