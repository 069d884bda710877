"""Tile sharding of one frame across ranks (one process per GPU) with a gather to rank 0.

Layout contract (shared with libvpx_hip.so's vpx_render_tiles / vpx_composite_tiles):
  - the frame is cut into 16x16 tiles in row-major tile order, t = ty * tiles_x + tx;
  - tile t belongs to rank t % R (round-robin: spatially uneven cost is spread evenly);
  - a rank's packed buffer holds its tiles in increasing t, 256 float4 each in lane order
    (tile_lanes: the tile's four 8x8 quadrants in row-major order, row-major inside each —
    one wave each), edge tiles zero-padded; every rank's buffer has the same length
    ceil(num_tiles / R) * 256 so the gather is one fixed-size collective;
  - rank 0 receives the R buffers back to back and composites them (unpack + running-
    average accumulate + tonemap) into its accumulator and RGB8 screen.
There is one exchange per frame (the gather); the world is replicated per GPU.  Over
RCCL (torch.distributed backend "nccl") the gather is R-1 point-to-point transfers into
rank 0, each on its own xGMI link on an MI355X node.

Two flows share that layout:
  - ShardedFrame: ranks send raw float4 samples (16 B/pixel); rank 0 owns the whole
    accumulator and composites (vpx_render_tiles + vpx_composite_tiles).
  - ShardedAccumFrame (bench default): the accumulator is sharded with the tiles — each
    rank keeps the running average of its own pixels and tonemaps them
    (vpx_render_tiles_accum), so only packed RGB8 (4 B/pixel) travels, and rank 0 only
    scatters it into the screen (vpx_composite_rgb8).  The gather of frame f is issued
    asynchronously and overlaps the render of frame f+1 (double-buffered RGB8).  Screen and
    accumulator values are bit-identical to the single-GPU frame.
"""
import numpy as np

TILE = 16


def tiles_xy(width, height):
    return (width + TILE - 1) // TILE, (height + TILE - 1) // TILE


def packed_len(width, height, n_ranks):
    """float4 elements per rank buffer (== vpx_tiles_packed_len)."""
    tx, ty = tiles_xy(width, height)
    return -(-(tx * ty) // n_ranks) * TILE * TILE


def tile_lanes():
    """(lx, ly) of a tile's 256 entries in packed order (csrc tile_lane_xy)."""
    lane = np.arange(TILE * TILE)
    return ((lane >> 6) & 1) * 8 + (lane & 7), (lane >> 7) * 8 + ((lane >> 3) & 7)


def rank_pixel_ids(width, height, rank, n_ranks):
    """Pixel ids (y*W + x) in packed order for one rank; -1 marks padding."""
    tx, ty = tiles_xy(width, height)
    tiles = np.arange(rank, tx * ty, n_ranks)
    lx, ly = tile_lanes()
    x = (tiles % tx)[:, None] * TILE + lx[None, :]
    y = (tiles // tx)[:, None] * TILE + ly[None, :]
    ids = np.where((x < width) & (y < height), y * width + x, -1).reshape(-1)
    out = np.full(packed_len(width, height, n_ranks), -1, np.int64)
    out[: ids.size] = ids
    return out


def pack(samples4, width, height, rank, n_ranks):
    """Host reference of a rank's packed buffer from a full-frame float4 sample image."""
    ids = rank_pixel_ids(width, height, rank, n_ranks)
    out = np.zeros((ids.size, 4), np.float32)
    ok = ids >= 0
    out[ok] = np.asarray(samples4, np.float32).reshape(-1, 4)[ids[ok]]
    return out


def unpack(gathered, width, height, n_ranks):
    """Host reference of vpx_composite_tiles' unpack step: R packed buffers -> image."""
    L = packed_len(width, height, n_ranks)
    g = np.asarray(gathered, np.float32).reshape(n_ranks, L, 4)
    img = np.zeros((width * height, 4), np.float32)
    for r in range(n_ranks):
        ids = rank_pixel_ids(width, height, r, n_ranks)
        ok = ids >= 0
        img[ids[ok]] = g[r][ok]
    return img


def unpack_u32(gathered, width, height, n_ranks):
    """Host reference of vpx_composite_rgb8: R packed uint32 buffers -> W*H screen."""
    L = packed_len(width, height, n_ranks)
    g = np.asarray(gathered).view(np.uint32).reshape(n_ranks, L)
    img = np.zeros(width * height, np.uint32)
    for r in range(n_ranks):
        ids = rank_pixel_ids(width, height, r, n_ranks)
        ok = ids >= 0
        img[ids[ok]] = g[r][ok]
    return img


def gather_async(buf, rank, n_ranks, out_parts=None, group=None):
    """Start the gather of every rank's packed buffer into rank 0's `out_parts` (list of
    R tensors, rank 0 only).  Returns the torch.distributed work handle: RCCL runs it on
    its own stream, so the caller's stream keeps rendering until work.wait()."""
    import torch.distributed as dist

    return dist.gather(buf, out_parts if rank == 0 else None, dst=0, group=group, async_op=True)


def gather_tiles(packed, rank, n_ranks, out=None, group=None):
    """Gather every rank's packed tensor to rank 0 (torch.distributed; RCCL on GPUs,
    gloo on CPU).  Returns the concatenated [R*L*4] tensor on rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist

    if n_ranks == 1:
        return packed
    if rank == 0:
        parts = [torch.empty_like(packed) for _ in range(n_ranks)]
        dist.gather(packed, parts, dst=0, group=group)
        if out is None:
            return torch.cat(parts)
        torch.cat(parts, out=out)
        return out
    dist.gather(packed, None, dst=0, group=group)
    return None


class ShardedFrame:
    """One rank's share of the tile-sharded render (GPU path: libvpx_hip.so + RCCL)."""

    def __init__(self, ctx, desc, rank, n_ranks, device):
        import torch

        self.ctx, self.desc, self.rank, self.n = ctx, desc, rank, n_ranks
        w, h = desc.width, desc.height
        self.L = ctx.packed_len(w, h, n_ranks)
        assert self.L == packed_len(w, h, n_ranks)
        self.packed = torch.zeros(self.L * 4, dtype=torch.float32, device=device)
        self.gathered = torch.empty(n_ranks * self.L * 4, dtype=torch.float32, device=device) if rank == 0 else None
        self.accum = torch.zeros(w * h * 4, dtype=torch.float32, device=device) if rank == 0 else None
        self.screen = torch.zeros(w * h, dtype=torch.int32, device=device) if rank == 0 else None
        self.frame = 0

    def step(self):
        p = self.desc.frame_params(frame_index=self.frame)
        self.ctx.render_tiles(p, self.rank, self.n, self.packed.data_ptr())
        g = gather_tiles(self.packed, self.rank, self.n, out=self.gathered)
        if self.rank == 0:
            self.ctx.composite_tiles(p, self.n, g.data_ptr(), self.accum.data_ptr(), self.screen.data_ptr())
        self.frame += 1


class ShardedAccumFrame:
    """One rank's share with the accumulator sharded (see the module docstring).  GPU
    path: libvpx_hip.so + RCCL; `host_gather=True` routes the gather through host memory
    (gloo), for rehearsing N ranks on one GPU.

    `render(frame)` accumulates one frame of this rank's tiles; `publish()` starts the
    gather of the RGB8 of the last rendered frame to rank 0 (and completes the previous
    publish, whose gather overlapped the renders since).  An accumulation window of spp
    frames (C4: 16) renders spp times and publishes once; `step()` = one frame + publish.

    The library must launch on torch's current stream: RCCL orders the gather after the
    work queued on that stream, and `work.wait()` orders later renders after the gather."""

    def __init__(self, ctx, desc, rank, n_ranks, device, host_gather=False):
        import torch

        self.ctx, self.desc, self.rank, self.n = ctx, desc, rank, n_ranks
        self.host = host_gather
        if not host_gather:
            cur = torch.cuda.current_stream(device).cuda_stream
            if not cur:  # the library never launches on the null stream (vpx_set_stream(0) = its own)
                raise ValueError("ShardedAccumFrame: torch's current stream is the default (null) stream; "
                                 "make a torch.cuda.Stream() current (torch.cuda.set_stream) and render on it")
            if ctx.stream_handle != cur:
                raise ValueError("ShardedAccumFrame: the vpx context must render on torch's current stream "
                                 "(ctx.set_stream(torch.cuda.current_stream().cuda_stream))")
        w, h = desc.width, desc.height
        self.L = ctx.packed_len(w, h, n_ranks)
        assert self.L == packed_len(w, h, n_ranks)
        self.accum = torch.zeros(self.L * 4, dtype=torch.float32, device=device)  # this rank's pixels
        self.rgb = [torch.zeros(self.L, dtype=torch.int32, device=device) for _ in range(2)]
        if rank == 0:
            self.gathered = [torch.empty(n_ranks * self.L, dtype=torch.int32, device=device) for _ in range(2)]
            self.parts = [list(g.view(n_ranks, self.L)) for g in self.gathered]  # gather straight into place
            self.screen = torch.zeros(w * h, dtype=torch.int32, device=device)
        self.pending = None  # (work, buffer, params) of the frame whose gather is in flight
        self.frame = 0
        self.buf = 0         # RGB8 buffer the renders write (the other one may be in flight)
        self.last = None     # params of the last rendered frame

    def _finish(self):
        work, b, p = self.pending
        self.pending = None
        if work is not None:
            work.wait()  # the render stream waits for the RCCL stream (no host block)
        if self.rank == 0:
            self.ctx.composite_rgb8(p, self.n, self.gathered[b].data_ptr(), self.screen.data_ptr())

    def render(self, frame=None):
        f = self.frame if frame is None else frame
        p = self.desc.frame_params(frame_index=f)
        self.ctx.render_tiles_accum(p, self.rank, self.n, self.accum.data_ptr(), self.rgb[self.buf].data_ptr())
        self.last = p
        self.frame = f + 1

    def render_window(self, first, n_frames):
        """Frames first .. first + n_frames - 1 of this rank's tiles in order: one library call
        (vpx_render_tiles_accum_window, several frames per chain of launches) when the context
        has it, else frame by frame.  Same accumulator and RGB8 as n_frames render() calls."""
        if n_frames <= 0:
            return
        win = getattr(self.ctx, "render_tiles_accum_window", None)
        if win is None:
            for f in range(first, first + n_frames):
                self.render(f)
            return
        p = self.desc.frame_params(frame_index=first)
        win(p, n_frames, self.rank, self.n, self.accum.data_ptr(), self.rgb[self.buf].data_ptr())
        self.last = self.desc.frame_params(frame_index=first + n_frames - 1)
        self.frame = first + n_frames

    def publish(self):
        import torch
        import torch.distributed as dist

        b, p = self.buf, self.last
        if self.pending is not None:
            self._finish()  # the previous publish: its gather overlapped the renders since
        if self.host:
            if self.rgb[b].is_cuda:
                torch.cuda.current_stream().synchronize()
            parts = [torch.empty(self.L, dtype=torch.int32) for _ in range(self.n)] if self.rank == 0 else None
            dist.gather(self.rgb[b].cpu(), parts, dst=0)
            if self.rank == 0:
                self.gathered[b].copy_(torch.cat(parts))
            self.pending = (None, b, p)
        else:
            self.pending = (gather_async(self.rgb[b], self.rank, self.n, self.parts[b] if self.rank == 0 else None),
                            b, p)
        self.buf ^= 1

    def step(self):
        self.render()
        self.publish()

    def flush(self):
        """Complete the last publish (its gather and rank 0's scatter)."""
        if self.pending is not None:
            self._finish()
