"""Multi-rank tile sharding on CPU: world_size 2 over gloo (127.0.0.1).

Exercises dist.py's layout contract and its gather (the same code path runs over RCCL on
GPUs): each rank produces its packed tile buffer — here from the CPU checker standing in
for vpx_render_tiles — the buffers are gathered to rank 0, unpacked and compared with the
monolithic frame bit for bit.
"""
import ctypes as C
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, w, h, q):
    sys.path.insert(0, REPO)
    import __graft_entry__ as entry

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pkg, orc = entry.load_package(), entry.load_oracle()
        desc = pkg.scene.model_scene("monu3", 64, w, h, 1, city_lights=True)
        o = orc.Oracle(pkg.abi, desc)
        ids = pkg.dist.rank_pixel_ids(w, h, rank, world)
        samples, _ = o.render_pixels(desc.frame_params(0), np.maximum(ids, 0), threads=2)
        samples[ids < 0] = 0
        packed = torch.from_numpy(samples.reshape(-1).copy())
        g = pkg.dist.gather_tiles(packed, rank, world)
        if rank == 0:
            img = pkg.dist.unpack(g.numpy(), w, h, world)
            full, _, _ = o.render(desc.frame_params(0), threads=2)
            q.put(bool(np.array_equal(img.view(np.uint32), full.view(np.uint32))))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _worker_rgb8(rank, world, port, w, h, q):
    """Sharded-accumulator flow: each rank owns the accumulator of its tiles and sends only
    packed RGB8; the gather is started asynchronously (double-buffered, one frame in flight)
    exactly as dist.ShardedAccumFrame does."""
    sys.path.insert(0, REPO)
    import __graft_entry__ as entry

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pkg, orc = entry.load_package(), entry.load_oracle()
        desc = pkg.scene.model_scene("monu3", 64, w, h, 1, city_lights=True)
        desc.flags = pkg.abi.VPX_FLAG_AA
        o = orc.Oracle(pkg.abi, desc)
        ids = pkg.dist.rank_pixel_ids(w, h, rank, world)
        L = ids.size
        bufs = [torch.zeros(L, dtype=torch.int32) for _ in range(2)]
        outs = [torch.empty(world * L, dtype=torch.int32) for _ in range(2)]
        acc = None
        pending, ok = None, True
        for f in range(3):
            acc, rgb, _ = o.render(desc.frame_params(f), accum=acc, threads=2)  # stands in for render_tiles_accum
            b = f & 1
            mine = np.zeros(L, np.uint32)
            mine[ids >= 0] = rgb[ids[ids >= 0]]
            bufs[b].copy_(torch.from_numpy(mine.view(np.int32)))
            if pending is not None:
                work, pb, prgb = pending
                work.wait()
                if rank == 0:
                    ok &= bool(np.array_equal(pkg.dist.unpack_u32(outs[pb].numpy(), w, h, world), prgb))
            parts = list(outs[b].view(world, L)) if rank == 0 else None
            pending = (pkg.dist.gather_async(bufs[b], rank, world, parts), b, rgb.copy())
        work, pb, prgb = pending
        work.wait()
        if rank == 0:
            ok &= bool(np.array_equal(pkg.dist.unpack_u32(outs[pb].numpy(), w, h, world), prgb))
            q.put(ok)
        dist.barrier()
    finally:
        dist.destroy_process_group()


class _OracleTileCtx:
    """Stands in for the vpx context on CPU: vpx_render_tiles_accum / vpx_composite_rgb8
    with the oracle's samples, written through the same raw pointers."""

    def __init__(self, pkg, orc, desc):
        self.pkg, self.desc = pkg, desc
        self.o = orc.Oracle(pkg.abi, desc)
        self.stream_handle = None

    def packed_len(self, w, h, n):
        return self.pkg.dist.packed_len(w, h, n)

    def render_tiles_accum(self, p, rank, n, acc_ptr, rgb_ptr):
        w, h = self.desc.width, self.desc.height
        ids = self.pkg.dist.rank_pixel_ids(w, h, rank, n)
        L = ids.size
        acc = np.ctypeslib.as_array((C.c_float * (4 * L)).from_address(acc_ptr)).reshape(L, 4)
        rgb = np.ctypeslib.as_array((C.c_uint32 * L).from_address(rgb_ptr))
        ok = ids >= 0
        sample, _ = self.o.render_pixels(p, ids[ok].astype(np.uint32), threads=2)
        a = np.ascontiguousarray(acc[ok])
        r = np.zeros(int(ok.sum()), np.uint32)
        for k in range(len(r)):
            self.o.lib.oracle_accumulate_tonemap(sample[k].ctypes.data, p.frame_index, a[k].ctypes.data,
                                                 r[k:k + 1].ctypes.data)
        acc[ok] = a
        rgb[ok] = r

    def render_tiles_accum_window(self, p, n_frames, rank, n, acc_ptr, rgb_ptr):
        """vpx_render_tiles_accum_window's contract: frames p.frame_index .. + n_frames - 1 in order."""
        self.window_calls = getattr(self, "window_calls", 0) + 1
        for f in range(p.frame_index, p.frame_index + n_frames):
            self.render_tiles_accum(self.desc.frame_params(f), rank, n, acc_ptr, rgb_ptr)

    def composite_rgb8(self, p, n, gathered_ptr, screen_ptr):
        w, h = self.desc.width, self.desc.height
        L = self.pkg.dist.packed_len(w, h, n)
        g = np.ctypeslib.as_array((C.c_uint32 * (n * L)).from_address(gathered_ptr))
        scr = np.ctypeslib.as_array((C.c_uint32 * (w * h)).from_address(screen_ptr))
        scr[:] = self.pkg.dist.unpack_u32(g, w, h, n)


def _worker_window(rank, world, port, w, h, spp, q):
    """dist.ShardedAccumFrame itself (host gather over gloo): two accumulation windows of
    `spp` frames each, one publish per window (bench.py's C4 step) — the first frame by frame,
    the second as one render_window call (vpx_render_tiles_accum_window); rank 0's screen after
    each flush equals the oracle's whole-frame RGB8 after frame spp - 1."""
    sys.path.insert(0, REPO)
    import __graft_entry__ as entry

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pkg, orc = entry.load_package(), entry.load_oracle()
        desc = pkg.scene.model_scene("monu3", 64, w, h, 1, city_lights=True)
        desc.flags = pkg.abi.VPX_FLAG_AA
        tctx = _OracleTileCtx(pkg, orc, desc)
        fr = pkg.dist.ShardedAccumFrame(tctx, desc, rank, world, torch.device("cpu"), host_gather=True)
        ok = True
        acc = None
        for f in range(spp):
            acc, want, _ = orc.Oracle(pkg.abi, desc).render(desc.frame_params(f), accum=acc, threads=2)
        for win in range(2):
            if win == 0:
                for f in range(spp):
                    fr.render(f)
            else:
                fr.render_window(0, spp)
                ok &= getattr(tctx, "window_calls", 0) == 1 and fr.last.frame_index == spp - 1 and fr.frame == spp
            fr.publish()
            fr.flush()
            if rank == 0:
                ok &= bool(np.array_equal(fr.screen.numpy().view(np.uint32), want))
        if rank == 0:
            q.put(ok)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_sharded_accum_frame_spp_window_two_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    mp.start_processes(_worker_window, args=(2, port, 40, 24, 3, q), nprocs=2, join=True, start_method="spawn")
    assert q.get(timeout=60) is True


def test_sharded_accumulator_rgb8_gather_two_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    mp.start_processes(_worker_rgb8, args=(2, port, 40, 24, q), nprocs=2, join=True, start_method="spawn")
    assert q.get(timeout=60) is True


@pytest.mark.parametrize("wh", [(40, 24), (33, 17)])
def test_gather_two_ranks_gloo(wh):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    mp.start_processes(_worker, args=(2, port, wh[0], wh[1], q), nprocs=2, join=True, start_method="spawn")
    assert q.get(timeout=60) is True


def test_layout_contract(pkg):
    d = pkg.dist
    for (w, h, r) in [(33, 17, 2), (100, 70, 3), (16, 16, 4), (1, 1, 2)]:
        L = d.packed_len(w, h, r)
        assert L == pkg.load_library().vpx_tiles_packed_len(w, h, 16, 16, r)
        seen = np.concatenate([d.rank_pixel_ids(w, h, k, r) for k in range(r)])
        seen = np.sort(seen[seen >= 0])
        assert np.array_equal(seen, np.arange(w * h))  # every pixel exactly once
        img = np.random.default_rng(0).random((w * h, 4)).astype(np.float32)
        packs = np.concatenate([d.pack(img, w, h, k, r) for k in range(r)])
        assert np.array_equal(d.unpack(packs, w, h, r), img)
