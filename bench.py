"""bench.py — Mray/s (primary+shadow) of the MI355X voxel ray-trace path.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C1] [--no-cpu]

A step = one frame of the C1 workload (BASELINE.json configs[1]): 1920x1080, 1024^3 world
(monu3.vox tiled), 1 spp, Trace depth 0 = primary ray + one light sample
with its shadow ray(s), accumulate + tonemap + RGB8: one vpx_render call (the wavefront
kernels of DESIGN.md §4).  Inputs (world, tables, accumulator) are resident in HBM before
timing.

N > 1 (torchrun, one rank per GPU): weak scaling — the frame grows with N (N x 1920x1080
pixels), its 16x16 tiles are dealt round-robin to ranks.  Default (--gather rgb8): each rank
accumulates and tonemaps its own tiles (the accumulator is sharded with them) and an RCCL
gather (torch.distributed, backend nccl) brings the packed RGB8 to rank 0's screen; the
gather of frame f overlaps the render of frame f+1.  --gather samples: ranks send float4
samples and rank 0 composites (unpack + accumulate + tonemap) into its full accumulator.
Timed region: barrier + sync on both sides (the last frame's gather included), max over
ranks.  value = all rays of all ranks / that time.

roofline: the dominant stage (largest device time in the last warmup frame, where every
stage is timed): its algorithmic bytes per launch = DDA cells read x 1 B (the finish stage:
W*H*36 B, accumulator float4 read+write + RGB8 write), SURVEY.md §8(d) / DESIGN.md §4,
divided by its average launch duration measured with HIP events on the library's stream
over the timed region (only that stage is timed there: each timed launch adds two event
records to the stream).
cpu_baseline: the CPU restatement (oracle/, C, -O2) on a bounded pixel sample of the same
frame on this host's cores (rank 0, N = 1 only).
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
import __graft_entry__ as entry  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "Mray/s (primary+shadow) at 1920×1080, 1024³ world; 1/2/4/8-GPU"


def weak_size(n, base=(1920, 1080)):
    """Frame of N x the config's own frame: for C1, 1 -> 1920x1080, 2 -> 3840x1080,
    4 -> 3840x2160, 8 -> 7680x2160."""
    a = 1 << math.ceil(math.log2(n) / 2) if n > 1 else 1
    b = n // a
    if a * b != n:
        a, b = n, 1
    return base[0] * a, base[1] * b


def build_scene(pkg, cfg, width=None, height=None):
    desc = pkg.scene.CONFIGS[cfg]()
    if width and (width, height) != (desc.width, desc.height):
        desc = desc.with_size(width, height)
    return desc


def cpu_baseline(pkg, desc, budget_s=12.0):
    """Oracle timed on a bounded sample (whole rows, evenly spaced) of the same frame."""
    orc = entry.load_oracle()
    t0 = time.time()
    o = orc.Oracle(pkg.abi, desc)
    gen_s = time.time() - t0
    threads = min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    p = desc.frame_params(0)
    W, H = desc.width, desc.height
    # calibrate on 2 rows, then size the sample to ~budget_s
    rows = np.array([H // 2, H // 3], np.int64)
    ids = (rows[:, None] * W + np.arange(W)[None, :]).reshape(-1)
    t = time.time()
    _, st = o.render_pixels(p, ids, threads)
    dt = max(time.time() - t, 1e-3)
    per_row = dt / len(rows)
    nrows = int(max(4, min(H, budget_s / per_row)))
    rows = np.linspace(0, H - 1, nrows).astype(np.int64)
    ids = (rows[:, None] * W + np.arange(W)[None, :]).reshape(-1)
    t = time.time()
    _, st = o.render_pixels(p, ids, threads)
    dt = time.time() - t
    rays = st.primary_rays + st.shadow_rays
    return {"value": round(rays / dt / 1e6, 4), "unit": "Mray/s", "cores": threads, "kind": "port",
            "sample": f"{nrows} evenly spaced rows of the {W}x{H} frame ({len(ids)} pixels, {rays} primary+shadow "
                      f"rays, {dt:.1f} s); world generated on host in {gen_s:.1f} s"}


STAGE_KERNELS = {"primary": "k_primary", "shade": "k_shade", "shadow": "k_shadow_tile", "resolve": "k_resolve",
                 "bounce": "k_nearest_tile", "finish": "k_finish"}


def pmc_traffic(kernel, config, W, H):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary of this
    workload (profiles/*_pmc_traffic.json, FETCH_SIZE x2 + WRITE_SIZE per the gfx950
    correction); None when no summary for this exact workload exists."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "*_pmc_traffic.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("config") == config and d.get("width") == W and d.get("height") == H and kernel in d.get("kernels", {}):
            best = d["kernels"][kernel]["hbm_bytes_per_launch"]
    return best


def run(args):
    pkg = entry.load_package()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n = args.gpus
    if world != n:
        raise SystemExit(f"--gpus {n} but WORLD_SIZE={world}")
    # VPX_BENCH_SHARED_DEVICE=1 rehearses the N-rank flow on ONE GPU (every rank on device 0,
    # gloo collectives through host copies) — for checking the sharded path on a 1-GPU box;
    # real multi-GPU runs use one GPU per rank and RCCL ("nccl").
    shared = os.environ.get("VPX_BENCH_SHARED_DEVICE") == "1"
    dev = 0 if shared else local
    torch.cuda.set_device(dev)
    dist = None
    if n > 1:
        import torch.distributed as dist
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    desc = pkg.scene.CONFIGS[args.config]()
    W, H = weak_size(n, (desc.width, desc.height))
    desc = build_scene(pkg, args.config, W, H)
    stream = torch.cuda.Stream()  # a real stream: the kernel and its HIP events share it
    torch.cuda.set_stream(stream)
    ctx = pkg.context.Context(dev)
    ctx.set_stream(stream.cuda_stream)
    ctx.load_scene(desc)
    torch.cuda.synchronize()
    acc = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda") if rank == 0 else None
    rgb = torch.zeros(W * H, dtype=torch.int32, device="cuda") if rank == 0 else None
    sharded = None
    if n > 1 and args.gather == "rgb8":
        sharded = pkg.dist.ShardedAccumFrame(ctx, desc, rank, n, torch.device("cuda", dev), host_gather=shared)
    elif n > 1:
        L = ctx.packed_len(W, H, n)
        packed = torch.zeros(L * 4, dtype=torch.float32, device="cuda")
        gbuf = torch.empty(n * L * 4, dtype=torch.float32, device="cuda") if rank == 0 else None
        gathered = list(gbuf.view(n, L * 4)) if rank == 0 else None  # gather straight into gbuf

    frame = [0]

    def step():
        p = desc.frame_params(frame_index=frame[0])
        if n == 1:
            ctx.render(p, acc.data_ptr(), rgb.data_ptr())
        elif sharded is not None:
            sharded.frame = frame[0]
            sharded.step()
        else:
            ctx.render_tiles(p, rank, n, packed.data_ptr())
            if shared:
                stream.synchronize()
                parts = [torch.empty(L * 4) for _ in range(n)] if rank == 0 else None
                dist.gather(packed.cpu(), parts, dst=0)
                if rank == 0:
                    gbuf.copy_(torch.cat(parts))
            else:
                dist.gather(packed, gathered, dst=0)
            if rank == 0:
                ctx.composite_tiles(p, n, gbuf.data_ptr(), acc.data_ptr(), rgb.data_ptr())
        frame[0] += 1

    launches = 4 * (desc.max_bounces + 1) + 4  # stage launches per frame, upper bound
    # the last warmup frame times every stage (HIP events on the library's stream): the stage split
    # and the dominant stage; the timed region then times only that stage, since every
    # timed launch adds two event records to the stream (all five C1 stages: +4.3 %)
    ctx.profile_select(None)
    for i in range(args.warmup):
        if i == args.warmup - 1:  # the last warmup frame (the first ones carry cold-start costs)
            if sharded is not None:
                sharded.flush()
            torch.cuda.synchronize()
            ctx.profile_enable(launches)
            ctx.profile_read(reset=True)
        step()
    if sharded is not None:
        sharded.flush()
    torch.cuda.synchronize()
    warm = ctx.profile_read(reset=True)
    timed_stages = [max(warm, key=lambda k: warm[k][0])] if args.warmup > 0 else None
    ctx.counters(reset=True)
    ctx.profile_select(timed_stages)
    ctx.profile_enable(args.steps * launches)
    ctx.profile_read(reset=True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if sharded is not None:
        sharded.flush()  # the last frame's gather + scatter belong to the timed region
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st = ctx.counters()
    local_rays = float(st.primary_rays + st.shadow_rays)
    vals = torch.tensor([elapsed, local_rays, float(st.primary_rays), float(st.shadow_rays), float(st.dda_cells)],
                        dtype=torch.float64, device="cpu" if shared else "cuda")
    if dist:
        mx = vals.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = vals.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed = mx[0].item()
        rays, prim, shad, cells = sm[1].item(), sm[2].item(), sm[3].item(), sm[4].item()
    else:
        rays, prim, shad, cells = local_rays, float(st.primary_rays), float(st.shadow_rays), float(st.dda_cells)
    if rank == 0:
        K = args.steps
        ms_step = elapsed * 1000.0 / K
        value = rays / elapsed / 1e6
        # roofline of the dominant kernel: the stage with the largest device time in the
        # timed region, its algorithmic bytes per launch (1 B per DDA cell
        # read; 36 B per pixel for the accumulate/tonemap stage) over its average launch time
        prof = ctx.profile_read()
        dom = max(prof, key=lambda k: prof[k][0])
        dom_ms, dom_launches, dom_cells = prof[dom]
        split = warm if timed_stages else prof
        kernel_ms = dom_ms / max(dom_launches, 1)
        # the library runs the last level's shadow -> resolve -> finish as one launch
        # (k_shadow_finish) unless built with VPX_FUSE_TAIL=0: then there is
        # no separate finish stage, and the shadow stage carries the 36 B per pixel
        fused = "finish" not in split
        kernels = dict(STAGE_KERNELS)
        if fused:
            kernels["shadow"] = "k_shadow_finish" if desc.max_bounces == 0 else "k_shadow_tile+k_shadow_finish"
        if dom == "finish":
            alg_bytes = float(st.primary_rays) / K * 36.0
        else:
            alg_bytes = float(dom_cells) / max(dom_launches, 1)
            if dom == "shadow" and fused:
                alg_bytes += float(st.primary_rays) * 36.0 / max(dom_launches, 1)
        achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
        frame_bytes = float(st.dda_cells) / K + float(st.primary_rays) / K * 36.0
        traffic = pmc_traffic(kernels[dom], args.config, W, H)
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "Mray/s", "n_gpus": n, "steps": K,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": f"synthetic world '{desc.name}': the reference's .vox asset decoded like ogt_vox, placed in a "
                    f"{desc.grids[0].n}^3 u8 grid on device; fixed lights/camera (SURVEY.md §8(d))",
            "config": {"workload": f"{args.config}: {W}x{H}, {desc.grids[0].n}^3 {desc.name}, 1 spp, "
                                   f"Trace depth {desc.max_bounces} (primary+shadow)",
                       "width": W, "height": H, "world_n": desc.grids[0].n, "max_bounces": desc.max_bounces,
                       "spp": 1, "parallelism": "single GPU" if n == 1 else (
                           (f"tile-shard x{n}, accumulator sharded, RCCL gather of RGB8 to rank 0 (overlapped)"
                            if args.gather == "rgb8" else f"tile-shard x{n} + RCCL gather of samples to rank 0")
                           if not shared else f"REHEARSAL: {n} ranks sharing one GPU, gloo gather via host")},
            "rays_per_step": {"primary": prim / K, "shadow": shad / K, "dda_cells": cells / K},
            "mpix_per_s": round(prim / elapsed / 1e6, 3),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "kernel": kernels[dom], "kernel_ms": round(kernel_ms, 4),
                         "alg_bytes_per_launch": round(alg_bytes),
                         "stages_ms": {k: round(v[0] / max(v[1], 1), 4) for k, v in split.items() if v[1]},
                         "stages_ms_from": "last warmup frame, every stage timed" if timed_stages else "timed region",
                         "frame_alg_bytes": round(frame_bytes),
                         "frame_achieved": round(frame_bytes / (ms_step * 1e-3) / 1e9, 2)},
            "cpu_baseline": None,
        }
        if n == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(pkg, desc, args.cpu_budget)
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C1")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--gather", choices=("rgb8", "samples"), default="rgb8",
                    help="N>1: sharded accumulator + RGB8 gather (default) or float4 samples to rank 0")
    run(ap.parse_args())


if __name__ == "__main__":
    main()
