"""bench.py — Mray/s (primary+shadow) of the MI355X voxel ray-trace path.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C1] [--no-cpu] [--no-extra]

A step = one image of the workload: spp accumulated frames (C1-C3: 1, C4: 16), each one
vpx_render call (primary rays, Trace(ray, max_bounces) flattened, the light samples with
their shadow rays, running-average accumulate, tonemap, RGB8; the wavefront kernels of
DESIGN.md §4).  The headline line is C1 (BASELINE.json configs[1]): 1920x1080, 1024^3 world
(monu3.vox tiled), 1 spp, depth 0.  Inputs (world, tables, accumulator)
are resident in HBM before timing.  Arithmetic (every config of the line, `arithmetic`): the
reference's own — FindNearest's FastReciprocal and the rsqrtps primary normalise from this
host's captured rcpss / rsqrtss tables (VPX_ARITH_X86_HOST), the mode whose
output matches the reference within north_star's 1e-4 (0 pixels beyond on every full-size
shard, tests/test_x86_arith.py); `other_arithmetic` times C1 in the exact mode beside it.

N > 1 (one rank process per GPU: under torchrun, or started by this script itself as a
torch.distributed.run child when run as plain `python bench.py --gpus N`): STRONG scaling — the configured frame (C1: 1920x1080
at every N; C3/C4: 3840x2160) is cut into 16x16 tiles dealt round-robin to the ranks; each
rank accumulates and tonemaps its own tiles (the accumulator is sharded with them) and an
RCCL gather (torch.distributed, backend nccl) brings the packed RGB8 of the step's last
frame to rank 0's screen, overlapped with the next step's renders.  Timed region: barrier
+ sync on both sides (the last gather included), max over ranks; value = all ranks' rays /
that time.  Weak scaling (about N x the pixels at the same field of view, weak_size) is the extra key
`weak_scaling`.

Extra keys: `extra_configs` C2 / C3 / C4 (same N, their stated sizes, fewer steps), each
with ms/step, Mray/s (primary+shadow), total Mray/s (incl. bounce rays) and its own
dominant-stage roofline.

roofline: the dominant stage (largest device time in the last warmup step, where every
stage is timed): its algorithmic bytes per launch = DDA cells read x 1 B (+ W*H*36 B for
the accumulate/tonemap work when the stage's kernel carries it), SURVEY.md §8(d) /
DESIGN.md §4, divided by its average launch duration measured with HIP events on the
library's stream over the timed region (only that stage is timed there).  traffic: HBM
bytes per launch from the rocprofv3 PMC summary committed for THIS library build
(profiles/*_pmc_traffic.json, matched by the library's sha256), else null.
cpu_baseline (rank 0, N = 1): the CPU restatement (oracle/liboracle_perf.so, -O3
x86-64-v3, bit-identical to the checker) on a bounded row sample of the C1 frame with every
thread of the box's CPU share, plus BASELINE.md §3's C0 / C0' frames (640x360, 1 thread and
all threads, median of 20 after 3 warm-ups).
"""
import argparse
import hashlib
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

# the reference's arithmetic (VPX_ARITH_X86_HOST) needs the host's rcpss / rsqrtss tables
X86_HOST = os.uname().machine in ("x86_64", "i686")
ARITH_NAMES = {0: "VPX_ARITH_EXACT", 1: "VPX_ARITH_X86_HOST"}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "Mray/s (primary+shadow) at 1920×1080, 1024³ world; 1/2/4/8-GPU"
# Z1: the reference's own scene shape (SetUpFirstZone: 21 volumes, 10 triangles, point + 5 spot +
# directional lights, depth 14, sky; scene.zone_scene) at 1920x1080
EXTRA_CONFIGS = ("C2", "C3", "C4", "Z1")
# Frames in flight per config (vpx_set_pipeline lanes, each on a dedicated hardware queue),
# from the A/B on one MI355X (ms per step, 2 / 3 / 4 lanes): C1 - / 0.551-0.554 /
# 0.578-0.594, C4 52.6 / 52.4 / 51.6; with the pools (round 3) C2 2.76-2.77 / 2.50-2.52 /
# 2.42-2.45 as the process's first config but 2.57-2.69 (3) vs 2.87-2.90 (4) as an extra
# config after C1 (the line the driver runs), C3 3.70-3.71 / 3.65 / 3.67-3.71.  Round 4: C2's
# single-volume levels fork their bounce walks beside the shadow walks when at most two lanes
# run (vpx_kernels.hip launch_render): C2 2.50-2.52 at 2 lanes vs 2.65-2.67 at 3 without forks
# as the first config (2.70 either way as an extra after C1).  Round-4 build (tools/gpu_r4m.sh,
# 2 / 3 / 4 lanes): C1 0.553-0.557 / 0.555-0.556 / 0.586-0.587, C4 45.0-45.1 / 43.2-43.5 / 44.5-44.8.
# Round 5, with each lane's two sample buffers and the live lists (three interleaved runs): C2
# 2.350-2.358 (2 lanes, forks) / 2.272-2.338 (3) / 2.412-2.441 (4), and 2.64-2.70 with forks
# at 3 lanes; C4 42.80-42.99 (3) / 43.70-43.92 (4); Z1 1.755-1.769 (2) / 1.532-1.540 (3).
# Round 6, accumulation windows (vpx_render_window, 4 frames a chain): C4 26.84-26.87 (4 lanes)
# / 28.50-28.57 (3), profiles/r06_window_ab.txt.
PIPELINE = {"C1": 3, "C2": 3, "C3": 3, "C4": 4, "Z1": 3}
# A rank's share of a multi-GPU frame is a small launch: with each lane's two sample buffers
# (round 5) four lanes keep more of it in flight for the big frames (rank 0's share at R = 8,
# tools/rank_share.py, 3 / 4 lanes: C3 0.586 / 0.564 ms, C4 9.93 / 8.63 ms per 16-spp step;
# C1 0.091 / 0.100 ms stays at 3; one GPU: C3 3.55 / 3.59 ms).
PIPELINE_MULTI = {"C3": 4, "C4": 4}
STAGE_KERNELS = {"primary": "k_primary", "shade": "k_shade", "shadow": "k_shadow_tile", "resolve": "k_resolve",
                 "bounce": "k_nearest_tile", "finish": "k_finish", "frame": "k_frame0", "instances": "k_instances"}


def weak_size(n, base=(1920, 1080)):
    """Frame of about N x the config's own pixels at the SAME field of view: both sides scaled
    by sqrt(N) (C1: 1 -> 1920x1080, 2 -> 2715x1527, 4 -> 3840x2160, 8 -> 5431x3055), rendered
    with the base frame's camera (its TL / TR / BL corners, camera.h:90-105, u = x / W), so the
    extra pixels sample the same view more densely instead of widening it onto free sky."""
    r = math.sqrt(n)
    return int(round(base[0] * r)), int(round(base[1] * r))


def lib_sha256(pkg):
    path = os.environ.get("VPX_LIB") or pkg.abi.LIB_PATH
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def pmc_summary(kernel, config, W, H, sha):
    """The committed rocprofv3 PMC summary of `kernel` for this workload AND this library
    build (tools/pmc_traffic.py: hbm_bytes_per_launch = FETCH_SIZE x2 + WRITE_SIZE per the
    gfx950 correction, valu_busy, wait_frac, l2_hit_rate) and the file it came from; (None,
    None) when no summary for this exact build / workload exists."""
    import glob
    best, src = None, None
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_traffic*.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        ks = d.get("kernels", {})
        parts = kernel.split("+")  # a stage of two launches (e.g. k_shadow_pool+k_shadow_slots)
        if (d.get("config") == config and d.get("width") == W and d.get("height") == H
                and d.get("lib_sha256") == sha and all(k in ks for k in parts)):
            best, src = combine_pmc([ks[k] for k in parts]), os.path.relpath(f, REPO)
    return best, src


def combine_pmc(ps):
    """One stage's PMC summary from its launches' (each launched once per frame): bytes add,
    the cycle fractions are averaged weighted by each launch's GRBM_GUI_ACTIVE cycles."""
    if len(ps) == 1:
        return ps[0]
    out = {"hbm_bytes_per_launch": sum(p["hbm_bytes_per_launch"] for p in ps)}
    wts = [p.get("gui_active_cycles") or 0 for p in ps]
    for key in ("valu_busy", "wait_frac", "issue_stall_frac", "issuing_frac", "waves_per_simd", "l2_hit_rate"):
        vals = [p.get(key) for p in ps]
        if all(v is not None for v in vals) and sum(wts) > 0:
            out[key] = round(sum(v * w for v, w in zip(vals, wts)) / sum(wts), 4)
    out["gui_active_cycles"] = sum(wts)
    return out


def limiter(pmc, kernel_ms):
    """What bounds the dominant kernel, from its committed counters: its real HBM fraction
    (measured traffic / busy time / peak) against its VALU busy fraction."""
    if not pmc:
        return {"hbm_frac_measured": None, "valu_busy": None, "bound_by": "unknown: no PMC summary for this build"}
    hbm = pmc["hbm_bytes_per_launch"] / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
    vb = pmc.get("valu_busy")
    wf, st = pmc.get("wait_frac"), pmc.get("issue_stall_frac")
    fmt = lambda x: "%.2f" % x if x is not None else "n/a"
    if vb is not None and vb >= 0.6 and vb > hbm:
        why = "VALU issue (valu_busy %.2f; real HBM %.3f of peak)" % (vb, hbm)
    elif hbm >= 0.6:
        why = "HBM bandwidth (real HBM %.2f of peak)" % hbm
    elif wf is not None and st is not None and st > wf:
        why = ("instruction issue: ready waves not issued, dependency / arbitration stalls %s of wave "
               "cycles vs %s parked on loads (valu_busy %s, real HBM %.3f of peak)" % (fmt(st), fmt(wf), fmt(vb), hbm))
    else:
        why = ("load latency: dependent gather chains (real HBM %.3f of peak, valu_busy %s, waves parked %s "
               "of cycles, issue-stalled %s)" % (hbm, fmt(vb), fmt(wf), fmt(st)))
    return {"hbm_frac_measured": round(hbm, 4), "valu_busy": vb, "wait_frac": wf, "issue_stall_frac": st,
            "issuing_frac": pmc.get("issuing_frac"), "waves_per_simd": pmc.get("waves_per_simd"),
            "l2_hit_rate": pmc.get("l2_hit_rate"), "bound_by": why}


def rank_summary(dist, n, render_ms, primary, device="cpu"):
    """Every rank's render time per step and primary rays per step, gathered (all ranks call
    it): the process group's backend and world size as torch.distributed sees them, min / max
    render ms and the slowest rank — so a multi-GPU line shows whether RCCL saw N ranks and
    which rank sets the time."""
    mine = torch.tensor([float(render_ms), float(primary)], dtype=torch.float64, device=device)
    every = [torch.zeros_like(mine) for _ in range(n)]
    dist.all_gather(every, mine)
    ms = [float(x[0]) for x in every]
    return {"process_group": {"backend": str(dist.get_backend()), "world_size": dist.get_world_size()},
            "render_ms_per_step": {"min": round(min(ms), 4), "max": round(max(ms), 4),
                                   "slowest_rank": int(np.argmax(ms)), "per_rank": [round(x, 4) for x in ms]},
            "primary_rays_per_step_per_rank": [int(x[1]) for x in every]}


class Env:
    """Rank / device / process-group state of this bench process."""

    def __init__(self, n):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.n = n
        if self.world != n:
            raise SystemExit(f"--gpus {n} but WORLD_SIZE={self.world}")
        # VPX_BENCH_SHARED_DEVICE=1 rehearses the N-rank flow on ONE GPU (every rank on device 0,
        # gloo collectives through host copies) — for checking the sharded path on a 1-GPU box;
        # real multi-GPU runs use one GPU per rank and RCCL ("nccl").
        self.shared = os.environ.get("VPX_BENCH_SHARED_DEVICE") == "1"
        self.dev = 0 if self.shared else self.local
        torch.cuda.set_device(self.dev)
        self.dist = None
        if n > 1:
            import torch.distributed as dist
            if self.shared:
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.dev))
            self.dist = dist
        self.stream = torch.cuda.Stream()  # a real stream: the kernels and their HIP events share it
        torch.cuda.set_stream(self.stream)

    def parallelism(self):
        if self.n == 1:
            return "single GPU"
        if self.shared:
            return f"REHEARSAL: {self.n} ranks sharing one GPU, gloo gather via host"
        return f"tile-shard x{self.n}, accumulator sharded, RCCL gather of RGB8 to rank 0 (overlapped)"


def run_config(pkg, env, cfg, steps, warmup, weak=False, sha=None, pipeline=None, serial_frames=0, arith=0):
    """Load `cfg` on this rank, run warmup + `steps` timed steps, return the result dict
    (rank 0; None elsewhere).  Frees the world before returning.  arith: vpx_set_arithmetic
    mode (0 exact, the default; 1 the reference's x86 rcpps / rsqrtps from this host)."""
    desc = pkg.scene.CONFIGS[cfg]()
    if weak:  # N x the pixels at the same field of view (the base frame's camera)
        desc = desc.with_resolution(*weak_size(env.n, (desc.width, desc.height)))
    W, H, spp = desc.width, desc.height, max(1, int(desc.spp))
    ctx = pkg.context.Context(env.dev)
    ctx.set_stream(env.stream.cuda_stream)
    ctx.load_scene(desc)
    if arith:
        ctx.set_arithmetic(arith)
    if pipeline is None:
        pipeline = PIPELINE_MULTI.get(cfg, PIPELINE.get(cfg, 0)) if env.n >= 4 else PIPELINE.get(cfg, 0)
    ctx.set_pipeline(pipeline)
    torch.cuda.synchronize()
    acc = rgb = sharded = None
    if env.n == 1:
        acc = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
        rgb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    else:
        sharded = pkg.dist.ShardedAccumFrame(ctx, desc, env.rank, env.n, torch.device("cuda", env.dev),
                                             host_gather=env.shared)

    def step():
        # accumulation window: w = 1/(f+1), per-frame seeds (renderer.cpp:1791-1828); one library
        # call per window (vpx_render_window: a rank's small share of several frames per chain)
        if sharded is None:
            if spp == 1:
                ctx.render(desc.frame_params(frame_index=0), acc.data_ptr(), rgb.data_ptr())
            else:
                ctx.render_window(desc.frame_params(frame_index=0), spp, acc.data_ptr(), rgb.data_ptr())
        else:
            sharded.render_window(0, spp)
            sharded.publish()

    launches = spp * (4 * (desc.max_bounces + 1) + 4)  # stage launches per step, upper bound
    # the last warmup step times every stage (HIP events on the library's stream): the stage
    # split and the dominant stage; the timed region then times only that stage, since every
    # timed launch adds two event records to the stream (all five C1 stages: +4.3 %)
    ctx.profile_select(None)
    for i in range(warmup):
        if i == warmup - 1:  # the last warmup step (the first ones carry cold-start costs)
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
    timed_stages = [max(warm, key=lambda k: warm[k][3])] if warmup > 0 else None  # by busy time
    ctx.counters(reset=True)
    ctx.profile_select(timed_stages)
    ctx.profile_enable(steps * launches)
    ctx.profile_read(reset=True)
    if env.dist:
        env.dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    if sharded is not None:
        sharded.flush()  # the last step's gather + scatter belong to the timed region
    torch.cuda.synchronize()
    t_local = time.perf_counter() - t0  # this rank's own render (+ its part of the gather), before the barrier
    if env.dist:
        env.dist.barrier()
    elapsed = time.perf_counter() - t0
    st = ctx.counters()
    vals = torch.tensor([elapsed, float(st.primary_rays), float(st.shadow_rays), float(st.bounce_rays),
                         float(st.dda_cells)], dtype=torch.float64, device="cpu" if env.shared else "cuda")
    ranks = None
    if env.dist:
        mx, sm = vals.clone(), vals.clone()
        env.dist.all_reduce(mx, op=env.dist.ReduceOp.MAX)
        env.dist.all_reduce(sm, op=env.dist.ReduceOp.SUM)
        elapsed = mx[0].item()
        prim, shad, bounce, cells = (sm[i].item() for i in range(1, 5))
        ranks = rank_summary(env.dist, env.n, t_local * 1000.0 / steps, float(st.primary_rays) / steps, vals.device)
    else:
        prim, shad, bounce, cells = float(st.primary_rays), float(st.shadow_rays), float(st.bounce_rays), \
            float(st.dda_cells)
    out = None
    if env.rank == 0:
        K = steps
        ms_step = elapsed * 1000.0 / K
        prof = ctx.profile_read()
        dom = max(prof, key=lambda k: prof[k][3])
        dom_ms, dom_launches, dom_cells, dom_busy = prof[dom]
        split = warm if timed_stages else prof
        # a launch's duration = the stage's busy time (the union of its launch intervals) per
        # launch: with frames in flight consecutive frames' launches overlap, and summing their
        # start-to-end times would count the shared time twice; launch_ms is that sum per
        # launch (what a kernel trace averages per dispatch)
        kernel_ms = dom_busy / max(dom_launches, 1)
        launch_ms = dom_ms / max(dom_launches, 1)
        # the last level's shadow -> resolve -> finish run as one launch (k_shadow_finish,
        # DESIGN.md §4): no separate finish stage, the shadow stage carries the 36 B per pixel
        fused = split.get("finish", (0.0, 0, 0, 0.0))[1] == 0  # stages with no launch stay in the table
        kernels = dict(STAGE_KERNELS)
        if len(desc.volumes) == 1 and not (desc.spheres or desc.triangles):  # the pools
            kernels["bounce"] = "k_nearest_pool"
        if desc.areas and desc.area_samples > 1:  # area lights: the shadow pool (+ k_shadow_slots)
            kernels.update(shadow="k_shadow_pool" if len(desc.volumes) == 1 and not (desc.spheres or desc.triangles)
                           else "k_shadow_pool+k_shadow_slots", finish="k_resolve_finish")
        if fused:
            kernels["shadow"] = "k_shadow_finish" if desc.max_bounces == 0 else "k_shadow_tile+k_shadow_finish"
        # rank 0's own work (its launches, cells and pixels)
        local_pix = float(st.primary_rays)
        if dom == "finish":
            alg_bytes = local_pix / K / spp * 36.0
        elif dom == "frame":  # k_frame0: the whole depth-0 frame (every stage's cells + the finish)
            alg_bytes = (sum(float(v[2]) for v in prof.values()) + local_pix * 36.0) / max(dom_launches, 1)
        else:
            alg_bytes = float(dom_cells) / max(dom_launches, 1)
            if dom == "shadow" and fused:
                alg_bytes += local_pix * 36.0 / max(dom_launches, 1)
        achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
        frame_bytes = (cells + prim * 36.0) / K
        pmc, pmc_src = pmc_summary(kernels[dom], cfg, W, H, sha) if env.n == 1 else (None, None)
        traffic = pmc["hbm_bytes_per_launch"] if pmc else None
        out = {
            "config": cfg, "value": round((prim + shad) / elapsed / 1e6, 3), "ms_per_step": round(ms_step, 4),
            "total_mray_s": round((prim + shad + bounce) / elapsed / 1e6, 3),
            "workload": f"{cfg}: {W}x{H}, {max(g.n for g in desc.grids)}^3 {desc.name}, {spp} spp, Trace depth "
                        f"{desc.max_bounces}"
                        + (f", {len(desc.volumes)} volumes" if len(desc.volumes) > 1 else "")
                        + (f", {len(desc.triangles)} triangles" if desc.triangles else "")
                        + (f", {len(desc.spots)} spot lights" if desc.spots else "")
                        + (f", {len(desc.areas)} area lights x {desc.area_samples} samples" if desc.areas else ""),
            "width": W, "height": H, "world_n": max(g.n for g in desc.grids), "max_bounces": desc.max_bounces, "spp": spp,
            "rays_per_step": {"primary": prim / K, "shadow": shad / K, "bounce": bounce / K, "dda_cells": cells / K},
            "mpix_per_s": round(prim / elapsed / 1e6, 3),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "traffic_source": (pmc_src + " (this library build: sha256 match)"
                                            if traffic is not None else
                                            "null: no PMC pass committed for this library build / workload"),
                         "traffic_over_alg": round(traffic / alg_bytes, 3) if traffic else None,
                         **limiter(pmc, kernel_ms),
                         "kernel": kernels[dom], "kernel_ms": round(kernel_ms, 4), "launch_ms": round(launch_ms, 4),
                         "kernel_ms_def": "busy time of the kernel's launches over the timed region (overlapping "
                                          "launches counted once) / launches; launch_ms = mean start-to-end per launch",
                         "alg_bytes_per_launch": round(alg_bytes),
                         "stages_ms": {k: round(v[3] / max(v[1], 1), 4) for k, v in split.items() if v[1]},
                         "stages_ms_from": "last warmup step, every stage timed" if timed_stages else "timed region",
                         "frame_alg_bytes": round(frame_bytes),
                         "frame_achieved": round(frame_bytes / (ms_step * 1e-3) / 1e9, 2)},
            "pipeline": pipeline,
        }
        if ranks is not None:
            out["ranks"] = ranks
    if env.n == 1 and serial_frames:
        # what a per-frame-synchronous host (the tmpl8 loop: Tick, then present, every frame,
        # template.cpp:300-305) sees: one frame at a time, no lanes, the host waits for each
        ctx.set_pipeline(0)
        for f in range(2):  # the serial path's own path-state buffers, warm
            ctx.render(desc.frame_params(frame_index=f), acc.data_ptr(), rgb.data_ptr())
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for f in range(serial_frames):
            ctx.render(desc.frame_params(frame_index=f % spp), acc.data_ptr(), rgb.data_ptr())
            torch.cuda.synchronize()
        if out is not None:
            out["serial_ms_per_frame"] = round((time.perf_counter() - t1) * 1000.0 / serial_frames, 4)
            out["serial_ms_per_step"] = round(out["serial_ms_per_frame"] * spp, 4)
            out["serial_def"] = (f"{serial_frames} frames at --pipeline 0 with a host synchronize after each "
                                 f"(a per-frame-synchronous Tick); a step is {spp} frame(s), so serial_ms_per_step = "
                                 "serial_ms_per_frame x spp compares with ms_per_step, the frames-in-flight figure")
    del acc, rgb, sharded
    ctx.close()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


# ------------------------------------------------------------------ CPU baseline
def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads():
    """Threads the box gives this job: OMP_NUM_THREADS (16 per GPU on the pool), else the
    affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def time_frames(o, desc, threads, warm=3, frames=20):
    """Median over `frames` whole-frame oracle renders after `warm` warm-ups."""
    p = desc.frame_params(0)
    acc = np.zeros((desc.width * desc.height, 4), np.float32)
    ts, st = [], None
    for i in range(warm + frames):
        t = time.perf_counter()
        _, _, st = o.render(p, accum=acc, threads=threads)
        if i >= warm:
            ts.append(time.perf_counter() - t)
    med = float(np.median(ts))
    rays = st.primary_rays + st.shadow_rays
    return {"ms_median": round(med * 1e3, 3), "ms_min": round(min(ts) * 1e3, 3), "ms_max": round(max(ts) * 1e3, 3),
            "mray_s": round(rays / med / 1e6, 4), "mpix_s": round(st.primary_rays / med / 1e6, 4),
            "rays_per_frame": {"primary": st.primary_rays, "shadow": st.shadow_rays}}


def cpu_baseline(pkg, desc, budget_s=12.0, arith=0):
    """The oracle (perf build) on the host: C1 row sample (value) + C0 / C0' frames, in the
    headline's arithmetic (x86: the oracle's FastReciprocal / rsqrtps with this host's own
    instructions, as the reference computes them)."""
    orc = entry.load_oracle()
    orc.set_x86_approx(pkg.abi, arith, perf=True)
    threads = cpu_threads()
    t0 = time.time()
    o = orc.Oracle(pkg.abi, desc, perf=True)
    gen_s = time.time() - t0
    p = desc.frame_params(0)
    W, H = desc.width, desc.height
    rows = np.array([H // 2, H // 3], np.int64)  # calibrate on 2 rows, then size the sample to ~budget_s
    ids = (rows[:, None] * W + np.arange(W)[None, :]).reshape(-1)
    t = time.time()
    o.render_pixels(p, ids, threads)
    per_row = max(time.time() - t, 1e-3) / len(rows)
    nrows = int(max(4, min(H, budget_s / 3 / per_row)))
    rows = np.linspace(0, H - 1, nrows).astype(np.int64)
    ids = (rows[:, None] * W + np.arange(W)[None, :]).reshape(-1)
    runs = []
    for _ in range(3):  # three passes over the same sample: median and spread
        t = time.time()
        _, st = o.render_pixels(p, ids, threads)
        runs.append((st.primary_rays + st.shadow_rays) / (time.time() - t) / 1e6)
    del o
    out = {"value": round(float(np.median(runs)), 4), "unit": "Mray/s", "cores": threads, "kind": "port",
           "sample": f"{nrows} evenly spaced rows of the {W}x{H} C1 frame ({len(ids)} pixels, "
                     f"{st.primary_rays + st.shadow_rays} primary+shadow rays per pass), median of 3 passes "
                     f"(min {min(runs):.3f}, max {max(runs):.3f} Mray/s); world generated on host in {gen_s:.1f} s",
           "cpu_model": cpu_model(), "machine_logical_cpus": os.cpu_count(),
           "threads_note": "cores = threads used = the box's CPU share (OMP_NUM_THREADS); std::thread pixel pool",
           "build": "oracle/liboracle_perf.so: gcc -O3 -march=x86-64-v3 -ffp-contract=off, FTZ/DAZ",
           "arithmetic": ARITH_NAMES[arith]}
    for key, cfg in (("c0", "C0"), ("c0_prime", "C0m")):  # 640x360, 1 spp, depth 0
        d = pkg.scene.CONFIGS[cfg]()
        oc = orc.Oracle(pkg.abi, d, perf=True)
        out[key] = {"workload": f"{d.width}x{d.height}, {d.grids[0].n}^3 {d.name}, 1 spp, depth 0",
                    "threads_1": time_frames(oc, d, 1), f"threads_{threads}": time_frames(oc, d, threads)}
    return out


def free_port():
    """A TCP port on 127.0.0.1 that was free a moment ago (the ranks' rendezvous)."""
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_command(argv, n, port):
    """The child command that runs this bench as N ranks, one process per GPU (the
    driver's own form: torch.distributed.run, rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def needs_launch(n, environ=os.environ):
    """--gpus N > 1 started as a plain process (no WORLD_SIZE from a launcher): this process
    must start the N rank processes itself."""
    return n > 1 and "WORLD_SIZE" not in environ


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C1")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip extra_configs / weak_scaling")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--arith", choices=("exact", "x86"), default="x86" if X86_HOST else "exact",
                    help="vpx_set_arithmetic of every config (x86, the default on x86 hosts: the reference's "
                         "FastReciprocal rcpps+NR and rsqrtps normalise, this host's tables, DESIGN.md §3 item 1); "
                         "the N=1 line also reports C1 in the other mode as other_arithmetic")
    ap.add_argument("--pipeline", type=int, default=None,
                    help="frames in flight per GPU (vpx_set_pipeline lanes; 0 = serial frames); default: "
                         "per config, PIPELINE")
    args = ap.parse_args()
    if needs_launch(args.gpus):
        # `python bench.py --gpus N` without torchrun: start the N ranks as child processes
        # before this process touches the GPU (no HIP call has been made yet), relay their
        # output (rank 0 prints the JSON line) and exit with their status
        import subprocess
        cmd = launch_command(sys.argv[1:], args.gpus, free_port())
        print("bench.py: launching", args.gpus, "ranks:", " ".join(cmd), file=sys.stderr, flush=True)
        sys.exit(subprocess.run(cmd).returncode)
    if os.environ.get("VPX_BENCH_LAUNCH_PROBE") == "1":  # tests/test_bench_launch.py: the ranks' view, no GPU work
        print(json.dumps({"rank": int(os.environ.get("RANK", "0")), "world": int(os.environ.get("WORLD_SIZE", "1")),
                          "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "argv": sys.argv[1:]}), flush=True)
        return
    pkg = entry.load_package()
    env = Env(args.gpus)
    sha = lib_sha256(pkg)
    arith = 1 if args.arith == "x86" else 0
    head = run_config(pkg, env, args.config, args.steps, args.warmup, sha=sha, pipeline=args.pipeline,
                      serial_frames=args.steps, arith=arith)
    other_arith = None
    if env.n == 1 and not args.no_extra and X86_HOST:
        # the same workload in the other arithmetic mode: with the reference's arithmetic as the
        # headline (VPX_ARITH_X86_HOST: FindNearest's FastReciprocal and the primary rsqrtps as this
        # host computes them, bit-identical to the oracle's x86 mode, tests/test_x86_arith.py), the
        # exact mode's C1 (exact 1/x, 1/sqrtf) beside it, and what the tables cost
        o = 1 - arith
        r = run_config(pkg, env, args.config, args.steps, args.warmup, sha=sha, pipeline=args.pipeline, arith=o)
        if r is not None:
            other_arith = {"mode": ARITH_NAMES[o], "ms_per_step": r["ms_per_step"], "value": r["value"],
                           "headline_mode": ARITH_NAMES[arith], "headline_ms_per_step": head["ms_per_step"],
                           "x86_cost": round((head["ms_per_step"] / r["ms_per_step"] if arith else
                                              r["ms_per_step"] / head["ms_per_step"]) - 1.0, 4)}
    extra, weak = {}, None
    if not args.no_extra:
        # the extras time as many steps as the headline: with frames in flight the timed region
        # includes one pipeline fill and drain, which 5 steps (the earlier K / 4) charged at
        # ~0.2 ms per step to C2 (2.70 vs 2.50 ms per step at 10 steps, same build and box)
        xs = max(3, args.steps)
        for cfg in EXTRA_CONFIGS:
            if cfg != args.config:
                r = run_config(pkg, env, cfg, xs, min(args.warmup, 2), sha=sha, pipeline=args.pipeline,
                               serial_frames=xs, arith=arith)
                if r is not None:
                    extra[cfg] = r
        if env.n > 1:
            weak = run_config(pkg, env, args.config, xs, min(args.warmup, 2), weak=True, sha=sha, pipeline=args.pipeline,
                              arith=arith)
    if env.rank == 0:
        out = {"metric": METRIC, "value": head["value"], "unit": "Mray/s", "n_gpus": env.n, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": head["ms_per_step"], "higher_is_better": True,
               "scaling": "strong", "vs_baseline": None, "dtype": "f32",
               "data": "synthetic worlds: the reference's .vox assets decoded like ogt_vox and tiled into the "
                       "build-defined 1024^3 / 2048^3 u8 grids on device; fixed lights/camera (SURVEY.md §8(d))",
               "config": {"workload": head["workload"], "width": head["width"], "height": head["height"],
                          "world_n": head["world_n"], "max_bounces": head["max_bounces"], "spp": head["spp"],
                          "parallelism": env.parallelism(), "frames_in_flight": head["pipeline"], "lib_sha256": sha},
               "rays_per_step": head["rays_per_step"], "mpix_per_s": head["mpix_per_s"],
               "total_mray_s": head["total_mray_s"], "roofline": head["roofline"], "cpu_baseline": None}
        out["arithmetic"] = out["config"]["arithmetic"] = ARITH_NAMES[arith]
        out["arithmetic_def"] = ("VPX_ARITH_X86_HOST: FindNearest's per-volume rD by FastReciprocal (rcpps + one Newton "
                                 "step, renderer.cpp:929-934) and the primary directions by rsqrtps "
                                 "(tmpl8math.h:2356-2360), from this host's captured tables, in every config of the "
                                 "line: the reference's own arithmetic, 0 pixels beyond 1e-4 on the full-size shards "
                                 "(tests/test_x86_arith.py)" if arith else "VPX_ARITH_EXACT: exact 1/x and 1/sqrtf")
        if other_arith is not None:
            out["other_arithmetic"] = other_arith
        for k in ("serial_ms_per_frame", "serial_ms_per_step", "serial_def", "ranks"):
            if k in head:
                out[k] = head[k]
        if extra:
            out["extra_configs"] = extra
        if weak is not None:
            out["weak_scaling"] = weak
        if env.n == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(pkg, pkg.scene.CONFIGS[args.config](), args.cpu_budget, arith)
        print(json.dumps(out), flush=True)
    if env.dist:
        env.dist.destroy_process_group()


if __name__ == "__main__":
    main()
