"""bench.py --gpus N started as a plain process (as the driver's scaling run may start it)
spawns its own N rank processes through torch.distributed.run before any GPU call."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _bench():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_needs_launch_only_without_a_launcher():
    b = _bench()
    assert not b.needs_launch(1, {})
    assert b.needs_launch(2, {})
    assert b.needs_launch(8, {"RANK": "0"})
    assert not b.needs_launch(8, {"WORLD_SIZE": "8"})


def test_launch_command_form():
    b = _bench()
    cmd = b.launch_command(["--gpus", "4", "--steps", "7"], 4, 29517)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29517" in cmd
    i = cmd.index(os.path.join(REPO, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "4", "--steps", "7"]


@pytest.mark.timeout(300)
def test_plain_process_starts_its_ranks():
    """`python bench.py --gpus 2` (no WORLD_SIZE) -> two rank processes with RANK 0 / 1 and
    WORLD_SIZE 2 that see the same arguments (probe mode: they report and stop)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env["VPX_BENCH_LAUNCH_PROBE"] = "1"
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3", "--no-cpu"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert sorted(d["rank"] for d in lines) == [0, 1]
    assert all(d["world"] == 2 for d in lines)
    assert all(d["argv"] == ["--gpus", "2", "--steps", "3", "--no-cpu"] for d in lines)


# ------------------------------------------------------------ bench line keys (round 4)
def test_weak_size_same_view_n_times_the_pixels():
    """weak_scaling: about N x the pixels with the base aspect (the same field of view)."""
    b = _bench()
    assert b.weak_size(1) == (1920, 1080)
    assert b.weak_size(4) == (3840, 2160)
    for n in (2, 4, 8):
        w, h = b.weak_size(n)
        assert abs(w * h / (1920 * 1080) - n) < 0.002 * n
        assert abs(w / h - 1920 / 1080) < 2e-3


def test_with_resolution_keeps_the_camera(pkg):
    """The weak frames render with the base frame's camera (corners), so u = x / W samples
    the same view; with_size instead re-derives the camera for the new aspect."""
    d = pkg.scene.model_scene("teapot", 32, 64, 36, 0)
    same = d.with_resolution(91, 51)
    assert (same.width, same.height) == (91, 51)
    for f in ("cam_pos", "top_left", "top_right", "bottom_left"):
        assert list(getattr(same.camera, f)) == list(getattr(d.camera, f))
    wide = d.with_size(128, 36)
    assert list(wide.camera.top_right) != list(d.camera.top_right)


def test_limiter_paths():
    b = _bench()
    assert b.limiter(None, 1.0)["bound_by"].startswith("unknown")
    # 142 MB in 0.54 ms = 263 GB/s real traffic; VALU busy 0.75 -> VALU-bound
    v = b.limiter({"hbm_bytes_per_launch": 142e6, "valu_busy": 0.75, "wait_frac": 0.47, "l2_hit_rate": 0.43}, 0.54)
    assert v["bound_by"].startswith("VALU") and abs(v["hbm_frac_measured"] - 142e6 / 0.54e-3 / 8e12) < 1e-4
    lat = b.limiter({"hbm_bytes_per_launch": 612e6, "valu_busy": 0.42, "wait_frac": 0.59}, 0.453)
    assert lat["bound_by"].startswith("load latency") and lat["valu_busy"] == 0.42
    bw = b.limiter({"hbm_bytes_per_launch": 7e9, "valu_busy": 0.3}, 1.0)
    assert bw["bound_by"].startswith("HBM")
    # ready waves not issued more than parked -> issue-bound, reported with both fractions
    iss = b.limiter({"hbm_bytes_per_launch": 1e8, "valu_busy": 0.46, "wait_frac": 0.34,
                     "issue_stall_frac": 0.36, "issuing_frac": 0.31}, 1.0)
    assert iss["bound_by"].startswith("instruction issue") and iss["issue_stall_frac"] == 0.36


def test_combine_pmc_two_launch_stage():
    b = _bench()
    one = {"hbm_bytes_per_launch": 5.0, "valu_busy": 0.5}
    assert b.combine_pmc([one]) is one
    c = b.combine_pmc([{"hbm_bytes_per_launch": 100, "valu_busy": 0.2, "wait_frac": 0.6, "gui_active_cycles": 3},
                       {"hbm_bytes_per_launch": 50, "valu_busy": 0.6, "wait_frac": 0.2, "gui_active_cycles": 1}])
    assert c["hbm_bytes_per_launch"] == 150 and c["gui_active_cycles"] == 4
    assert abs(c["valu_busy"] - 0.3) < 1e-9 and abs(c["wait_frac"] - 0.5) < 1e-9
    assert "l2_hit_rate" not in c  # missing in a part -> left out


def _rank_summary_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b = _bench()
        r = b.rank_summary(dist, world, 1.0 + rank, 1000.0 * (rank + 1))
        if rank == 0:
            q.put(r)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_rank_summary_two_ranks_gloo():
    """N > 1 lines carry the process group's backend / world size and per-rank render times
    (min, max, slowest rank): world size 2 over gloo."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_rank_summary_worker, args=(2, port, q), nprocs=2, join=True, start_method="spawn")
    r = q.get(timeout=60)
    assert r["process_group"] == {"backend": "gloo", "world_size": 2}
    assert r["render_ms_per_step"] == {"min": 1.0, "max": 2.0, "slowest_rank": 1, "per_rank": [1.0, 2.0]}
    assert r["primary_rays_per_step_per_rank"] == [1000, 2000]
