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
