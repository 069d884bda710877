"""Host cost of the sharded flow's step (dist.ShardedAccumFrame: render + publish, RCCL
gather) against the plain single-GPU step, on C1 at world size 1 over RCCL.

Reports, per step: wall time of K synchronized steps, and the host time to ISSUE them
(no sync inside the loop) — when issue time approaches the GPU time, the N-GPU strong
scaling run is host-bound.  Run on the GPU box:  python tools/host_overhead.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as entry  # noqa: E402

pkg = entry.load_package()
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
import torch.distributed as dist  # noqa: E402

torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
cfg = os.environ.get("CFG", "C1")
desc = pkg.scene.CONFIGS[cfg]()
ctx = pkg.context.Context(0)
ctx.set_stream(s.cuda_stream)
ctx.load_scene(desc)
W, H = desc.width, desc.height
K = int(os.environ.get("K", "50"))


def timed(fn, k):
    for i in range(5):
        fn(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(k):
        fn(i)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t1 - t0) / k * 1e3, (t2 - t0) / k * 1e3


acc = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
rgb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
params = [desc.frame_params(frame_index=i) for i in range(8)]
issue, wall = timed(lambda i: ctx.render(params[i % 8], acc.data_ptr(), rgb.data_ptr()), K)
print(f"{cfg} plain vpx_render: issue {issue:.4f} ms/step, wall {wall:.4f} ms/step")

sh = pkg.dist.ShardedAccumFrame(ctx, desc, 0, 1, torch.device("cuda", 0))


def sharded_step(i):
    sh.render(i)
    sh.publish()


issue, wall = timed(sharded_step, K)
sh.flush()
print(f"{cfg} ShardedAccumFrame (world 1, RCCL gather): issue {issue:.4f} ms/step, wall {wall:.4f} ms/step")

# the host side alone: a tiny frame, so the GPU work is negligible
small = desc.with_size(64, 64)
sm = pkg.dist.ShardedAccumFrame(ctx, small, 0, 1, torch.device("cuda", 0))


def small_step(i):
    sm.render(i)
    sm.publish()


issue, wall = timed(small_step, K)
sm.flush()
print(f"64x64 ShardedAccumFrame: issue {issue:.4f} ms/step, wall {wall:.4f} ms/step (host + launch floor)")
acc2 = torch.zeros(64 * 64 * 4, dtype=torch.float32, device="cuda")
rgb2 = torch.zeros(64 * 64, dtype=torch.int32, device="cuda")
sp = [small.frame_params(frame_index=i) for i in range(8)]
issue, wall = timed(lambda i: ctx.render(sp[i % 8], acc2.data_ptr(), rgb2.data_ptr()), K)
print(f"64x64 plain vpx_render: issue {issue:.4f} ms/step, wall {wall:.4f} ms/step (host + launch floor)")
ctx.close()
dist.destroy_process_group()
