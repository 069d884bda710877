"""One rank's GPU time in the N-GPU strong-scaling run, measured on one GPU: rank 0's share
of a config's frame (vpx_render_tiles_accum, rank 0 of R) for R = 1, 2, 4, 8 — the render
part of bench.py --gpus R without the gather.  CFG (default C1), K frames per R, PIPE frames
in flight (vpx_set_pipeline lanes, default 0); WINDOW=1 (default) renders an spp > 1 step as
one accumulation window (vpx_render_tiles_accum_window, as bench.py does), WINDOW=0 frame by
frame.
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as entry  # noqa: E402

pkg = entry.load_package()
cfg = os.environ.get("CFG", "C1")
desc = pkg.scene.CONFIGS[cfg]()
K = int(os.environ.get("K", "20"))
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
ctx = pkg.context.Context(0)
ctx.set_stream(s.cuda_stream)
ctx.load_scene(desc)
ctx.set_pipeline(int(os.environ.get("PIPE", "0")))
if os.environ.get("ARITH", "x86") == "x86":  # the bench line's arithmetic (VPX_ARITH_X86_HOST)
    ctx.set_arithmetic(pkg.abi.VPX_ARITH_X86_HOST)
W, H = desc.width, desc.height
spp = max(1, int(desc.spp))
WINDOW = os.environ.get("WINDOW", "1") == "1"
out = []
for R in [int(x) for x in os.environ.get("RS", "1,2,4,8").split(",")]:
    L = ctx.packed_len(W, H, R)
    acc = torch.zeros(L * 4, dtype=torch.float32, device="cuda")
    rgb = torch.zeros(L, dtype=torch.int32, device="cuda")
    params = [desc.frame_params(frame_index=f) for f in range(spp)]

    def step():
        if WINDOW and spp > 1:  # bench.py's step: one vpx_render_tiles_accum_window per window
            ctx.render_tiles_accum_window(params[0], spp, 0, R, acc.data_ptr(), rgb.data_ptr())
            return
        for p in params:
            ctx.render_tiles_accum(p, 0, R, acc.data_ptr(), rgb.data_ptr())

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        step()
    issue = (time.perf_counter() - t0) * 1e3 / K  # host time to enqueue a step (no sync inside)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / K
    out.append((R, ms, issue))
    del acc, rgb
base = out[0][1]
print(cfg, f"pipe={os.environ.get('PIPE', '0')} arith={os.environ.get('ARITH', 'x86')} window={int(WINDOW)}", " ".join(f"R={R}: {ms:.4f} ms (x{base / ms:.2f})" for R, ms, _ in out))
if os.environ.get("ISSUE"):
    print("  host issue ms per step:", " ".join(f"R={R}: {i:.4f}" for R, _, i in out))
ctx.close()
