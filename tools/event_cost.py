"""Frame time of C1 with and without the per-stage profile events (vpx_profile_enable)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as entry  # noqa: E402

pkg = entry.load_package()
desc = pkg.scene.CONFIGS[os.environ.get("CFG", "C1")]()
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
ctx = pkg.context.Context(0)
ctx.set_stream(stream.cuda_stream)
ctx.load_scene(desc)
W, H = desc.width, desc.height
acc = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
rgb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
K = 40
frame = 0
for mode in ("off", "on", "off", "on"):
    if mode == "on":
        ctx.profile_enable(K * 8 + 8)
        ctx.profile_read(reset=True)
    else:
        ctx.profile_enable(0)
    for _ in range(3):
        ctx.render(desc.frame_params(frame_index=frame), acc.data_ptr(), rgb.data_ptr())
        frame += 1
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        ctx.render(desc.frame_params(frame_index=frame), acc.data_ptr(), rgb.data_ptr())
        frame += 1
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1000.0 / K
    extra = ""
    if mode == "on":
        prof = ctx.profile_read(reset=True)
        extra = " stages " + " ".join(f"{k}={v[0] / max(v[1], 1):.4f}" for k, v in prof.items() if v[1])
    print(f"profile {mode}: {ms:.4f} ms/frame{extra}", flush=True)
