"""Latency floor of one frame: C1's world and camera at a tiny resolution (the work of
a few tiles), repeated; run under rocprofv3 --kernel-trace to see which kernel holds it."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as entry  # noqa: E402

pkg = entry.load_package()
desc = pkg.scene.CONFIGS[os.environ.get("CFG", "C1")]()
W, H = int(os.environ.get("TW", "64")), int(os.environ.get("TH", "64"))
small = desc.with_size(W, H)
ctx = pkg.context.Context(0)
ctx.load_scene(small)
acc = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
rgb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
K = int(os.environ.get("K", "20"))
for i in range(3):
    ctx.render(small.frame_params(frame_index=i), acc.data_ptr(), rgb.data_ptr())
torch.cuda.synchronize()
ctx.profile_enable(K * 16)
ctx.profile_read(reset=True)
for i in range(K):
    ctx.render(small.frame_params(frame_index=i), acc.data_ptr(), rgb.data_ptr())
torch.cuda.synchronize()
prof = ctx.profile_read()
print(f"{W}x{H}", " ".join(f"{k}={v[0] / max(v[1], 1) * 1e3:.1f}us" for k, v in prof.items() if v[1]))
