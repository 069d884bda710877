"""Where C4's frame goes: the stage times of the full C4 frame (world + 64 instances) against
the same camera and lights with the world volume alone (instances dropped), and the zone
scene Z1's stages (frames in flight off, every stage timed with HIP events).
  python tools/c4_split.py   (GPU)"""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as entry  # noqa: E402

pkg = entry.load_package()
abi = pkg.abi


def stages(desc, frames=6, pipeline=0):
    ctx = pkg.context.Context(0)
    s = torch.cuda.Stream()
    ctx.set_stream(s.cuda_stream)
    ctx.load_scene(desc)
    ctx.set_pipeline(pipeline)
    W, H = desc.width, desc.height
    acc = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
    rgb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    for f in range(2):
        ctx.render(desc.frame_params(f), acc.data_ptr(), rgb.data_ptr())
    torch.cuda.synchronize()
    ctx.profile_select(None)
    ctx.profile_enable(frames * 80)
    ctx.profile_read(reset=True)
    ctx.counters(reset=True)
    t = time.perf_counter()
    for f in range(frames):
        ctx.render(desc.frame_params(f), acc.data_ptr(), rgb.data_ptr())
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) * 1000 / frames
    pr = ctx.profile_read()
    st = ctx.counters()
    out = {"ms_per_frame": round(ms, 4),
           "stages_ms": {k: round(v[0] / frames, 4) for k, v in pr.items() if v[1]},
           "launches_per_frame": {k: v[1] / frames for k, v in pr.items() if v[1]},
           "rays_per_frame": {"primary": st.primary_rays / frames, "shadow": st.shadow_rays / frames,
                              "bounce": st.bounce_rays / frames, "cells": st.dda_cells / frames}}
    ctx.close()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


res = {}
c4 = pkg.scene.CONFIGS["C4"]()
res["C4 full (65 volumes)"] = stages(c4)
w = pkg.scene.CONFIGS["C4"]()
w.volumes = (abi.Volume * 1)(w.volumes[0])
res["C4 world only"] = stages(w)
res["Z1 zone 1920x1080 d14"] = stages(pkg.scene.CONFIGS["Z1"](), frames=4)
print(json.dumps(res, indent=1))
