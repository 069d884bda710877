"""Debug: step/skip phase split of walk_wave (needs a -DVPX_PHASE_PROF build in VPX_LIB)."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as entry  # noqa: E402
import bench  # noqa: E402

pkg = entry.load_package()
lib = pkg.abi.load_library()
lib.vpx_debug_phase.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
desc = pkg.scene.CONFIGS[os.environ.get("CFG", "C1")]()
if os.environ.get("TW"):  # the same world and camera at another resolution (latency-floor studies)
    desc = desc.with_size(int(os.environ["TW"]), int(os.environ["TH"]))
ctx = pkg.context.Context(0)
ctx.load_scene(desc)
W, H = desc.width, desc.height
acc = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
rgb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
ph = (C.c_ulonglong * 32)()
for f in range(4):
    ctx.render(desc.frame_params(frame_index=f), acc.data_ptr(), rgb.data_ptr())
    torch.cuda.synchronize()
    lib.vpx_debug_phase(ph, 1)
for name, off in (("nearest", 0), ("shadow", 16)):
    cs, ck, ns, nk, ls, lk, walks, fb, cf = list(ph)[off:off + 9]
    walks = max(walks, 1)
    print(f"[{name}] walk calls(waves)={walks}  step: cycles={cs:.3e} iters={ns} lanes/iter={ls / max(ns, 1):.1f} "
          f"cyc/iter={cs / max(ns, 1):.0f} | skip: cycles={ck:.3e} iters={nk} lanes/iter={lk / max(nk, 1):.1f} "
          f"cyc/iter={ck / max(nk, 1):.0f} | per walk: step it={ns / walks:.1f} skip it={nk / walks:.1f} | "
          f"refused lanes/iter={fb / max(nk, 1):.2f} | finished lanes/step iter={cf / max(ns, 1):.1f}")
v = list(ph)
if v[10]:
    print(f"[instances] wave visits={v[10]} lane visits={v[11]} ({v[11] / v[10]:.1f}/wave visit) past sphere cull={v[12]} "
          f"past Setup3DDDA={v[13]} wave visits with a walk={v[14]}")
if v[28]:
    print(f"[instance shadows] slots={v[27]} in {v[28]} waves ({v[27] / v[28]:.1f}/wave); volume visits: waves={v[25]} "
          f"lanes walking={v[26]} ({v[26] / max(v[25], 1):.1f}/wave visit, {v[25] / v[28]:.1f} visits/wave)")
