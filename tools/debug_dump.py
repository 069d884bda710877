"""Dump GPU outputs for offline comparison with the oracle (debug helper)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as g
sys.path.insert(0, os.path.join(g.REPO, "tests"))
import cases as T
pkg = g.load_package()
out = {}
for name in ("city128_d0", "monu3_128"):
    desc = T.SCENES[name](pkg.scene)
    ctx = __import__("test_gpu_parity").make_ctx(pkg, desc)
    org, dirs = T.random_rays(4096, 7)
    rays = pkg.context.make_rays(org, dirs)
    h = pkg.context.hits_to_numpy(ctx.find_nearest(rays), len(rays))
    out[name + "_t"] = h["t"]; out[name + "_n"] = h["normal"]; out[name + "_cells"] = h["cells"]
    ctx.close()
    acc, rgb, st = __import__("test_gpu_parity").render_gpu(pkg, desc)
    out[name + "_acc"] = acc; out[name + "_rgb"] = rgb
np.savez(os.path.join(g.REPO, "gpurun_out", "dump.npz"), **out)
print("dumped", list(out))
