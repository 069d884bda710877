"""Per-ray walk statistics of the skipping walker on the C1 world (CPU model)."""
import ctypes as C, os, subprocess, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as g
so = "/tmp/walkstats.so"
subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-std=c++17", "-ffp-contract=off", "-I", f"{REPO}/raytracer-voxpopuli_amd/csrc",
                f"{REPO}/tools/native/walkstats.cpp", "-o", so], check=True)
lib = C.CDLL(so)
V = C.c_void_p
lib.build_masks.argtypes = [V, C.c_uint32, V, V, V]
lib.walk_stats.argtypes = [V, V, V, V, C.c_uint32, V, V, C.c_uint32, C.c_float, V]
pkg, orc = g.load_package(), g.load_oracle()
cfg = sys.argv[1] if len(sys.argv) > 1 else "C1"
d = pkg.scene.CONFIGS[cfg]()
o = orc.Oracle(pkg.abi, d)
cells = o.cells[0]; n = d.grids[0].n
nb = [(n + 3) // 4]; nb.append((nb[0] + 3) // 4); nb.append((nb[1] + 3) // 4)
l1, l2, l3 = (np.zeros(b ** 3, np.uint64) for b in nb)
lib.build_masks(cells.ctypes.data, n, l1.ctypes.data, l2.ctypes.data, l3.ctypes.data)
# primary rays -> DDA setup (numpy float32, identity volume)
rng = np.random.default_rng(0)
W, H = d.width, d.height
m = 20000
xs, ys = rng.integers(0, W, m), rng.integers(0, H, m)
cam = d.camera
f = lambda a: np.array(a[:], np.float32)
tl, tr, bl, cp = f(cam.top_left), f(cam.top_right), f(cam.bottom_left), f(cam.cam_pos)
u = (xs.astype(np.float32) * np.float32(1.0 / W))[:, None]; v = (ys.astype(np.float32) * np.float32(1.0 / H))[:, None]
P = (tl + (tr - tl) * u) + (bl - tl) * v
D = P - cp; D = D / np.sqrt((D * D).sum(1, keepdims=True))
with np.errstate(divide="ignore"):
    rD = (np.float32(1) / D).astype(np.float32)
t0 = np.max(np.minimum((0 - cp) * rD, (1 - cp) * rD), 1); t1 = np.min(np.maximum((0 - cp) * rD, (1 - cp) * rD), 1)
ok = (t1 >= t0) & (t0 > 0)
D, rD, t0 = D[ok], rD[ok], t0[ok].astype(np.float32)
ds = (D < 0).astype(np.float32)
pos = (cp + D * (t0[:, None] + np.float32(5e-5))) * np.float32(n)
P0 = np.clip(pos.astype(np.int64), 0, n - 1)
step = (1 - 2 * ds).astype(np.int32)
cell = np.float32(1.0 / n)
tdel = (cell * step.astype(np.float32)) * rD
tmax = ((np.ceil(pos) - ds) * cell - cp) * rD
st = np.concatenate([t0[:, None], tmax, tdel], 1).astype(np.float32)
si = np.concatenate([P0, step], 1).astype(np.int32)
out = np.zeros(8, np.uint64)
lib.walk_stats(cells.ctypes.data, l1.ctypes.data, l2.ctypes.data, l3.ctypes.data, n, np.ascontiguousarray(st).ctypes.data,
               np.ascontiguousarray(si).ctypes.data, len(st), C.c_float(1e34), out.ctypes.data)
R = len(st)
print(f"{cfg}: rays entering grid {R}/{m}; per ray: cells {out[0]/R:.1f} iters {out[1]/R:.1f} steps {out[2]/R:.1f} "
      f"skip16 {out[3]/R:.2f} skip64 {out[4]/R:.2f} zero-skips {out[5]/R:.2f} max iters {out[6]} fast-path skips {out[7]/max(out[3]+out[4],1):.3f}")
wy = np.zeros(8, np.uint64)
lib.why_out.argtypes = [V]
lib.why_out(wy.ctypes.data)
print("fast-path failures by axis reason (nonnormal, d>=2^E, tie/stuck, 2nd crossing):", wy[:4])
