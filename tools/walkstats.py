"""Per-ray walk statistics of the skipping walker on the C1 world (CPU model)."""
import ctypes as C, os, subprocess, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as g
so = "/tmp/walkstats.so"
subprocess.run(["g++", "-O2", *sys.argv[2:], "-shared", "-fPIC", "-std=c++17", "-ffp-contract=off", "-I", f"{REPO}/raytracer-voxpopuli_amd/csrc",
                f"{REPO}/tools/native/walkstats.cpp", "-o", so], check=True)
lib = C.CDLL(so)
V = C.c_void_p
lib.build_masks.argtypes = [V, C.c_uint32, V, V]
pkg, orc = g.load_package(), g.load_oracle()
cfg = sys.argv[1] if len(sys.argv) > 1 else "C1"
d = pkg.scene.CONFIGS[cfg]()
o = orc.Oracle(pkg.abi, d)
cells = o.cells[0]; n = d.grids[0].n
nb = [(n + 3) // 4]; nb.append((nb[0] + 3) // 4); nb.append((nb[1] + 3) // 4)
l1, l2 = np.zeros(nb[1] ** 3 * 64, np.uint64), np.zeros(nb[2] ** 3 * 64, np.uint64)
lib.build_masks(cells.ctypes.data, n, l1.ctypes.data, l2.ctypes.data)
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
# ---- box-choice simulation on primary rays and shadow rays toward the lights
lib.walk_sim.argtypes = [V, V, V, C.c_uint32, V, V, V, C.c_uint32, V, V, V]
def sim(st_, si_, bnd, tout=None):
    o = np.zeros(8, np.uint64)
    lib.walk_sim(cells.ctypes.data, l1.ctypes.data, l2.ctypes.data, n, np.ascontiguousarray(st_).ctypes.data,
                 np.ascontiguousarray(si_).ctypes.data, np.ascontiguousarray(bnd, np.float32).ctypes.data, len(st_),
                 o.ctypes.data, None if tout is None else tout.ctypes.data, None)
    return o
def dda_state(org, dirs):
    with np.errstate(divide="ignore", invalid="ignore"):
        rD = (np.float32(1) / dirs).astype(np.float32)
        inside = np.all((org >= 0) & (org <= 1), 1)
        t0 = np.where(inside, 0, np.max(np.minimum((0 - org) * rD, (1 - org) * rD), 1)).astype(np.float32)
        t1 = np.min(np.maximum((0 - org) * rD, (1 - org) * rD), 1)
    ok = inside | ((t1 >= t0) & (t0 > 0))
    ds = (dirs < 0).astype(np.float32)
    pos = (org + dirs * (t0[:, None] + np.float32(5e-5))) * np.float32(n)
    P0 = np.clip(pos.astype(np.int64), 0, n - 1)
    stp = (1 - 2 * ds).astype(np.int32)
    tdel = (cell * stp.astype(np.float32)) * rD
    tmx = ((np.ceil(pos) - ds) * cell - org) * rD
    s1 = np.concatenate([t0[:, None], tmx, tdel], 1).astype(np.float32)
    s2 = np.concatenate([P0, stp], 1).astype(np.int32)
    return s1[ok], s2[ok], ok
th = np.zeros(len(st), np.float32)
base = sim(st, si, np.full(len(st), 1e34, np.float32), th)
hitp = (cp + D * th[:, None])[th > 0].astype(np.float32)
Dh = D[th > 0]
org = (hitp - Dh * np.float32(2e-4)).astype(np.float32)
L = np.float32([0.5, 1.5, 0.5])
dl = L - org
dist = np.sqrt((dl * dl).sum(1)).astype(np.float32)
sets = {"primary": (st, si, np.full(len(st), 1e34, np.float32))}
s1, s2, ok = dda_state(org, (dl / dist[:, None]).astype(np.float32))
sets["shadow-point"] = (s1, s2, dist[ok])
dd = np.float32([0.3, 1.0, 0.2]); dd = dd / np.sqrt((dd * dd).sum())
s1, s2, ok = dda_state(org, np.broadcast_to(dd, org.shape).astype(np.float32).copy())
sets["shadow-dir"] = (s1, s2, np.full(ok.sum(), 1e34, np.float32))
nbk = nb[0]
bocc = np.ascontiguousarray((np.pad(cells.reshape(n, n, n), [(0, nbk * 4 - n)] * 3, constant_values=255)
                            .reshape(nbk, 4, nbk, 4, nbk, 4) != 255).any(axis=(1, 3, 5)).astype(np.uint8))
lib.build_slabs.argtypes = [V, C.c_uint32]
lib.build_slabs(bocc.ctypes.data, nbk)
lib.set_mode.argtypes = [C.c_int]
lib.slab_out.restype = C.c_uint64
modes = [int(x) for x in os.environ.get("MODES", "0").split()]
lib.set_full.argtypes = [C.c_int]
lib.set_full(int(os.environ.get("FULL", "0")))  # 1: whole boxes (the exact multi-binade tier)
for name, (a, b, bnd), mode in [(nm_, v, md) for nm_, v in sets.items() for md in modes]:
    lib.set_mode(mode)
    R = len(a)
    o = sim(a, b, bnd)
    print(f"mode {mode}: slab skips {lib.slab_out() / R:.1f} per ray")
    print(f"{name} ({R} rays): cells {o[0]/R:.0f} steps {o[1]/R:.1f} skips {o[2]/R:.1f} (max {o[7]}) "
          f"lean-clipped {o[6]/max(o[2],1):.4f} cost {(o[1] + 5.8 * o[2]) / R:.0f}")
    lib.small_out.restype = C.c_uint64
    print(f"   steps in empty bricks with a cube below the skip minimum: {lib.small_out() / R:.1f} per ray")
    cr = np.zeros(16, np.uint64); lib.cross_out.argtypes = [V]; lib.cross_out(cr.ctypes.data)
    print("   clipped boxes by binade crossings of the full box (max over axes):", cr[:10])
    s2 = np.zeros(4, np.uint64); lib.seg2_out.argtypes = [V]; lib.seg2_out(s2.ctypes.data)
    print("   skips by #axes needing the 2nd segment:", s2, "frac any:", round(float(s2[1:].sum()) / max(1, float(s2.sum())), 4))
