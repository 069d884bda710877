"""Wave-cost model of the primary walk: per-ray (steps, skips) from the CPU walker on whole
16x16 tiles, then the cost of 64-lane waves (max over lanes) without and with compacting
the unfinished rays of a tile after a budget.  Usage: python tools/wavecost.py [C1]"""
import ctypes as C, os, subprocess, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as g
so = "/tmp/walkstats.so"
subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-std=c++17", "-ffp-contract=off", "-I",
                f"{REPO}/raytracer-voxpopuli_amd/csrc", f"{REPO}/tools/native/walkstats.cpp", "-o", so], check=True)
lib = C.CDLL(so)
V = C.c_void_p
pkg, orc = g.load_package(), g.load_oracle()
cfg = sys.argv[1] if len(sys.argv) > 1 else "C1"
d = pkg.scene.CONFIGS[cfg]()
o = orc.Oracle(pkg.abi, d)
cells = o.cells[0]; n = d.grids[0].n
nb = [(n + 3) // 4]; nb.append((nb[0] + 3) // 4); nb.append((nb[1] + 3) // 4)
l1, l2 = np.zeros(nb[1] ** 3 * 64, np.uint64), np.zeros(nb[2] ** 3 * 64, np.uint64)
lib.build_masks.argtypes = [V, C.c_uint32, V, V]
lib.build_masks(cells.ctypes.data, n, l1.ctypes.data, l2.ctypes.data)
W, H = d.width, d.height
rng = np.random.default_rng(1)
T = 200
tx, ty = rng.integers(0, W // 16, T), rng.integers(0, H // 16, T)
xs = (tx[:, None] * 16 + np.arange(256)[None, :] % 16).reshape(-1)
ys = (ty[:, None] * 16 + np.arange(256)[None, :] // 16).reshape(-1)
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
ds = (D < 0).astype(np.float32)
pos = (cp + D * (t0[:, None] + np.float32(5e-5))) * np.float32(n)
P0 = np.clip(pos.astype(np.int64), 0, n - 1)
step = (1 - 2 * ds).astype(np.int32)
cell = np.float32(1.0 / n)
tdel = (cell * step.astype(np.float32)) * rD
tmax = ((np.ceil(pos) - ds) * cell - cp) * rD
st = np.ascontiguousarray(np.concatenate([t0[:, None], tmax, tdel], 1).astype(np.float32))
si = np.ascontiguousarray(np.concatenate([P0, step], 1).astype(np.int32))
per = np.zeros((len(st), 2), np.uint32)
out = np.zeros(8, np.uint64)
lib.walk_sim.argtypes = [V, V, V, C.c_uint32, V, V, V, C.c_uint32, V, V, V]
bnd = np.full(len(st), 1e34, np.float32)
MODE = int(os.environ.get("MODE", "0"))  # walkstats box experiments (1: anisotropic slabs)
if MODE:
    nbk = nb[0]
    bocc = np.ascontiguousarray((np.pad(cells.reshape(n, n, n), [(0, nbk * 4 - n)] * 3, constant_values=255)
                                .reshape(nbk, 4, nbk, 4, nbk, 4) != 255).any(axis=(1, 3, 5)).astype(np.uint8))
    lib.build_slabs.argtypes = [V, C.c_uint32]
    lib.build_slabs(bocc.ctypes.data, nbk)
    lib.set_mode.argtypes = [C.c_int]
    lib.set_mode(MODE)
lib.walk_sim(cells.ctypes.data, l1.ctypes.data, l2.ctypes.data, n, st.ctypes.data, si.ctypes.data, bnd.ctypes.data,
             len(st), out.ctypes.data, None, per.ctypes.data)
SKIP = float(os.environ.get("SKIPCOST", "5.8"))
cost = (per[:, 0] + per[:, 1] + 1) + SKIP * per[:, 1]
cost = np.where(ok, cost, 0).reshape(T, 256)
okt = ok.reshape(T, 256)
def waves(c):  # c: costs of the rays to walk, in order -> sum over 64-lane waves of the max
    return sum(c[i:i + 64].max() for i in range(0, len(c), 64)) if len(c) else 0
base = sum(waves(cost[t][okt[t]]) for t in range(T))
ideal = cost.sum() / 64
print(f"{cfg}: {okt.sum()} walking rays in {T} tiles; mean cost {cost[okt].mean():.1f}, p99 {np.percentile(cost[okt], 99):.0f}")
print(f"  no compaction: {base:.0f}   perfect packing bound: {ideal:.0f} ({base / ideal:.2f}x)")
for B in (20, 40, 60, 80, 120):
    tot = 0
    for t in range(T):
        c = cost[t][okt[t]]
        nw = (len(c) + 63) // 64
        first = sum(min(B, c[i:i + 64].max()) for i in range(0, len(c), 64))
        rem = c[c > B] - B
        tot += first + waves(rem)
    print(f"  compact after {B:4d}: {tot:.0f} ({tot / base:.2f} of no compaction)")
# Ordering the tile's walking rays by their cost before dealing them to waves (e.g. sorted
# by the previous frame's per-pixel walk cost): sum over waves of the max.
srt = sum(waves(np.sort(cost[t][okt[t]])) for t in range(T))
print(f"  sorted by cost within the tile: {srt:.0f} ({srt / base:.2f} of pixel order)")
for q in (4, 8, 16):  # coarse buckets of the cost (what a counting sort on a quantised cost gives)
    tot = 0
    for t in range(T):
        c = cost[t][okt[t]]
        key = np.minimum((c * q / max(c.max() if len(c) else 1, 1)).astype(int), q - 1)
        tot += waves(c[np.argsort(key, kind="stable")])
    print(f"  {q} cost buckets: {tot:.0f} ({tot / base:.2f})")
