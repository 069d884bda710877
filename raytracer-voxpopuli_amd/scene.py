"""Scene descriptions for the trace path: worlds, volumes, materials, lights, camera.

Everything here is HOST-side input preparation restating the reference's scene setup:
  - models: `decode_vox(path)` decodes a MagicaVoxel .vox file with the library's own
    decoder (vpx_vox_decode: what ogt_vox hands Scene::LoadModel, template/scene.cpp:
    474-475).  The benchmark / test workloads (C0-C4) name the reference's assets
    (teapot, monu3, roomGlass); the .vox files themselves do not travel with this repo,
    so `load_model(name)` decodes `<VPX_ASSETS_DIR>/<name>.vox` when that directory is
    given and otherwise reads the package's decoded asset store `assets/<name>.npz` (models[0]
    + palette of all 12 reference assets as ogt_vox returns them; tests/test_vox_decode.py
    checks vpx_vox_decode against the test fixtures and the store against the fixtures);
  - `load_model_grid`  Scene::LoadModel placement      template/scene.cpp:449-529
  - `palette_materials` LoadModel's palette override    template/scene.cpp:516-520
  - lights / materials / camera defaults                renderer.cpp:93-100,357-443; camera.h
  - the build-defined tiled worlds of SURVEY.md §8(d) (C1/C2/C3/C4): the reference has no
    world larger than 128^3 of its own (every .vox is <= 126 voxels a side).
The device never sees this module's numpy arrays except through libvpx_hip.so uploads.
"""
import ctypes as C
import dataclasses
import math
import os

import numpy as np

from . import abi

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
ASSETS = os.path.join(HERE, "assets")  # decoded models (no test data is read by the product)
NONE = abi.MAT_NONE


# ----------------------------------------------------------------------------- models
def decode_vox(src):
    """A .vox file (path or bytes) -> (size[3], voxels uint8[sx*sy*sz], palette uint8[256,4])
    through vpx_vox_decode (models[0] and the palette as ogt_vox v0.997 returns them)."""
    data = src if isinstance(src, (bytes, bytearray)) else open(src, "rb").read()
    lib = abi.load_library()
    buf = (C.c_uint8 * max(1, len(data))).from_buffer_copy(bytes(data) or b"\0")
    size = (C.c_uint32 * 3)()
    abi.check(lib, None, lib.vpx_vox_decode(buf, len(data), size, None, 0, None), "vpx_vox_decode (size)")
    n = int(size[0]) * int(size[1]) * int(size[2])
    vox = np.empty(n, np.uint8)
    pal = np.empty((256, 4), np.uint8)
    abi.check(lib, None, lib.vpx_vox_decode(buf, len(data), size, vox.ctypes.data, n, pal.ctypes.data),
              "vpx_vox_decode")
    return np.array(size[:], np.int64), vox, pal


def load_model(name):
    """(size[3], voxels uint8[sx*sy*sz], palette uint8[256,4]) as ogt_vox returns them:
    decoded from $VPX_ASSETS_DIR/<name>.vox when set, else from the package's asset store."""
    d = os.environ.get("VPX_ASSETS_DIR")
    if d:
        return decode_vox(os.path.join(d, name + ".vox"))
    z = np.load(os.path.join(ASSETS, name + ".npz"))
    return z["size"].astype(np.int64), z["voxels"].astype(np.uint8), z["palette"].astype(np.uint8)


def orient_model(size, voxels):
    """Grid-oriented model (x, z, y) as LoadModel places it; empty -> NONE.
    Returns (array[mz, my, mx], (mx, my, mz)) with index x + y*mx + z*mx*my."""
    sx, sy, sz = (int(v) for v in size)
    v = voxels.reshape(sz, sy, sx)
    o = np.ascontiguousarray(v.transpose(1, 0, 2))  # [y_model][z_model][x] = [gz][gy][gx]
    o = np.where(o == 0, np.uint8(NONE), o).astype(np.uint8)
    return o, (sx, sz, sy)


def load_model_grid(size, voxels, n, scale_model=(1.0, 1.0, 1.0)):
    """Scene::LoadModel into an n^3 grid (template/scene.cpp:449-529): ResetGrid() to
    NONE, downscale only when size_x > n, (x, y, z) -> (x*s.x, z*s.y, y*s.z)."""
    sx, sy, sz = (int(v) for v in size)
    scl = np.array(scale_model, np.float32)
    if sx > n:
        scl = scl * (np.float32(n) / np.array([sx, sy, sz], np.float32))
    grid = np.full(n * n * n, NONE, np.uint8)
    v = voxels.reshape(sz, sy, sx)
    zz, yy, xx = np.nonzero(v)
    vals = v[zz, yy, xx]
    gx = (xx.astype(np.float32) * scl[0]).astype(np.int64)
    gy = (zz.astype(np.float32) * scl[1]).astype(np.int64)
    gz = (yy.astype(np.float32) * scl[2]).astype(np.int64)
    ok = (gx >= 0) & (gy >= 0) & (gz >= 0) & (gx < n) & (gy < n) & (gz < n)
    idx = gx[ok] + gy[ok] * n + gz[ok] * n * n
    # later voxels (z-major, then y, then x) overwrite earlier ones, as the loop does:
    # keep the last occurrence of every target cell explicitly
    order = np.lexsort((xx[ok], yy[ok], zz[ok]))
    tgt, val = idx[order], vals[ok][order]
    _, last = np.unique(tgt[::-1], return_index=True)
    keep = len(tgt) - 1 - last
    grid[tgt[keep]] = val[keep]
    return grid


def load_model_partial(size, voxels, n, columns, thickness, scale_model=(1.0, 1.0, 1.0)):
    """Scene::LoadModelPartial (template/scene.cpp:531-604), as ModifyingProp::Update calls
    it every 0.9 s (src/Game/ModifyingProp.cpp:11-21): ResetGrid() to NONE, LoadModel's
    mapping, only voxels with x in [columns - thickness, columns + thickness] (uint32
    arithmetic: the lower bound wraps when thickness > columns).  Returns (grid, box)
    where box = (x0, y0, z0, x1, y1, z1) bounds the non-NONE cells (None if empty) —
    the dirty region to upload after a device-side ResetGrid."""
    sx = int(size[0])
    v = np.asarray(voxels, np.uint8).reshape(int(size[2]), int(size[1]), sx).copy()
    lo, hi = (int(columns) - int(thickness)) % (1 << 32), int(columns) + int(thickness)
    keep = (np.arange(sx) >= lo) & (np.arange(sx) <= hi)
    v[:, :, ~keep] = 0
    grid = load_model_grid(size, v.reshape(-1), n, scale_model)
    nz = np.nonzero(grid.reshape(n, n, n) != NONE)
    if len(nz[0]) == 0:
        return grid, None
    z, y, x = nz
    return grid, (int(x.min()), int(y.min()), int(z.min()), int(x.max()) + 1, int(y.max()) + 1, int(z.max()) + 1)


def default_materials():
    lib = abi.load_library()
    mats = (abi.Material * 256)()
    abi.check(lib, None, lib.vpx_default_materials(mats), "vpx_default_materials")
    return mats


def palette_materials(mats, voxels, palette):
    """LoadModel's palette override (template/scene.cpp:516-520): every used index gets
    albedo = rgb/255 and roughness 1."""
    for i in np.unique(voxels[voxels > 0]):
        c = palette[int(i)]
        m = mats[int(i)]
        for k in range(3):
            m.albedo[k] = float(np.float32(c[k]) / np.float32(255.0))
        m.roughness = 1.0
    return mats


# ------------------------------------------------------------------------------ grids
@dataclasses.dataclass
class GridSpec:
    """A voxel grid: either dense host bytes or the build-defined tiled generator."""
    n: int
    dense: np.ndarray = None          # uint8[n^3], index x + y*n + z*n*n
    model: np.ndarray = None          # grid-oriented model for the tiled generator
    model_dims: tuple = None          # (mx, my, mz)
    period: tuple = None              # (px, py, pz)
    ground: int = 2

    def upload(self, lib, ctx, grid_id):
        if self.dense is not None:
            arr = np.ascontiguousarray(self.dense, np.uint8)
            abi.check(lib, ctx, lib.vpx_upload_grid(ctx, grid_id, arr.ctypes.data_as(C.c_void_p), self.n),
                      "vpx_upload_grid")
        else:
            m = np.ascontiguousarray(self.model, np.uint8)
            mx, my, mz = self.model_dims
            px, py, pz = self.period
            abi.check(lib, ctx, lib.vpx_generate_tiled_grid(ctx, grid_id, self.n, m.ctypes.data_as(C.c_void_p), mx,
                                                            my, mz, px, py, pz, self.ground),
                      "vpx_generate_tiled_grid")


def _tiled_numpy(spec):
    """Host-side tiled world (numpy), same contract as vpx_generate_tiled_grid."""
    n = spec.n
    mx, my, mz = spec.model_dims
    px, py, pz = spec.period
    m = spec.model.reshape(mz, my, mx)
    x = np.arange(n)
    lx = x % px
    okx = lx < mx
    out = np.empty((n, n, n), np.uint8)
    for z in range(n):
        lz = z % pz
        sl = out[z]
        if lz >= mz:
            sl[:] = NONE
        else:
            ys = np.arange(n)
            ly = (ys - spec.ground) % py
            oky = (ys >= spec.ground) & (ly < my)
            plane = m[lz][np.minimum(ly, my - 1)][:, np.minimum(lx, mx - 1)]
            sl[:] = np.where(oky[:, None] & okx[None, :], plane, NONE)
        sl[: spec.ground] = 0
    return out.reshape(-1)


def tiled_grid(model_name, n, ground=2, period_scale=2):
    size, vox, pal = load_model(model_name)
    o, dims = orient_model(size, vox)
    period = tuple(int(period_scale * d) for d in dims)
    return GridSpec(n=n, model=o.reshape(-1), model_dims=dims, period=period, ground=ground), vox, pal


# ------------------------------------------------------------------------------ scene
@dataclasses.dataclass
class SceneDesc:
    name: str
    grids: list
    volumes: object            # ctypes array of abi.Volume
    materials: object          # ctypes array of 256 abi.Material
    points: list
    spots: list
    areas: list
    dir_light: abi.DirLight
    camera: abi.Camera
    width: int
    height: int
    max_bounces: int = 0
    flags: int = 0
    aa_strength: float = 1.0
    area_samples: int = 3
    sky: tuple = abi.SKY_DEFAULT
    sky_texture: object = None    # float32 (H, W, 3): Renderer::skyPixels (used with VPX_FLAG_SKY)
    sky_hdr: float = 1.0          # HDRLightContribution (renderer.h:224)
    spheres: list = dataclasses.field(default_factory=list)
    triangles: list = dataclasses.field(default_factory=list)
    spp: int = 1

    def frame_params(self, frame_index=0, seed_base=0, width=None, height=None):
        p = abi.FrameParams()
        p.width = width or self.width
        p.height = height or self.height
        p.max_bounces = self.max_bounces
        p.frame_index = frame_index
        p.seed_base = seed_base
        p.flags = self.flags
        p.aa_strength = self.aa_strength
        p.area_samples = self.area_samples
        p.sky = abi.vec3(self.sky)
        return p

    def with_size(self, width, height):
        """Same scene at another resolution (camera ASPECT follows W/H, camera.h:183)."""
        d = dataclasses.replace(self, width=width, height=height)
        d.camera = look_at(self._cam_pos, self._cam_target, width, height)
        d._cam_pos, d._cam_target = self._cam_pos, self._cam_target
        return d

    def with_resolution(self, width, height):
        """Same scene and the SAME camera (its TL / TR / BL corners, camera.h:90-105) at another
        resolution: pixel (x, y) samples u = x / W, v = y / H of the same view, so more pixels
        sample it more densely (the weak-scaling frames of bench.py) instead of widening it."""
        d = dataclasses.replace(self, width=width, height=height)
        d._cam_pos, d._cam_target = self._cam_pos, self._cam_target
        return d


def synthetic_sky(width=512, height=256, sun=(0.35, 0.25)):
    """Build-defined stand-in for assets/sky_19.hdr (missing from the reference tree,
    SURVEY F7): an equirectangular RGB float image laid out like stbi_loadf's output (row v
    = polar angle acos(D.y) / pi from the zenith, column u = atan2(D.z, D.x) / 2pi).  A
    zenith-to-horizon gradient, a darker ground half and an HDR sun disc (values up to
    ~40) so that misses exercise the full float range.  Deterministic (no RNG)."""
    v = (np.arange(height, dtype=np.float64) + 0.5) / height          # 0 = zenith
    u = (np.arange(width, dtype=np.float64) + 0.5) / width
    theta = v[:, None] * np.pi
    up = np.cos(theta)
    zen = np.array([0.25, 0.45, 0.95])
    hor = np.array([0.95, 0.9, 0.85])
    gnd = np.array([0.18, 0.15, 0.12])
    a = np.clip(up, 0.0, 1.0)[..., None]
    sky = np.where((up > 0)[..., None], hor + (zen - hor) * a ** 0.6, gnd * (0.6 + 0.4 * (1 + up[..., None])))
    img = np.broadcast_to(sky, (height, width, 3)).copy()
    su, sv = sun
    du = np.minimum(np.abs(u[None, :] - su), 1 - np.abs(u[None, :] - su)) * 2.0
    dv = v[:, None] - sv
    disc = np.exp(-(du * du + dv * dv) / (2 * 0.02 ** 2))
    img += disc[..., None] * np.array([40.0, 36.0, 30.0])
    return np.ascontiguousarray(img, np.float32)


def with_sky(desc, texture=None, hdr_contribution=1.0):
    """activateSky = true with a sky texture (Renderer::skyPixels, HDRLightContribution)."""
    d = dataclasses.replace(desc, sky_texture=synthetic_sky() if texture is None else texture,
                            sky_hdr=float(hdr_contribution), flags=desc.flags | abi.VPX_FLAG_SKY)
    d._cam_pos, d._cam_target = desc._cam_pos, desc._cam_target
    return d


def look_at(pos, target, width, height):
    lib = abi.load_library()
    cam = abi.Camera()
    p = (C.c_float * 3)(*pos)
    t = (C.c_float * 3)(*target)
    abi.check(lib, None, lib.vpx_camera_look_at(p, t, width, height, C.byref(cam)), "vpx_camera_look_at")
    return cam


def prev_camera(pos, target, width, height):
    """Renderer::prevCamera after CopyToPrevCamera (renderer.cpp:710-711, 1893-1902)."""
    lib = abi.load_library()
    pc = abi.PrevCamera()
    p = (C.c_float * 3)(*pos)
    t = (C.c_float * 3)(*target)
    abi.check(lib, None, lib.vpx_prev_camera_look_at(p, t, width, height, C.byref(pc)), "vpx_prev_camera_look_at")
    return pc


def volume(position=(0.0, 0.0, 0.0), scale=(1.0, 1.0, 1.0), rotation=(0.0, 0.0, 0.0), grid_id=0):
    lib = abi.load_library()
    v = abi.Volume()
    f = lambda a: (C.c_float * 3)(*a)
    abi.check(lib, None, lib.vpx_volume_set_transform(f(position), f(scale), f(rotation), C.byref(v)),
              "vpx_volume_set_transform")
    v.grid_id = grid_id
    return v


def point_light(position=(0.5, 0.5, 3.5), color=(1.0, 1.0, 1.0)):  # PointLight.h:13
    return abi.PointLight(abi.vec3(position), abi.vec3(color))


def spot_light(position=(-1.0, 0.5, -1.0), direction=(1.0, 0.0, 0.0), color=(1.5, 1.5, 1.5),
               angle=None):  # SpotLight.h:23, angle = CosDegrees(45)
    if angle is None:
        angle = float(np.float32(math.cos(float(np.float32(45.0) * np.float32(math.pi) / np.float32(180.0)))))
    return abi.SpotLight(abi.vec3(position), abi.vec3(direction), abi.vec3(color), angle)


def area_light(position=(-0.0, 0.5, -3.5), color=(1.0, 1.0, 1.0), mult=1.2, radius=1.2):  # SphereAreaLight.h:13
    return abi.AreaLight(abi.vec3(position), abi.vec3(color), mult, radius)


def dir_light(direction=(1.0, 0.0, 0.0), color=(0.0, 0.0, 0.0)):  # DirectionalLight.h:12
    return abi.DirLight(abi.vec3(direction), abi.vec3(color))


def _scene(name, grids, vols, mats, points, spots, areas, dl, cam_pos, cam_target, w, h, **kw):
    varr = (abi.Volume * len(vols))(*vols)
    d = SceneDesc(name=name, grids=grids, volumes=varr, materials=mats, points=points, spots=spots, areas=areas,
                  dir_light=dl, camera=look_at(cam_pos, cam_target, w, h), width=w, height=h, **kw)
    d._cam_pos, d._cam_target = tuple(cam_pos), tuple(cam_target)
    return d


# ---------------------------------------------------------------------------- configs
# BASELINE.json configs; worlds and cameras beyond the reference's own are build-defined
# (SURVEY.md §8(d)).  C1 is the metric's workload.
C0_CAM = ((0.5, 0.35, -0.6), (0.5, 0.2, 0.3))
CITY_CAM = ((1.25, 0.9, -0.35), (0.45, 0.15, 0.55))
CITY_LIGHTS = dict(points=[point_light((0.5, 1.5, 0.5), (1.0, 1.0, 1.0))],
                   dir_light=dir_light((-0.3, -1.0, -0.2), (1.0, 1.0, 1.0)))


def model_scene(model="teapot", n=128, width=640, height=360, max_bounces=0, cam=C0_CAM, city_lights=False):
    """C0: the reference's own setup — Scene({0}, n) + LoadModel + SetTransform({0})."""
    size, vox, pal = load_model(model)
    grid = GridSpec(n=n, dense=load_model_grid(size, vox, n))
    mats = palette_materials(default_materials(), vox, pal)
    if city_lights:
        pts, dl = CITY_LIGHTS["points"], CITY_LIGHTS["dir_light"]
    else:
        pts, dl = [point_light()], dir_light()
    return _scene(f"{model}{n}", [grid], [volume()], mats, pts, [], [], dl, cam[0], cam[1], width, height,
                  max_bounces=max_bounces)


def city_scene(model="monu3", n=1024, width=1920, height=1080, max_bounces=0, areas=None, cam=CITY_CAM):
    """C1/C2/C3: a .vox model tiled with a 2x period above a white ground slab."""
    spec, vox, pal = tiled_grid(model, n)
    mats = palette_materials(default_materials(), vox, pal)
    pts = list(CITY_LIGHTS["points"]) if areas is None else []
    dl = CITY_LIGHTS["dir_light"]
    return _scene(f"{model}-city{n}", [spec], [volume()], mats, pts, [], list(areas or []), dl, cam[0], cam[1],
                  width, height, max_bounces=max_bounces)


def pillars_grid(n):
    """The procedural world of host/vpx_demo.cpp (same formula, for the C++-host test)."""
    z, y, x = np.meshgrid(np.arange(n, dtype=np.int64), np.arange(n, dtype=np.int64), np.arange(n, dtype=np.int64),
                          indexing="ij")
    h = ((x >> 4) * 7 + (z >> 4) * 13) % 5 * n // 16
    g = np.full((n, n, n), 255, np.uint8)
    pil = ((x & 15) < 8) & ((z & 15) < 8) & (y < 2 + h)
    g[pil] = (16 + h % 4)[pil].astype(np.uint8)
    g[y < 2] = 0
    return g.reshape(-1)


def pillars_scene(n=256, width=640, height=360, max_bounces=0):
    grid = GridSpec(n=n, dense=pillars_grid(n))
    return _scene(f"pillars{n}", [grid], [volume()], default_materials(), list(CITY_LIGHTS["points"]), [], [],
                  CITY_LIGHTS["dir_light"], CITY_CAM[0], CITY_CAM[1], width, height, max_bounces=max_bounces)


C3_AREAS = [area_light((0.5, 2.0, 0.5)), area_light((-1.5, 1.5, 0.5)), area_light((2.5, 1.5, 0.5)),
            area_light((0.5, 1.5, -1.5))]


def instanced_scene(n=2048, inst_n=64, width=3840, height=2160, model="monu3", spp=16):
    """C4: the city plus 64 transformed instances of one 64^3 model grid (4x4x4 lattice
    floating above it, scale 0.1, fixed rotations).  The reference semantics are a linear
    loop over 65 volumes (renderer.cpp:952-993)."""
    spec, vox, pal = tiled_grid(model, n)
    size, mv, _ = load_model(model)
    inst = GridSpec(n=inst_n, dense=load_model_grid(size, mv, inst_n))
    mats = palette_materials(default_materials(), vox, pal)
    vols = [volume(grid_id=0)]
    for k in range(4):
        for j in range(4):
            for i in range(4):
                c = (0.125 + 0.25 * i, 1.125 + 0.25 * j, 0.125 + 0.25 * k)
                pos = tuple(v - 0.5 for v in c)
                rot = (0.0, 0.3 * (i + 4 * j + 16 * k), 0.1 * k)
                vols.append(volume(pos, (0.1, 0.1, 0.1), rot, grid_id=1))
    return _scene(f"{model}-inst{n}", [spec, inst], vols, mats, [], [], list(C3_AREAS),
                  CITY_LIGHTS["dir_light"], (1.6, 1.9, -1.2), (0.5, 0.7, 0.5), width, height, spp=spp)


def _cos_degrees(d):
    """CosDegrees (tmpl8math.h) in float: cosf(d * PI / 180)."""
    r = np.float32(np.float32(d) * np.float32(math.pi) / np.float32(180.0))
    return float(np.float32(math.cos(float(r))))


def zone_scene(width=1920, height=1080, max_bounces=14, sky=True):
    """The reference's own scene shape: Renderer::SetUpFirstZone (renderer.cpp:592-657) with
    its CreateBridge (:482-529) and CreateBridgeBlind (:531-590), CreateTrianglePattern
    (:460-469) and SetUpLights (:93-100: 1 point light, 5 spot lights, the directional light
    with its default zero colour, renderer.cpp:638-654 for the spots), maxBounces 14
    (renderer.h:175), activateSky (renderer.h:216; the HDR asset is missing from the reference
    tree, so the synthetic sky stands in), the camera's default pose (camera.h:20-21).
    21 volumes (Scene(position, N) + SetTransform, so the reference's matrices) and 10
    triangles.  Build-defined where the reference draws at run time: the Rand() material picks
    (fixed values from the same ranges), the FastNoise2 smoke of the 64^3 checkpoint volume
    (GenerateSomeSmoke) — a deterministic smoke ball instead — and the Text model's random
    materials (LoadModelRandomMaterials) — its palette materials instead."""
    MET_LOW, GLASS, PINK = 7, 8, 4
    mats = default_materials()
    psize, pvox, ppal = load_model("player")
    tsize, tvox, tpal = load_model("Text")
    mats = palette_materials(mats, pvox, ppal)
    mats = palette_materials(mats, tvox, tpal)
    grids, gid = [], {}

    def grid(key, n, dense):
        if key not in gid:
            gid[key] = len(grids)
            grids.append(GridSpec(n=n, dense=dense))
        return gid[key]

    def solid(m):  # a 1^3 Scene after ResetGrid(m)
        return grid(f"solid{m}", 1, np.full(1, m, np.uint8))

    n = 64  # the checkpoint's smoke: a ball of smoke cells (SMOKE_LOW_DENSITY..SMOKE_PLAYER - 1)
    z, y, x = np.meshgrid(*(np.arange(n, dtype=np.float32),) * 3, indexing="ij")
    r = np.sqrt((x - 31.5) ** 2 + (y - 31.5) ** 2 + (z - 31.5) ** 2)
    smoke = np.where(r < 20.0, (9 + (r.astype(np.int64) % 5)).astype(np.uint8), np.uint8(NONE)).reshape(-1)
    vols = []

    def vol(pos, scl, g):
        vols.append(volume(pos, scl, (0.0, 0.0, 0.0), grid_id=g))

    vol((0.0, 0.0, 0.0), (1.0, 1.0, 1.0), grid("player", 16, load_model_grid(psize, pvox, 16)))  # the player
    vol((0.0, -1.0, 0.0), (5.0, 1.0, 5.0), solid(MET_LOW))  # environment (ResetGrid METAL_LOW)
    vol((6.0, 0.0, 0.0), (5.0, 5.0, 5.0), solid(MET_LOW))
    vol((-10.0, 2.0, 0.0), (5.0, 5.0, 5.0), solid(MET_LOW))
    vol((0.0, 4.0, 0.0), (10.0, 1.0, 10.0), solid(MET_LOW))
    vol((0.0, 0.3, 0.0), (3.0, 3.0, 3.0), grid("smoke", 64, smoke))  # checkpoint
    vol((0.0, 3.0, -3.0), (5.0, 5.0, 5.0), grid("text", 32, load_model_grid(tsize, tvox, 32)))  # Text
    none64 = grid("none64", 64, np.full(64 ** 3, NONE, np.uint8))
    # CreateBridge({0, 0, 0}) (enterOffset {0}, door GLASS)
    vol((0.0, 4.0, -7.0), (10.0, 1.0, 5.0), solid(1))
    vol((-1.0, 0.0, -11.0), (3.0, 10.0, 1.0), solid(GLASS))
    vol((-5.0, 1.0, -12.0), (2.0, 3.0, 10.0), solid(2))
    vol((-3.0, 1.0, -19.0), (7.0, 1.0, 1.0), solid(3))
    vol((0.0, -1.0, -18.0), (5.0, 1.0, 5.0), solid(6))  # Rand(METAL_HIGH, GLASS)
    vol((0.0, 0.3, -17.0), (2.0, 2.0, 2.0), none64)
    # CreateBridgeBlind({0, 0, -17}, {0, -6, 0}, GLASS)
    vol((0.0, -2.0, -24.0), (10.0, 1.0, 5.0), solid(0))
    vol((-1.0, 0.0, -28.0), (3.0, 10.0, 1.0), solid(GLASS))
    vol((5.0, -41.0, -29.0), (2.0, 3.0, 10.0), solid(MET_LOW))
    vol((-5.0, 1.0, -29.0), (2.0, 3.0, 10.0), solid(PINK))  # not reset: the Scene ctor's NON_METAL_PINK
    vol((3.0, 51.0, -36.0), (7.0, 1.0, 1.0), solid(GLASS))  # Rand(METAL_HIGH, GLASS)
    vol((-3.0, 1.0, -36.0), (7.0, 1.0, 1.0), solid(2))
    vol((0.0, -1.0, -35.0), (5.0, 1.0, 5.0), solid(1))
    vol((0.0, 0.3, -34.0), (2.0, 2.0, 2.0), none64)
    tris = []
    for i in range(10):  # CreateTrianglePattern: scale 0.25 from (-1.75, 0, 3), step 2 * scale
        px = float(np.float32(-1.75) + np.float32(0.5) * np.float32(i))
        tris.append(abi.Triangle(abi.vec3((px, 0.0, 3.0)), abi.vec3((-0.25, 0.0, 0.0)), abi.vec3((0.0, 0.25, 0.0)),
                                 abi.vec3((0.25, 0.0, 0.0)), i % 8, (C.c_uint32 * 3)()))
    spots = []
    fixed = [(0.9, 0.3, 0.6, 30.0), (0.2, 0.8, 0.4, 25.0), (0.7, 0.6, 0.1, 40.0)]
    for i in range(5):
        if i >= 2:
            cr, cg, cb, deg = fixed[i - 2]
            pos = (-3.0, float(np.float32(math.sin(float(i))) + np.float32(1.0)), -25.0 - 2.0 * i)
            spots.append(spot_light(pos, (1.0, 0.0, 0.0), (cr, cg, cb), _cos_degrees(deg)))
        else:
            spots.append(spot_light((0.0, 0.0, -22.0 - 3.0 * i), (0.0, 1.0, 0.0)))
    d = _scene("zone1", grids, vols, mats, [point_light()], spots, [], dir_light(), (0.0, 0.0, -2.0),
               (0.0, 0.0, -1.0), width, height, max_bounces=max_bounces)
    d.triangles = tris
    return with_sky(d) if sky else d


CONFIGS = {
    "C0": lambda: model_scene("teapot", 128, 640, 360, 0),
    "C0m": lambda: model_scene("monu3", 128, 640, 360, 0),
    "C1": lambda: city_scene("monu3", 1024, 1920, 1080, 0),
    "C2": lambda: city_scene("roomGlass", 1024, 1920, 1080, 4),
    "C3": lambda: city_scene("monu3", 2048, 3840, 2160, 0, areas=C3_AREAS),
    "C4": lambda: instanced_scene(),
    # the reference's own scene shape (SetUpFirstZone, depth 14): 21 volumes, 10 triangles,
    # point + 5 spot + directional lights (build-defined where the reference draws at run time)
    "Z1": lambda: zone_scene(1920, 1080, 14),
}
