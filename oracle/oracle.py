"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module; it is the checker, never the thing measured or shipped.  Parity status of the
trace path: UNPINNED (see vpx_oracle.h and DESIGN.md §3).
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
# the same source built -O3 -march=x86-64-v3 (AVX2/FMA/BMI2: the reference's /arch:AVX2) with
# -ffp-contract=off, so bit-identical results (tests/test_cpu_oracle.py); bench.py's
# cpu_baseline times this build
PERF_LIB_PATH = os.path.join(HERE, "liboracle_perf.so")
_LIBS = {}


def build(target="liboracle.so"):
    subprocess.run(["make", "-s", "-C", HERE, target], check=True)


def _lib(abi, perf=False):
    path = PERF_LIB_PATH if perf else LIB_PATH
    if path in _LIBS:
        return _LIBS[path]
    if not os.path.exists(path):
        build(os.path.basename(path))
    lib = C.CDLL(path)
    P = C.POINTER
    lib.oracle_find_nearest.argtypes = [C.c_void_p, P(abi.Ray), C.c_uint32, P(abi.Hit)]
    lib.oracle_is_occluded.argtypes = [C.c_void_p, P(abi.Ray), C.c_uint32, C.c_void_p, C.c_void_p]
    lib.oracle_trace.argtypes = [C.c_void_p, P(abi.Ray), C.c_void_p, C.c_uint32, C.c_int32, P(C.c_float), C.c_int32,
                                 C.c_void_p, P(abi.Stats)]
    lib.oracle_render_pixels.argtypes = [C.c_void_p, P(abi.FrameParams), C.c_void_p, C.c_uint32, C.c_void_p,
                                         P(abi.Stats), C.c_int]
    lib.oracle_render_reproject.argtypes = [C.c_void_p, P(abi.FrameParams), P(abi.PrevCamera), C.c_void_p,
                                            C.c_void_p, P(abi.Stats), C.c_int]
    lib.oracle_render.argtypes = [C.c_void_p, P(abi.FrameParams), C.c_void_p, C.c_void_p, P(abi.Stats), C.c_int]
    lib.oracle_accumulate_tonemap.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]
    lib.oracle_accumulate_tonemap.restype = None
    lib.oracle_focus_distance.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
    lib.oracle_focus_distance.restype = C.c_float
    lib.oracle_load_model.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, P(C.c_float),
                                      C.c_void_p]
    lib.oracle_load_model.restype = None
    lib.oracle_load_model_partial.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                              P(C.c_float), C.c_uint32, C.c_uint32, C.c_void_p]
    lib.oracle_load_model_partial.restype = None
    lib.oracle_emissive_sphere.argtypes = [C.c_void_p, C.c_uint32, C.c_uint8, C.c_float]
    lib.oracle_emissive_sphere.restype = None
    lib.oracle_orient_model.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p]
    lib.oracle_orient_model.restype = None
    lib.oracle_tiled_world.argtypes = [C.c_void_p] + [C.c_uint32] * 8 + [C.c_void_p]
    lib.oracle_tiled_world.restype = None
    lib.oracle_grid_checksum.argtypes = [C.c_void_p, C.c_uint64]
    lib.oracle_grid_checksum.restype = C.c_uint64
    lib.oracle_wang_hash.argtypes = [C.c_uint32]
    lib.oracle_wang_hash.restype = C.c_uint32
    lib.oracle_xorshift32.argtypes = [P(C.c_uint32)]
    lib.oracle_xorshift32.restype = C.c_uint32
    lib.oracle_random_float.argtypes = [P(C.c_uint32)]
    lib.oracle_random_float.restype = C.c_float
    lib.oracle_pixel_seed.argtypes = [C.c_uint32] * 6
    lib.oracle_pixel_seed.restype = C.c_uint32
    lib.oracle_offset_ray.argtypes = [P(C.c_float), P(C.c_float), P(C.c_float)]
    lib.oracle_offset_ray.restype = None
    lib.oracle_cube_intersect.argtypes = [P(C.c_float)] * 5
    lib.oracle_cube_intersect.restype = C.c_float
    lib.oracle_bvh_random_tris.argtypes = [C.c_uint32, P(abi.BvhTri)]
    lib.oracle_bvh_random_tris.restype = C.c_uint32
    lib.oracle_bvh_build.argtypes = [P(abi.BvhTri), C.c_uint32, P(abi.BvhNode), P(C.c_uint32)]
    lib.oracle_bvh_build.restype = C.c_uint32
    lib.oracle_bvh_intersect.argtypes = [P(abi.BvhNode), P(abi.BvhTri), P(C.c_uint32), P(abi.Ray), C.c_uint32,
                                         P(C.c_float)]
    lib.oracle_bvh_intersect.restype = C.c_int
    _LIBS[path] = lib
    return lib


def set_x86_approx(abi, on, perf=False):
    """The reference's x86 arithmetic in the restatement (oracle_set_x86_approx): FindNearest's
    FastReciprocal and the primary rsqrtps normalise computed with this host's rcpss / rsqrtss
    (renderer.cpp:929-934, tmpl8math.h:2356-2360); process-wide for that build of the library."""
    lib = _lib(abi, perf)
    lib.oracle_set_x86_approx.argtypes = [C.c_int]
    return lib.oracle_set_x86_approx(1 if on else 0)


class BasicBVH:
    """src/BVH/BasicBVH.{h,cpp} restated (oracle_bvh_*): build once, intersect rays."""

    def __init__(self, abi, tris):
        self.lib = _lib(abi)
        self.abi = abi
        n = len(tris)
        self.tris = tris
        self.nodes = (abi.BvhNode * max(1, 2 * n - 1))()
        self.idx = (C.c_uint32 * max(1, n))()
        self.used = self.lib.oracle_bvh_build(tris, n, self.nodes, self.idx)

    @staticmethod
    def random_tris(abi, seed=0x12345678):
        """BasicBVH::BasicBVH()'s 64 triangles from xorshift32 state `seed`; (tris, state after)."""
        tris = (abi.BvhTri * 64)()
        after = _lib(abi).oracle_bvh_random_tris(seed, tris)
        return tris, after

    def intersect(self, rays):
        out = np.zeros(len(rays), np.float32)
        rc = self.lib.oracle_bvh_intersect(self.nodes, self.tris, self.idx, rays, len(rays),
                                           out.ctypes.data_as(C.POINTER(C.c_float)))
        assert rc == 0
        return out


class OracleGrid(C.Structure):
    _fields_ = [("cells", C.c_void_p), ("n", C.c_uint32)]


def _scene_struct(abi):
    class OracleScene(C.Structure):
        _fields_ = [("grids", C.POINTER(OracleGrid)), ("num_grids", C.c_uint32),
                    ("volumes", C.POINTER(abi.Volume)), ("num_volumes", C.c_uint32),
                    ("materials", C.POINTER(abi.Material)),
                    ("points", C.POINTER(abi.PointLight)), ("num_points", C.c_uint32),
                    ("spots", C.POINTER(abi.SpotLight)), ("num_spots", C.c_uint32),
                    ("areas", C.POINTER(abi.AreaLight)), ("num_areas", C.c_uint32),
                    ("dir", abi.DirLight),
                    ("spheres", C.POINTER(abi.Sphere)), ("num_spheres", C.c_uint32),
                    ("triangles", C.POINTER(abi.Triangle)), ("num_triangles", C.c_uint32),
                    ("camera", abi.Camera),
                    ("sky_pixels", C.c_void_p), ("sky_w", C.c_uint32), ("sky_h", C.c_uint32),
                    ("sky_hdr", C.c_float)]
    return OracleScene


class Oracle:
    """CPU restatement bound to one SceneDesc (grids materialised on the host)."""

    def __init__(self, abi, desc, grid_cells=None, perf=False):
        self.abi = abi
        self.lib = _lib(abi, perf)
        self.desc = desc
        self._keep = []
        cells = grid_cells if grid_cells is not None else [self.host_grid(g) for g in desc.grids]
        self.cells = [np.ascontiguousarray(c, np.uint8) for c in cells]
        grids = (OracleGrid * len(self.cells))(*[OracleGrid(c.ctypes.data, g.n) for c, g in zip(self.cells, desc.grids)])
        S = _scene_struct(abi)
        s = S()
        s.grids, s.num_grids = grids, len(self.cells)
        s.volumes, s.num_volumes = desc.volumes, len(desc.volumes)
        s.materials = desc.materials
        arr = lambda T, xs: (T * max(1, len(xs)))(*xs)
        pts, sps, ars = arr(abi.PointLight, desc.points), arr(abi.SpotLight, desc.spots), arr(abi.AreaLight, desc.areas)
        s.points, s.num_points = pts, len(desc.points)
        s.spots, s.num_spots = sps, len(desc.spots)
        s.areas, s.num_areas = ars, len(desc.areas)
        s.dir = desc.dir_light
        sph, tri = arr(abi.Sphere, desc.spheres), arr(abi.Triangle, desc.triangles)
        s.spheres, s.num_spheres = sph, len(desc.spheres)
        s.triangles, s.num_triangles = tri, len(desc.triangles)
        s.camera = desc.camera
        self._keep += [grids, pts, sps, ars, sph, tri]
        self.s = s
        self.set_sky(getattr(desc, "sky_texture", None), getattr(desc, "sky_hdr", 1.0))

    def set_sky(self, rgb, hdr_contribution=1.0):
        if rgb is None:
            self.s.sky_pixels, self.s.sky_w, self.s.sky_h = None, 0, 0
            return
        a = np.ascontiguousarray(rgb, np.float32)
        self._sky = a
        self.s.sky_pixels, self.s.sky_h, self.s.sky_w = a.ctypes.data, a.shape[0], a.shape[1]
        self.s.sky_hdr = float(hdr_contribution)

    def host_grid(self, spec):
        """Materialise a GridSpec on the host with the oracle's own generator."""
        if spec.dense is not None:
            return spec.dense
        n = spec.n
        out = np.empty(n * n * n, np.uint8)
        m = np.ascontiguousarray(spec.model, np.uint8)
        mx, my, mz = spec.model_dims
        px, py, pz = spec.period
        self.lib.oracle_tiled_world(m.ctypes.data, mx, my, mz, px, py, pz, spec.ground, n, out.ctypes.data)
        return out

    def set_camera(self, cam):
        self.s.camera = cam

    @property
    def ptr(self):
        return C.byref(self.s)

    def find_nearest(self, rays):
        n = len(rays)
        hits = (self.abi.Hit * max(1, n))()
        assert self.lib.oracle_find_nearest(self.ptr, rays, n, hits) == 0
        return hits

    def is_occluded(self, rays):
        n = len(rays)
        occ = np.zeros(max(1, n), np.uint8)
        cells = np.zeros(max(1, n), np.uint32)
        assert self.lib.oracle_is_occluded(self.ptr, rays, n, occ.ctypes.data, cells.ctypes.data) == 0
        return occ[:n], cells[:n]

    def trace(self, rays, seeds, depth, sky, area_samples=3):
        n = len(rays)
        seeds = np.ascontiguousarray(seeds, np.uint32)
        out = np.zeros((max(1, n), 3), np.float32)
        st = self.abi.Stats()
        assert self.lib.oracle_trace(self.ptr, rays, seeds.ctypes.data, n, depth, self.abi.sky_arg(sky), area_samples,
                                     out.ctypes.data, C.byref(st)) == 0
        return out[:n], st

    def render_pixels(self, params, pixel_ids, threads=0):
        ids = np.ascontiguousarray(pixel_ids, np.uint32)
        out = np.zeros((max(1, len(ids)), 4), np.float32)
        st = self.abi.Stats()
        assert self.lib.oracle_render_pixels(self.ptr, C.byref(params), ids.ctypes.data, len(ids), out.ctypes.data,
                                             C.byref(st), threads) == 0
        return out[: len(ids)], st

    def render(self, params, accum=None, threads=0):
        w, h = params.width, params.height
        acc = np.zeros((h * w, 4), np.float32) if accum is None else accum
        rgb = np.zeros(h * w, np.uint32)
        st = self.abi.Stats()
        assert self.lib.oracle_render(self.ptr, C.byref(params), acc.ctypes.data, rgb.ctypes.data, C.byref(st),
                                      threads) == 0
        return acc, rgb, st

    def render_reproject(self, params, prev, history, threads=0):
        """One static-camera frame; history float32[H*W, 4] updated in place."""
        rgb = np.zeros(params.width * params.height, np.uint32)
        st = self.abi.Stats()
        assert self.lib.oracle_render_reproject(self.ptr, C.byref(params), C.byref(prev), history.ctypes.data,
                                                rgb.ctypes.data, C.byref(st), threads) == 0
        return rgb, st

    def focus_distance(self, width, height):
        return self.lib.oracle_focus_distance(self.ptr, width, height)
