"""Python handle on one libvpx_hip.so context (one GPU).  Thin: every call is the C-ABI."""
import ctypes as C

import numpy as np

from . import abi


class Context:
    def __init__(self, device=0, devices=None):
        """One device (vpx_create), or a device set (vpx_create_multi: `devices` list, the
        frame tile-sharded over them and gathered to devices[0])."""
        self.lib = abi.load_library()
        h = C.c_void_p()
        if devices is not None:
            arr = (C.c_int * len(devices))(*[int(d) for d in devices])
            rc = self.lib.vpx_create_multi(arr, len(devices), C.byref(h))
            if rc != abi.VPX_OK:
                raise abi.VpxError(f"vpx_create_multi(devices={list(devices)}) failed ({rc})")
            device = int(devices[0])
        else:
            rc = self.lib.vpx_create(int(device), C.byref(h))
            if rc != abi.VPX_OK:
                raise abi.VpxError(f"vpx_create(device={device}) failed ({rc}): no usable HIP device")
        self.h = h
        self.device = device
        self.devices = list(devices) if devices is not None else [device]
        self.scene = None
        self.stream_handle = None

    # ------------------------------------------------------------------ lifetime
    def close(self):
        if self.h:
            self.lib.vpx_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc, what):
        abi.check(self.lib, self.h, rc, what)

    def set_stream(self, stream_handle):
        self._chk(self.lib.vpx_set_stream(self.h, C.c_void_p(stream_handle or 0)), "vpx_set_stream")
        self.stream_handle = stream_handle or None  # None: the context's own stream

    def synchronize(self):
        self._chk(self.lib.vpx_synchronize(self.h), "vpx_synchronize")

    def set_pipeline(self, depth):
        """Frames in flight (vpx_set_pipeline): 0 / 1 off, 2..4 lanes."""
        self._chk(self.lib.vpx_set_pipeline(self.h, int(depth)), "vpx_set_pipeline")

    def set_arithmetic(self, mode):
        """vpx_set_arithmetic: abi.VPX_ARITH_EXACT (default) or abi.VPX_ARITH_X86_HOST (the
        reference's rcpps+NR / rsqrtps as this host's CPU computes them)."""
        self._chk(self.lib.vpx_set_arithmetic(self.h, int(mode)), "vpx_set_arithmetic")

    # ------------------------------------------------------------------- scene
    def load_scene(self, desc, upload_grids=True):
        if upload_grids:
            for gid, g in enumerate(desc.grids):
                g.upload(self.lib, self.h, gid)
        self._chk(self.lib.vpx_set_volumes(self.h, desc.volumes, len(desc.volumes)), "vpx_set_volumes")
        self._chk(self.lib.vpx_set_materials(self.h, desc.materials, 256), "vpx_set_materials")
        pts = (abi.PointLight * max(1, len(desc.points)))(*desc.points)
        sps = (abi.SpotLight * max(1, len(desc.spots)))(*desc.spots)
        ars = (abi.AreaLight * max(1, len(desc.areas)))(*desc.areas)
        self._chk(self.lib.vpx_set_lights(self.h, pts, len(desc.points), sps, len(desc.spots), ars, len(desc.areas),
                                          C.byref(desc.dir_light)), "vpx_set_lights")
        sph = (abi.Sphere * max(1, len(desc.spheres)))(*desc.spheres)
        tri = (abi.Triangle * max(1, len(desc.triangles)))(*desc.triangles)
        self._chk(self.lib.vpx_set_shapes(self.h, sph, len(desc.spheres), tri, len(desc.triangles)),
                  "vpx_set_shapes")
        self.set_camera(desc.camera)
        self.set_sky(desc.sky_texture, desc.sky_hdr)
        self.scene = desc

    def set_sky(self, rgb, hdr_contribution=1.0):
        """Renderer::skyPixels (float32 (H, W, 3) equirectangular) + HDRLightContribution;
        None removes the texture."""
        if rgb is None:
            self._chk(self.lib.vpx_set_sky(self.h, None, 0, 0, float(hdr_contribution)), "vpx_set_sky")
            return
        a = np.ascontiguousarray(rgb, np.float32)
        h, w, ch = a.shape
        assert ch == 3, "sky texture must be (H, W, 3) RGB floats"
        self._chk(self.lib.vpx_set_sky(self.h, a.ctypes.data_as(C.c_void_p), w, h, float(hdr_contribution)),
                  "vpx_set_sky")

    def set_camera(self, cam):
        self._chk(self.lib.vpx_set_camera(self.h, C.byref(cam)), "vpx_set_camera")

    # ------------------------------------------------------------ world edits
    def grid_fill(self, grid_id, value):
        """Scene::ResetGrid(type) (template/scene.cpp:356-359) on the device copy."""
        self._chk(self.lib.vpx_grid_fill(self.h, grid_id, int(value)), "vpx_grid_fill")

    def grid_write_box(self, grid_id, box, origin):
        """Dirty-region upload: box = uint8 array (dz, dy, dx) written at origin (x0, y0, z0)."""
        b = np.ascontiguousarray(box, np.uint8)
        dz, dy, dx = b.shape
        x0, y0, z0 = origin
        self._chk(self.lib.vpx_grid_write_box(self.h, grid_id, b.ctypes.data_as(C.c_void_p), x0, y0, z0, dx, dy, dz),
                  "vpx_grid_write_box")

    def grid_emissive_sphere(self, grid_id, mat, radius):
        """Scene::CreateEmmisiveSphere(mat, radius) (template/scene.cpp:685-711)."""
        self._chk(self.lib.vpx_grid_emissive_sphere(self.h, grid_id, int(mat), float(radius)),
                  "vpx_grid_emissive_sphere")

    def grid_checksum(self, grid_id=0):
        out = C.c_uint64()
        self._chk(self.lib.vpx_grid_checksum(self.h, grid_id, C.byref(out)), "vpx_grid_checksum")
        return out.value

    # ---------------------------------------------------------------- hot path
    def render(self, params, accum_ptr, rgb_ptr=None, stats=False):
        st = abi.Stats() if stats else None
        self._chk(self.lib.vpx_render(self.h, C.byref(params), C.c_void_p(accum_ptr), C.c_void_p(rgb_ptr or 0),
                                      C.byref(st) if st is not None else None), "vpx_render")
        return st

    def render_reproject(self, params, prev, history_ptr, rgb_ptr=None, stats=False):
        """One frame of the static-camera path (vpx_render_reproject); history is a DEVICE
        float4[W*H] pointer (illuminationHistoryBuffer, updated in place)."""
        st = abi.Stats() if stats else None
        self._chk(self.lib.vpx_render_reproject(self.h, C.byref(params), C.byref(prev), C.c_void_p(history_ptr),
                                                C.c_void_p(rgb_ptr or 0), C.byref(st) if st is not None else None),
                  "vpx_render_reproject")
        return st

    def render_tiles(self, params, rank, n_ranks, packed_ptr, stats=False, tile=16):
        st = abi.Stats() if stats else None
        self._chk(self.lib.vpx_render_tiles(self.h, C.byref(params), tile, tile, rank, n_ranks,
                                            C.c_void_p(packed_ptr), C.byref(st) if st is not None else None),
                  "vpx_render_tiles")
        return st

    def render_tiles_accum(self, params, rank, n_ranks, accum_packed_ptr, rgb_packed_ptr, stats=False, tile=16):
        """This rank's tiles, accumulated into its own packed accumulator + packed RGB8."""
        st = abi.Stats() if stats else None
        self._chk(self.lib.vpx_render_tiles_accum(self.h, C.byref(params), tile, tile, rank, n_ranks,
                                                  C.c_void_p(accum_packed_ptr), C.c_void_p(rgb_packed_ptr),
                                                  C.byref(st) if st is not None else None), "vpx_render_tiles_accum")
        return st

    def render_window(self, params, n_frames, accum_ptr, rgb_ptr=None):
        """Frames params.frame_index .. + n_frames - 1 accumulated in order (vpx_render_window):
        the results of n_frames render() calls; small frames share one chain of launches."""
        self._chk(self.lib.vpx_render_window(self.h, C.byref(params), n_frames, C.c_void_p(accum_ptr),
                                             C.c_void_p(rgb_ptr or 0)), "vpx_render_window")

    def render_tiles_accum_window(self, params, n_frames, rank, n_ranks, accum_packed_ptr, rgb_packed_ptr, tile=16):
        """render_tiles_accum over an accumulation window (vpx_render_tiles_accum_window): the
        rank's share of several frames in one chain of launches."""
        self._chk(self.lib.vpx_render_tiles_accum_window(self.h, C.byref(params), n_frames, tile, tile, rank, n_ranks,
                                                         C.c_void_p(accum_packed_ptr), C.c_void_p(rgb_packed_ptr)),
                  "vpx_render_tiles_accum_window")

    def composite_rgb8(self, params, n_ranks, gathered_ptr, rgb_ptr, tile=16):
        self._chk(self.lib.vpx_composite_rgb8(self.h, C.byref(params), tile, tile, n_ranks, C.c_void_p(gathered_ptr),
                                              C.c_void_p(rgb_ptr)), "vpx_composite_rgb8")

    def packed_len(self, width, height, n_ranks, tile=16):
        return int(self.lib.vpx_tiles_packed_len(width, height, tile, tile, n_ranks))

    def composite_tiles(self, params, n_ranks, gathered_ptr, accum_ptr, rgb_ptr=None, tile=16):
        self._chk(self.lib.vpx_composite_tiles(self.h, C.byref(params), tile, tile, n_ranks, C.c_void_p(gathered_ptr),
                                               C.c_void_p(accum_ptr), C.c_void_p(rgb_ptr or 0)),
                  "vpx_composite_tiles")

    def profile_enable(self, max_launches):
        self._chk(self.lib.vpx_profile_enable(self.h, int(max_launches)), "vpx_profile_enable")

    def bvh_set(self, tris):
        """BasicBVH of `tris` (ctypes array of abi.BvhTri) built and uploaded (vpx_bvh_set)."""
        self._chk(self.lib.vpx_bvh_set(self.h, tris, len(tris)), "vpx_bvh_set")

    def bvh_intersect(self, rays):
        """BasicBVH::IntersectBVH per ray: float32 t after the traversal."""
        out = np.zeros(len(rays), np.float32)
        self._chk(self.lib.vpx_bvh_intersect(self.h, rays, len(rays), out.ctypes.data_as(C.POINTER(C.c_float))),
                  "vpx_bvh_intersect")
        return out

    def profile_select(self, stages=None):
        """Time only these stage names (abi.STAGES); None: all."""
        mask = 0xFFFFFFFF if stages is None else sum(1 << abi.STAGES.index(s) for s in stages)
        self._chk(self.lib.vpx_profile_select(self.h, mask), "vpx_profile_select")

    def profile_read(self, reset=True):
        """Per-stage device times / launches / DDA cells / busy time (the union of the launch
        intervals): {stage: (ms_total, launches, cells, busy_ms)}."""
        pr = abi.Profile()
        self._chk(self.lib.vpx_profile_read(self.h, C.byref(pr), 1 if reset else 0), "vpx_profile_read")
        return {name: (pr.stage_ms[i], pr.stage_launches[i], pr.stage_cells[i], pr.stage_busy_ms[i])
                for i, name in enumerate(abi.STAGES)}

    def counters(self, reset=False):
        st = abi.Stats()
        self._chk(self.lib.vpx_get_counters(self.h, C.byref(st), 1 if reset else 0), "vpx_get_counters")
        return st

    # ------------------------------------------------------------- unit entries
    def find_nearest(self, rays):
        n = len(rays)
        hits = (abi.Hit * max(1, n))()
        self._chk(self.lib.vpx_find_nearest(self.h, rays, n, hits), "vpx_find_nearest")
        return hits

    def is_occluded(self, rays):
        n = len(rays)
        occ = np.zeros(max(1, n), np.uint8)
        self._chk(self.lib.vpx_is_occluded(self.h, rays, n, occ.ctypes.data_as(C.c_void_p)), "vpx_is_occluded")
        return occ[:n]

    def trace(self, rays, seeds, depth, sky=abi.SKY_DEFAULT, area_samples=3):
        """Renderer::Trace per ray; sky=None samples the sky texture (activateSky)."""
        n = len(rays)
        seeds = np.ascontiguousarray(seeds, np.uint32)
        out = np.zeros((max(1, n), 3), np.float32)
        self._chk(self.lib.vpx_trace(self.h, rays, seeds.ctypes.data_as(C.c_void_p), n, depth, abi.sky_arg(sky),
                                     area_samples, out.ctypes.data_as(C.c_void_p)), "vpx_trace")
        return out[:n]

    def focus_distance(self, width, height):
        f = C.c_float()
        self._chk(self.lib.vpx_focus_distance(self.h, width, height, C.byref(f)), "vpx_focus_distance")
        return f.value


def make_rays(origins, directions, tmax=1e34, inside=0):
    """ctypes array of abi.Ray from (n,3) arrays."""
    o = np.asarray(origins, np.float32).reshape(-1, 3)
    d = np.asarray(directions, np.float32).reshape(-1, 3)
    n = len(o)
    arr = (abi.Ray * n)()
    view = np.frombuffer(arr, dtype=np.dtype([("o", "<f4", 3), ("d", "<f4", 3), ("t", "<f4"), ("g", "<u4")]))
    view["o"] = o
    view["d"] = d
    view["t"] = np.broadcast_to(np.asarray(tmax, np.float32), (n,))
    view["g"] = np.broadcast_to(np.asarray(inside, np.uint32), (n,))
    return arr


def hits_to_numpy(hits, n):
    dt = np.dtype([("t", "<f4"), ("normal", "<f4", 3), ("vox_index", "<i4"), ("material", "<u4"), ("cells", "<u4"),
                   ("inside_glass", "<u4")])
    return np.frombuffer(hits, dtype=dt, count=n).copy()
