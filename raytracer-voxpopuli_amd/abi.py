"""ctypes mirror of include/vpx.h and the loader for libvpx_hip.so.

The library is the product: there is no fallback.  `load_library()` raises when the
shared object is missing or does not export the ABI version this module expects.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libvpx_hip.so")
ABI_VERSION = 2  # 2: vpx_profile 160 B (stage_busy_ms), packed tiles in 8x8 quadrants

VPX_OK = 0
VPX_E_INVALID, VPX_E_DEVICE, VPX_E_NOMEM, VPX_E_STATE = -1, -2, -3, -4  # include/vpx.h status codes
VPX_FLAG_AA = 0x1
VPX_FLAG_DOF = 0x2
VPX_FLAG_NO_TONEMAP = 0x4
VPX_ARITH_EXACT, VPX_ARITH_X86_HOST = 0, 1  # vpx_set_arithmetic modes
VPX_FLAG_SKY = 0x8  # activateSky: misses sample the vpx_set_sky texture (renderer.cpp:2308-2326)
MAT_NONE = 255
SKY_DEFAULT = (0.392, 0.584, 0.829)  # SampleSky with activateSky == false, renderer.cpp:2310-2313

f3 = C.c_float * 3


class Volume(C.Structure):
    _fields_ = [("grid_id", C.c_uint32), ("reserved", C.c_uint32), ("matrix", C.c_float * 16),
                ("inv_matrix", C.c_float * 16), ("b0", f3), ("b1", f3)]


class Material(C.Structure):
    _fields_ = [("albedo", f3), ("roughness", C.c_float), ("emissive", C.c_float), ("ior", C.c_float),
                ("pad", C.c_float * 2)]


class PointLight(C.Structure):
    _fields_ = [("position", f3), ("color", f3)]


class SpotLight(C.Structure):
    _fields_ = [("position", f3), ("direction", f3), ("color", f3), ("angle", C.c_float)]


class AreaLight(C.Structure):
    _fields_ = [("position", f3), ("color", f3), ("color_multiplier", C.c_float), ("radius", C.c_float)]


class DirLight(C.Structure):
    _fields_ = [("direction", f3), ("color", f3)]


class Sphere(C.Structure):
    _fields_ = [("center", f3), ("radius", C.c_float), ("material", C.c_uint32), ("pad", C.c_uint32 * 3)]


class Triangle(C.Structure):
    _fields_ = [("position", f3), ("v0", f3), ("v1", f3), ("v2", f3), ("material", C.c_uint32),
                ("pad", C.c_uint32 * 3)]


class Camera(C.Structure):
    _fields_ = [("cam_pos", f3), ("top_left", f3), ("top_right", f3), ("bottom_left", f3), ("right", f3),
                ("up", f3), ("focal_distance", C.c_float), ("defocus_jitter", C.c_float)]


class FrameParams(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("max_bounces", C.c_int32),
                ("frame_index", C.c_uint32), ("seed_base", C.c_uint32), ("flags", C.c_uint32),
                ("aa_strength", C.c_float), ("area_samples", C.c_int32), ("sky", f3), ("reserved", C.c_uint32)]


class Ray(C.Structure):
    _fields_ = [("origin", f3), ("direction", f3), ("tmax", C.c_float), ("inside_glass", C.c_uint32)]


class Hit(C.Structure):
    _fields_ = [("t", C.c_float), ("normal", f3), ("vox_index", C.c_int32), ("material", C.c_uint32),
                ("cells", C.c_uint32), ("inside_glass", C.c_uint32)]


class Stats(C.Structure):
    _fields_ = [("primary_rays", C.c_uint64), ("shadow_rays", C.c_uint64), ("bounce_rays", C.c_uint64),
                ("dda_cells", C.c_uint64), ("kernel_ms", C.c_float), ("total_ms", C.c_float)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class PrevCamera(C.Structure):
    _fields_ = [("cam_pos", f3), ("left_normal", f3), ("right_normal", f3), ("top_normal", f3),
                ("bottom_normal", f3), ("pad", C.c_float)]


class Profile(C.Structure):
    _fields_ = [("stage_ms", C.c_float * 8), ("stage_launches", C.c_uint32 * 8), ("stage_cells", C.c_uint64 * 8),
                ("stage_busy_ms", C.c_float * 8)]


class BvhTri(C.Structure):  # vpx_bvh_tri: BasicBVH Tri (BasicBVH.h:3-7) without the centroid
    _fields_ = [("v0", C.c_float * 3), ("v1", C.c_float * 3), ("v2", C.c_float * 3)]


class BvhNode(C.Structure):  # vpx_bvh_node: BVHNode (BasicBVH.h:11-20)
    _fields_ = [("aabb_min", C.c_float * 3), ("aabb_max", C.c_float * 3), ("left_first", C.c_uint32),
                ("tri_count", C.c_uint32)]


BVH_MAX_TRIS = 512
BVH_MAX_DEPTH = 63

STAGES = ("primary", "shade", "shadow", "resolve", "bounce", "finish", "frame", "instances")

STRUCT_SIZES = {PrevCamera: 64, Profile: 160, Volume: 160, Material: 32, PointLight: 24, SpotLight: 40, AreaLight: 32, DirLight: 24,
                Sphere: 32, Triangle: 64, Camera: 80, FrameParams: 48, Ray: 32, Hit: 32, Stats: 40,
                BvhTri: 36, BvhNode: 32}


def np_dtype(struct):
    """numpy dtype with the exact layout of a ctypes Structure (for record arrays)."""
    return np.dtype(struct)


def as_ptr(arr, struct=None):
    if arr is None:
        return None
    if struct is not None:
        return arr.ctypes.data_as(C.POINTER(struct))
    return arr.ctypes.data_as(C.c_void_p)


# name -> (restype, argtypes); every symbol include/vpx.h declares
SIGNATURES = {
    "vpx_create": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "vpx_create_multi": (C.c_int, [C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_void_p)]),
    "vpx_destroy": (C.c_int, [C.c_void_p]),
    "vpx_last_error": (C.c_char_p, [C.c_void_p]),
    "vpx_abi_version": (C.c_int, []),
    "vpx_set_stream": (C.c_int, [C.c_void_p, C.c_void_p]),
    "vpx_synchronize": (C.c_int, [C.c_void_p]),
    "vpx_set_pipeline": (C.c_int, [C.c_void_p, C.c_uint32]),
    "vpx_gl_register_buffer": (C.c_int, [C.c_void_p, C.c_uint]),
    "vpx_gl_map": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]),
    "vpx_gl_unmap": (C.c_int, [C.c_void_p]),
    "vpx_upload_grid": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]),
    "vpx_generate_tiled_grid": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p] + [C.c_uint32] * 7),
    "vpx_grid_checksum": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint64)]),
    "vpx_set_volumes": (C.c_int, [C.c_void_p, C.POINTER(Volume), C.c_uint32]),
    "vpx_set_materials": (C.c_int, [C.c_void_p, C.POINTER(Material), C.c_uint32]),
    "vpx_set_lights": (C.c_int, [C.c_void_p, C.POINTER(PointLight), C.c_uint32, C.POINTER(SpotLight), C.c_uint32,
                                 C.POINTER(AreaLight), C.c_uint32, C.POINTER(DirLight)]),
    "vpx_set_shapes": (C.c_int, [C.c_void_p, C.POINTER(Sphere), C.c_uint32, C.POINTER(Triangle), C.c_uint32]),
    "vpx_set_camera": (C.c_int, [C.c_void_p, C.POINTER(Camera)]),
    "vpx_set_sky": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_float]),
    "vpx_render": (C.c_int, [C.c_void_p, C.POINTER(FrameParams), C.c_void_p, C.c_void_p, C.POINTER(Stats)]),
    "vpx_render_tiles": (C.c_int, [C.c_void_p, C.POINTER(FrameParams), C.c_uint32, C.c_uint32, C.c_uint32,
                                   C.c_uint32, C.c_void_p, C.POINTER(Stats)]),
    "vpx_render_tiles_accum": (C.c_int, [C.c_void_p, C.POINTER(FrameParams), C.c_uint32, C.c_uint32, C.c_uint32,
                                         C.c_uint32, C.c_void_p, C.c_void_p, C.POINTER(Stats)]),
    "vpx_composite_rgb8": (C.c_int, [C.c_void_p, C.POINTER(FrameParams), C.c_uint32, C.c_uint32, C.c_uint32,
                                     C.c_void_p, C.c_void_p]),
    "vpx_render_window": (C.c_int, [C.c_void_p, C.POINTER(FrameParams), C.c_uint32, C.c_void_p, C.c_void_p]),
    "vpx_render_tiles_accum_window": (C.c_int, [C.c_void_p, C.POINTER(FrameParams), C.c_uint32, C.c_uint32,
                                                C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p]),
    "vpx_tiles_packed_len": (C.c_uint64, [C.c_uint32] * 5),
    "vpx_composite_tiles": (C.c_int, [C.c_void_p, C.POINTER(FrameParams), C.c_uint32, C.c_uint32, C.c_uint32,
                                      C.c_void_p, C.c_void_p, C.c_void_p]),
    "vpx_get_counters": (C.c_int, [C.c_void_p, C.POINTER(Stats), C.c_int]),
    "vpx_grid_fill": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint8]),
    "vpx_grid_write_box": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p] + [C.c_uint32] * 6),
    "vpx_grid_emissive_sphere": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint8, C.c_float]),
    "vpx_render_reproject": (C.c_int, [C.c_void_p, C.POINTER(FrameParams), C.POINTER(PrevCamera), C.c_void_p,
                                       C.c_void_p, C.POINTER(Stats)]),
    "vpx_prev_camera_look_at": (C.c_int, [C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_uint32, C.c_uint32,
                                          C.POINTER(PrevCamera)]),
    "vpx_profile_enable": (C.c_int, [C.c_void_p, C.c_uint32]),
    "vpx_profile_select": (C.c_int, [C.c_void_p, C.c_uint32]),
    "vpx_profile_read": (C.c_int, [C.c_void_p, C.POINTER(Profile), C.c_int]),
    "vpx_profile_busy_union": (C.c_float, [C.POINTER(C.c_float), C.c_uint32]),
    "vpx_find_nearest": (C.c_int, [C.c_void_p, C.POINTER(Ray), C.c_uint32, C.POINTER(Hit)]),
    "vpx_is_occluded": (C.c_int, [C.c_void_p, C.POINTER(Ray), C.c_uint32, C.c_void_p]),
    "vpx_trace": (C.c_int, [C.c_void_p, C.POINTER(Ray), C.c_void_p, C.c_uint32, C.c_int32, C.POINTER(C.c_float),
                            C.c_int32, C.c_void_p]),
    "vpx_focus_distance": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_float)]),
    "vpx_camera_look_at": (C.c_int, [C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_uint32, C.c_uint32,
                                     C.POINTER(Camera)]),
    "vpx_volume_set_transform": (C.c_int, [C.POINTER(C.c_float)] * 3 + [C.POINTER(Volume)]),
    "vpx_volume_bounds": (C.c_int, [C.POINTER(Volume), C.POINTER(C.c_float)]),
    "vpx_default_materials": (C.c_int, [C.POINTER(Material)]),
    "vpx_pixel_seed": (C.c_uint32, [C.c_uint32] * 6),
    "vpx_bvh_set": (C.c_int, [C.c_void_p, C.POINTER(BvhTri), C.c_uint32]),
    "vpx_bvh_intersect": (C.c_int, [C.c_void_p, C.POINTER(Ray), C.c_uint32, C.POINTER(C.c_float)]),
    "vpx_bvh_build_host": (C.c_int, [C.POINTER(BvhTri), C.c_uint32, C.POINTER(BvhNode), C.POINTER(C.c_uint32),
                                     C.POINTER(C.c_uint32)]),
    "vpx_bvh_random_tris": (C.c_int, [C.POINTER(C.c_uint32), C.POINTER(BvhTri)]),
    "vpx_bvh_depth": (C.c_uint32, [C.POINTER(BvhNode), C.c_uint32]),
    "vpx_set_arithmetic": (C.c_int, [C.c_void_p, C.c_uint32]),
    "vpx_x86_arith_tables": (C.c_int, [C.c_void_p, C.c_uint64, C.POINTER(C.c_uint32)]),
    "vpx_x86_arith_verify": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64),
                                       C.POINTER(C.c_uint32)]),
    "vpx_vox_decode": (C.c_int, [C.c_void_p, C.c_uint64, C.POINTER(C.c_uint32), C.c_void_p, C.c_uint64, C.c_void_p]),
}

_LIB = None


class VpxError(RuntimeError):
    pass


def load_library(path=None):
    """Load libvpx_hip.so (in-tree) and bind every exported symbol.  Raises if absent."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = path or os.environ.get("VPX_LIB") or LIB_PATH
    if not os.path.exists(p):
        raise VpxError(f"{p} is missing: run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
    # One HIP runtime per process: torch's wheel bundles its own libamdhip64 (soname
    # libamdhip64.so.7, but needed by torch as libamdhip64.so).  Loaded first, the library would
    # bind /opt/rocm's copy and torch would then load a second runtime, after which the
    # library's first hipGetDeviceCount fails (measured on the box: vpx_create -> VPX_E_DEVICE).
    # With torch loaded first the library's DT_NEEDED resolves to torch's runtime by soname.
    try:
        import torch  # noqa: F401
    except ImportError:  # plain C-ABI use without torch: /opt/rocm's runtime only
        pass
    lib = C.CDLL(p)
    old_ok = os.environ.get("VPX_LIB_OLD") == "1"  # A/B runs against an earlier build (tools/gpu_ab.sh)
    for name, (res, args) in SIGNATURES.items():
        if old_ok and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)  # AttributeError = the library does not export the ABI
        fn.restype = res
        fn.argtypes = args
    if lib.vpx_abi_version() != ABI_VERSION:
        raise VpxError(f"ABI version mismatch: library {lib.vpx_abi_version()} != {ABI_VERSION}")
    if path is None:
        _LIB = lib
    return lib


def check(lib, ctx, rc, what):
    if rc != VPX_OK:
        msg = lib.vpx_last_error(ctx).decode() if ctx else ""
        raise VpxError(f"{what} failed ({rc}): {msg}")


def vec3(v):
    return f3(*[float(x) for x in v])


def sky_arg(sky):
    """vpx_trace's sky argument: a constant colour, or None = the uploaded sky texture."""
    return None if sky is None else vec3(sky)
