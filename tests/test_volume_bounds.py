"""The world boxes the device culls volume walks with (vpx_volume_bounds, host-side, no GPU).

FindNearest and IsOccluded skip a volume whose inflated world box the ray's segment [0, t]
misses (misses_volume): the reference's Setup3DDDA then fails or enters the cube beyond ray.t,
so no cell is read (renderer.cpp:209-243, 946-1018; scene.cpp:719-749, 761, 1015).  The box
holds the cube b0..b1 under the inverse of the affine part of inv_matrix, the only part
TransformPosition(_SSEM) reads (tmpl8math.cpp:345-402).  Round 6: SetTransform's inverse leaves
inv_matrix[15] = 1 +- 1 ulp on 20 of C4's 64 rotated instances; the bounds (then spheres) used
to demand an exact (0, 0, 0, 1) bottom row and left those instances unbounded, so every ray set
up their walks (C4 42.4 -> 33.5 ms per step once fixed).  The spheres became boxes tested
against the segment, not the line: the zone scene's long thin volumes passed ~7 spheres per
ray for ~2 cubes entered.
"""
import ctypes as C

import numpy as np
import pytest


def bounds(pkg, vol):
    out = (C.c_float * 6)()
    assert pkg.abi.load_library().vpx_volume_bounds(C.byref(vol), out) == pkg.abi.VPX_OK
    return np.array(list(out), np.float64)


def cube_corners_world(vol):
    """The cube's corners through the affine inverse of inv_matrix (rows 0-2), in double."""
    im = np.array(list(vol.inv_matrix), np.float64).reshape(4, 4)
    a, t = im[:3, :3], im[:3, 3]
    b0, b1 = np.array(list(vol.b0)), np.array(list(vol.b1))
    q = np.array([[b1[0] if k & 1 else b0[0], b1[1] if k & 2 else b0[1], b1[2] if k & 4 else b0[2]]
                  for k in range(8)])
    return np.linalg.solve(a, (q - t).T).T


@pytest.mark.parametrize("scene", ["C4", "zone"])
def test_every_volume_gets_a_finite_enclosing_sphere(pkg, scene):
    sc = pkg.scene
    desc = sc.instanced_scene(n=128, inst_n=64, width=64, height=64) if scene == "C4" else sc.zone_scene(64, 48, 1)
    rows = [list(v.inv_matrix)[12:] for v in desc.volumes]
    if scene == "C4":  # the case that used to fall back to +inf: a bottom row 1 ulp off
        assert any(r != [0.0, 0.0, 0.0, 1.0] for r in rows)
    for i, vol in enumerate(desc.volumes):
        b = bounds(pkg, vol)
        assert np.isfinite(b).all(), (i, b, rows[i])
        c = cube_corners_world(vol)
        lo, hi = b[:3], b[3:]
        assert (c > lo).all() and (c < hi).all(), (i, c.min(0), c.max(0), lo, hi)  # padded: strictly inside
        half = np.linalg.norm(c.max(0) - c.min(0)) / 2
        slack = 1.5e-3 * half + 1.5e-3 * (1 + np.abs((lo + hi) / 2).sum() + half) + 1e-6
        assert (c.min(0) - lo < slack).all() and (hi - c.max(0) < slack).all(), i  # and not loose


def test_singular_volume_is_never_culled(pkg):
    vol = pkg.scene.volume((0.0, 0.0, 0.0), (1.0, 1.0, 1.0))
    for k in range(16):
        vol.inv_matrix[k] = 0.0
    b = bounds(pkg, vol)
    assert (b[:3] == -np.inf).all() and (b[3:] == np.inf).all()
    assert pkg.abi.load_library().vpx_volume_bounds(None, (C.c_float * 6)()) == pkg.abi.VPX_E_INVALID
