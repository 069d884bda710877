"""Hand-derived known answers for single reference functions (parity item 2c).

Each expected value here is derived independently of oracle/vpx_oracle.c, from the text of
the reference function cited (float32 arithmetic in the reference's operand order, numpy
scalars, no FMA unless the reference uses one), and compared bit for bit with the oracle's
restatement through its known-answer hooks (oracle_kat_*, oracle_accumulate_tonemap).
The GPU parity suite pins the device to the oracle, so these pin the device too.

  GetNormalVoxel        template/scene.cpp:121-148 (ties -> diagonal normals)
  PointLightEvaluate    renderer.cpp:102-131        SpotLightEvaluate  renderer.cpp:133-159
  AreaLightEvaluation   renderer.cpp:161-207        DirectionalLight   renderer.cpp:315-338
  SchlickReflectance    renderer.cpp:1588-1594      SchlickNonMetal    renderer.cpp:1611-1616
  Refract / Reflect     renderer.cpp:913-925        Absorption         renderer.cpp:1596-1608
  accumulate blend      renderer.cpp:1797-1828 (_mm256_fmadd_ps(1-w, acc, px*w))
  ApplyReinhardJodie    renderer.cpp:2222-2240      RGBF32_to_RGB8     template/precomp.h:372-388
"""
import ctypes as C
from fractions import Fraction

import numpy as np
import pytest

f = np.float32
P = C.POINTER


def vec(*a):
    return np.array(a, np.float32)


def dot(a, b):  # tmpl8math.h:2259-2262: a.x*b.x + a.y*b.y + a.z*b.z, left to right
    return f(f(f(a[0] * b[0]) + f(a[1] * b[1])) + f(a[2] * b[2]))


def length(v):  # tmpl8math.h:2319-2322
    return np.sqrt(dot(v, v))


def normalize(v):  # tmpl8math.h:2350-2354 with rsqrtf = 1.0f / sqrtf(x) (:411-414)
    return v * (f(1.0) / np.sqrt(dot(v, v)))


def std_min(a, b):  # std::min: (b < a) ? b : a
    return b if b < a else a


def xform_vec(v, m):  # TransformVector (tmpl8math.cpp:349-353), row-major, left to right
    return vec(f(f(m[0] * v[0]) + f(m[1] * v[1])) + f(m[2] * v[2]),
               f(f(m[4] * v[0]) + f(m[5] * v[1])) + f(m[6] * v[2]),
               f(f(m[8] * v[0]) + f(m[9] * v[1])) + f(m[10] * v[2]))


def dsign(d):  # Ray::ComputeDsign (scene.cpp:49-57): sign bit, -0 -> 1
    return vec(*[f(np.signbit(x)) for x in d])


# ------------------------------------------------------------------ RNG (tmpl8math.cpp)
class Rng:
    def __init__(self, s):
        self.s = int(s) & 0xFFFFFFFF

    def u(self):  # RandomUInt, xorshift32 (13, 17, 5), tmpl8math.cpp:119-125
        s = self.s
        s ^= (s << 13) & 0xFFFFFFFF
        s ^= s >> 17
        s ^= (s << 5) & 0xFFFFFFFF
        self.s = s
        return s

    def rf(self):  # RandomFloat = RandomUInt() * 2.3283064365387e-10f (:130-133)
        return f(f(self.u()) * f(2.3283064365387e-10))

    def random_direction(self):  # RandomDirection (tmpl8math.cpp:76-93): +octant, rejection
        while True:
            p = vec(self.rf(), self.rf(), self.rf())
            if dot(p, p) < f(1):
                return normalize(p)


# ------------------------------------------------------------------------ fixtures
@pytest.fixture(scope="module")
def lib(orc, abi):
    lib = orc._lib(abi)
    F3 = P(C.c_float)
    lib.oracle_kat_normal.argtypes = [F3, F3, C.c_float, C.c_uint32, F3, F3]
    lib.oracle_kat_light.argtypes = [C.c_void_p, C.c_int, C.c_uint32, F3, F3, C.c_float, F3, C.c_uint32, C.c_int32,
                                     P(C.c_uint32), F3]
    lib.oracle_kat_shading.argtypes = [C.c_int, F3, F3]
    return lib


def fp(a):
    a = np.ascontiguousarray(a, np.float32)
    return a, a.ctypes.data_as(P(C.c_float))


def bits(x):
    return np.asarray(x, np.float32).view(np.uint32)


IDENTITY = np.eye(4, dtype=np.float32).reshape(-1)


def oracle_normal(lib, o, d, t, n, m=IDENTITY):
    out = np.zeros(3, np.float32)
    _, po = fp(o)
    _, pd = fp(d)
    _, pm = fp(m)
    assert lib.oracle_kat_normal(po, pd, f(t), n, pm, out.ctypes.data_as(P(C.c_float))) == 0
    return out


def ref_normal(o, d, t, n, m=IDENTITY):
    """GetNormalVoxel (scene.cpp:121-148) on the ray (o, normalize(d)) at t."""
    dn = normalize(np.asarray(d, np.float32))
    ip = np.asarray(o, np.float32) + f(t) * dn  # IntersectionPoint: O + t * D (scene.h:80-83)
    i1 = ip * f(n)
    fg = i1 - np.floor(i1)  # fracf: v - floorf(v)
    dd = vec(*[std_min(fg[k], f(1) - fg[k]) for k in range(3)])
    mind = std_min(std_min(dd[0], dd[1]), dd[2])
    sign = dsign(dn) * f(2) - f(1)
    nn = vec(*[sign[k] if mind == dd[k] else f(0) for k in range(3)])
    return normalize(xform_vec(nn, m))


# --------------------------------------------------------------- GetNormalVoxel
def test_normal_voxel_ties_are_diagonal(lib):
    """Hand-worked: a +x ray entering the face x = 5/8 of an 8^3 grid.  Off the edges the
    normal is (-1, 0, 0); on an edge (frac(y) = 0) both axes tie at d = 0 and the normal is
    (-1, sign_y, 0) / sqrt(2) with sign_y = 2*Dsign.y - 1 (+0 -> -1, -0 -> +1); on a corner
    all three tie: (-1, -1, -1) / sqrt(3)."""
    inv2, inv3 = f(1) / np.sqrt(f(2)), f(1) / np.sqrt(f(3))
    cases = [
        ((0.0, 0.40, 0.5625), (1.0, 0.0, 0.0), vec(-1, 0, 0)),
        ((0.0, 0.375, 0.5625), (1.0, 0.0, 0.0), vec(-1, -1, 0) * inv2),
        ((0.0, 0.375, 0.5625), (1.0, -0.0, 0.0), vec(-1, 1, 0) * inv2),
        ((0.0, 0.375, 0.5), (1.0, 0.0, 0.0), vec(-1, -1, -1) * inv3),
        ((0.0, 0.375, 0.5), (1.0, -0.0, -0.0), vec(-1, 1, 1) * inv3),
    ]
    for o, d, want in cases:
        got = oracle_normal(lib, vec(*o), vec(*d), 0.625, 8)
        assert np.array_equal(bits(got), bits(want)), (o, d, got, want)
        assert np.array_equal(bits(got), bits(ref_normal(o, d, 0.625, 8)))


def test_normal_voxel_scaled_transform_and_random_hits(lib):
    """The object-space normal goes through TransformVector(matrix) and normalize; the
    diagonal case with a non-uniform scale, then random hits against the restated formula."""
    m = np.diag(np.float32([2.0, 1.0, 0.5, 1.0])).reshape(-1)
    got = oracle_normal(lib, vec(0.0, 0.375, 0.5625), vec(1.0, 0.0, 0.0), 0.625, 8, m)
    want = vec(-2, -1, 0) * (f(1) / np.sqrt(f(5)))
    assert np.array_equal(bits(got), bits(want))
    rng = np.random.default_rng(3)
    for _ in range(400):
        o = rng.uniform(-0.2, 1.2, 3).astype(np.float32)
        d = rng.normal(0, 1, 3).astype(np.float32)
        if rng.random() < 0.3:
            d[rng.integers(0, 3)] = 0.0
        t = f(rng.uniform(0.0, 1.5))
        n = int(rng.choice([8, 64, 128]))
        mm = np.eye(4, dtype=np.float32)
        mm[:3, :3] = rng.uniform(-1, 1, (3, 3))
        got = oracle_normal(lib, o, d, t, n, mm.reshape(-1))
        want = ref_normal(o, d, t, n, mm.reshape(-1))
        assert np.array_equal(bits(got), bits(want)), (o, d, t, n)


# -------------------------------------------------------------------- lights
def light_scene(pkg, blocker=False):
    sc, abi = pkg.scene, pkg.abi
    n = 16
    g = np.full(n ** 3, abi.MAT_NONE, np.uint8)
    if blocker:  # a wall of voxels at z cell 12 between the hit and lights above +z
        g.reshape(n, n, n)[12, :, :] = 20
    mats = sc.default_materials()
    mats[20].albedo[0], mats[20].albedo[1], mats[20].albedo[2] = 0.8, 0.6, 0.25
    pts = [sc.point_light((0.3, 0.6, 1.4), (1.0, 0.9, 0.7))]
    sps = [sc.spot_light((0.5, 0.5, 1.6), (0.0, 0.0, -1.0), (1.5, 1.2, 1.0), angle=0.8)]
    ars = [sc.area_light((0.6, 0.5, 1.7), (1.0, 0.95, 0.9), 1.2, 0.3)]
    dl = sc.dir_light((0.2, -0.3, -1.0), (0.9, 0.8, 0.7))
    return sc._scene("kat", [sc.GridSpec(n=n, dense=g)], [sc.volume()], mats, pts, sps, ars, dl,
                     (0.5, 0.5, -1.0), (0.5, 0.5, 0.5), 8, 8)


HIT_O = vec(0.41, 0.37, 0.05)
HIT_D = vec(0.02, -0.01, 1.0)
HIT_T = f(0.2)
HIT_N = vec(0.0, 0.0, 1.0)


def oracle_light(lib, orc, abi, desc, kind, seed=0x1234567, samples=3, n=HIT_N):
    o = orc.Oracle(abi, desc)
    out = np.zeros(3, np.float32)
    s = C.c_uint32(seed)
    _, po = fp(HIT_O)
    _, pd = fp(HIT_D)
    nn, pn = fp(n)
    assert lib.oracle_kat_light(o.ptr, kind, 0, po, pd, HIT_T, pn, 20, samples, C.byref(s),
                                out.ctypes.data_as(P(C.c_float))) == 0
    return out, s.value


def hit_point():
    return HIT_O + HIT_T * normalize(HIT_D)  # Ray ctor normalises D; O + t * D


def albedo():
    return vec(0.8, 0.6, 0.25)


def test_point_light_known_answer(pkg, orc, abi, lib):
    """PointLightEvaluate: max(0, cos) * color * (1 / (dst * dst)) * albedo, dir * (1 / dst)."""
    ip = hit_point()
    d = vec(0.3, 0.6, 1.4) - ip
    dst = length(d)
    dn = d * (f(1) / dst)
    c = dot(dn, HIT_N)
    li = (max(f(0), c) * vec(1.0, 0.9, 0.7)) * (f(1) / (dst * dst))
    want = li * albedo()
    got, s = oracle_light(lib, orc, abi, light_scene(pkg), 0)
    assert np.array_equal(bits(got), bits(want)) and s == 0x1234567  # no RNG draw
    got, _ = oracle_light(lib, orc, abi, light_scene(pkg, blocker=True), 0)
    assert not got.any()  # occluded -> 0
    got, _ = oracle_light(lib, orc, abi, light_scene(pkg), 0, n=vec(0, 0, -1))
    assert not got.any()  # cos <= 0 -> 0


def test_spot_light_known_answer(pkg, orc, abi, lib):
    """SpotLightEvaluate: dir / dst (division), cone cos against the spot direction (no N.L),
    alpha = 1 - (1 - cos) * 1 / (1 - angle), max(0, cos) * color / (dst * dst) * k * alpha."""
    ip = hit_point()
    d = vec(0.5, 0.5, 1.6) - ip
    dst = length(d)
    dn = d / dst
    c = dot(dn, vec(0.0, 0.0, -1.0))
    assert c <= f(0.8)  # this spot points away from the hit: outside the cone
    got, _ = oracle_light(lib, orc, abi, light_scene(pkg), 1)
    assert not got.any()
    desc = light_scene(pkg)
    desc.spots[0] = pkg.scene.spot_light((0.5, 0.5, 1.6), (0.0, 0.0, 1.0), (1.5, 1.2, 1.0), angle=0.8)
    c = dot(dn, vec(0.0, 0.0, 1.0))
    alpha = f(1) - f(f(f(1) - c) * f(1)) / f(f(1) - f(0.8))
    li = (max(f(0), c) * vec(1.5, 1.2, 1.0)) / (dst * dst)
    want = (li * albedo()) * alpha
    got, _ = oracle_light(lib, orc, abi, desc, 1)
    assert np.array_equal(bits(got), bits(want))


@pytest.mark.parametrize("samples", [1, 3, 5])
def test_area_light_known_answer(pkg, orc, abi, lib, samples):
    """AreaLightEvaluation: `samples` RandomDirection points on the light's +octant, each
    cos * color * mult * (r * r) * PI * 4 / (dst * dst) (PI4 expands textually), averaged,
    times albedo; the RNG advances through every sample's rejection loop."""
    ip = hit_point()
    rng = Rng(0x2468ACE)
    inc = vec(0, 0, 0)
    for _ in range(samples):
        rp = rng.random_direction()
        rp = rp * f(0.3)
        rp = rp + vec(0.6, 0.5, 1.7)
        d = rp - ip
        dst = length(d)
        dn = d * (f(1) / dst)
        c = dot(dn, HIT_N)
        if c <= f(0):
            continue
        li = ((((c * vec(1.0, 0.95, 0.9)) * f(1.2)) * f(f(0.3) * f(0.3))) * f(3.14159265358979323846264)) * f(4.0)
        li = li / (dst * dst)
        inc = inc + li
    inc = inc / f(samples)
    want = inc * albedo()
    got, s = oracle_light(lib, orc, abi, light_scene(pkg), 2, seed=0x2468ACE, samples=samples)
    assert np.array_equal(bits(got), bits(want))
    assert s == rng.s


def test_directional_light_known_answer(pkg, orc, abi, lib):
    """DirectionalLightEvaluate: dir = -direction (not normalised), max(0, dot) * color * k."""
    dirv = -vec(0.2, -0.3, -1.0)
    c = dot(dirv, HIT_N)
    want = (max(f(0), c) * vec(0.9, 0.8, 0.7)) * albedo()
    got, _ = oracle_light(lib, orc, abi, light_scene(pkg), 3)
    assert np.array_equal(bits(got), bits(want))
    got, _ = oracle_light(lib, orc, abi, light_scene(pkg, blocker=True), 3)
    assert not got.any()


# ------------------------------------------------------------------- shading
def shading(lib, fn, inp, nout):
    a, pa = fp(inp)
    out = np.zeros(nout, np.float32)
    assert lib.oracle_kat_shading(fn, pa, out.ctypes.data_as(P(C.c_float))) == 0
    return out


def pow5(x):  # powf(x, 5) as the build decides it: the correctly rounded float
    return f(np.float64(x) ** 5)


def test_schlick_known_answers(lib):
    rng = np.random.default_rng(11)
    for _ in range(300):
        c = f(rng.uniform(-1, 1))
        ior = f(rng.choice([1.45, 1.0 / 1.45, 1.0, 2.4]))
        r0 = f(f(1) - ior) / f(f(1) + ior)  # SchlickReflectance (renderer.cpp:1588-1594)
        r0 = r0 * r0
        want = r0 + (f(1) - r0) * pow5(f(1) - c)
        assert bits(shading(lib, 0, [c, ior], 1)[0]) == bits(want)
        want = f(0.04) + (f(1) - f(0.04)) * pow5(f(1) - c)  # SchlickReflectanceNonMetal (:1611-1616)
        assert bits(shading(lib, 1, [c], 1)[0]) == bits(want)


def test_refract_reflect_known_answers(lib):
    rng = np.random.default_rng(12)
    for _ in range(300):
        d = normalize(rng.normal(0, 1, 3).astype(np.float32))
        n = normalize(rng.normal(0, 1, 3).astype(np.float32))
        ratio = f(rng.choice([1.45, 1.0 / 1.45, 1.0]))
        c = std_min(dot(-d, n), f(1))  # Refract (renderer.cpp:919-925)
        rper = ratio * (d + c * n)
        rpar = -np.sqrt(np.abs(f(1) - dot(rper, rper))) * n
        want = rper + rpar
        got = shading(lib, 2, np.concatenate([d, n, [ratio]]), 3)
        assert np.array_equal(bits(got), bits(want))
        want = d - (f(2) * n) * dot(n, d)  # Reflect (:913-916): direction - 2 * normal * dot
        got = shading(lib, 4, np.concatenate([d, n]), 3)
        assert np.array_equal(bits(got), bits(want))


def test_absorption_known_answers(lib):
    """Absorption: expf(-distanceTraveled * intensity * (1 - color)) per channel, the
    scalar product first (left to right), expf as the correctly rounded float."""
    rng = np.random.default_rng(13)
    for _ in range(300):
        col = rng.uniform(0, 1, 3).astype(np.float32)
        inten, dist = f(rng.uniform(0, 22)), f(rng.uniform(0, 2))
        e = f(-dist * inten) * (f(1) - col)
        want = np.array([f(np.exp(np.float64(x))) for x in e], np.float32)
        got = shading(lib, 3, np.concatenate([col, [inten, dist]]), 3)
        assert np.array_equal(bits(got), bits(want))


# ------------------------------------------------------------ accumulate + tonemap
def f32_round(q):
    """Round an exact rational to the nearest float32 (ties to even)."""
    x = f(float(q))
    cands = [np.nextafter(x, f(-np.inf)), x, np.nextafter(x, f(np.inf))]
    best = min(cands, key=lambda c: (abs(Fraction(float(c)) - q), int(np.float32(c).view(np.uint32)) & 1))
    return f(best)


def fmaf(a, b, c):  # _mm256_fmadd_ps: a * b + c with one rounding
    return f32_round(Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c)))


def ref_tonemap(c):
    lum = dot(c, vec(0.2126, 0.7152, 0.0722))  # GetLuminance
    rh = c / (f(1) + c)                         # color / (1.0f + color)
    la = c / (f(1) + lum)                       # color / (1.0f + luminance)
    o = la + rh * (rh - la)                     # lerp(la, rh, rh) = a + t * (b - a)
    ch = [int(np.uint32(f(255) * std_min(f(1), o[k]))) for k in range(3)]  # (uint)(255 * min(1, v))
    return (ch[0] << 16) + (ch[1] << 8) + ch[2]


def test_accumulate_tonemap_known_answers(orc, abi):
    lib = orc._lib(abi)
    rng = np.random.default_rng(14)
    for frame in (0, 1, 2, 7, 15):
        for _ in range(200):
            px = (rng.uniform(0, 3, 4) * (rng.random(4) < 0.9)).astype(np.float32)
            px[3] = 0
            acc = rng.uniform(0, 2, 4).astype(np.float32)
            acc[3] = 0
            w = f(1) / (f(frame) + f(1))
            iw = f(1) - w
            want_acc = np.array([fmaf(iw, acc[k], f(px[k] * w)) for k in range(4)], np.float32)
            want_rgb = ref_tonemap(want_acc[:3])
            a = acc.copy()
            rgb = np.zeros(1, np.uint32)
            lib.oracle_accumulate_tonemap(px.ctypes.data, frame, a.ctypes.data, rgb.ctypes.data)
            assert np.array_equal(bits(a), bits(want_acc)), (frame, px, acc)
            assert int(rgb[0]) == want_rgb, (frame, px, acc)
