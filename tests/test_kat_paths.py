"""Hand-derived known answers for WHOLE paths and the DDA set-up.

The expected values come from a second restatement written here in numpy float32 straight
from the reference text — independent of oracle/vpx_oracle.c — and are compared bit for bit
with the oracle's entries (oracle_trace / oracle_find_nearest / oracle_is_occluded); the GPU
parity suite pins the device to those entries, and test_kat_paths_on_device (GPU) pins the
device to this restatement directly.  Every operation below is the reference's, in its
operand order, rounded to float32 after each step (the build's -ffp-contract=off reading of
/fp:fast); the two documented parity decisions are taken as decided: exact
1/x for FastReciprocal (renderer.cpp:929-934) and correctly rounded sin / cos / exp / pow5.

  Renderer::Trace              renderer.cpp:1076-1328  (every material branch, depth 1)
  Renderer::FindNearest        renderer.cpp:946-1018   (TransformPosition_SSEM pairwise sums,
                                                        tmpl8math.cpp:369-402)
  Renderer::IsOccluded         renderer.cpp:209-243    (TransformPosition, left-to-right sums)
  Scene::Setup3DDDA            template/scene.cpp:719-749 (general case: outside the cube,
                                                        negative directions, scaled/rotated volume)
  Scene::FindNearest / IsOccluded  template/scene.cpp:751-811, 1009-1047
  Scene::FindMaterialExit / FindSmokeExit  template/scene.cpp:875-1006
  PointLightEvaluate / DirectionalLightEvaluate / Illumination  renderer.cpp:102-131, 315-338, 738-764
"""
import ctypes as C
import math
from fractions import Fraction

import numpy as np
import pytest

pytestmark = pytest.mark.filterwarnings("ignore:divide by zero:RuntimeWarning")  # 1/0 = inf, as the reference

f32 = np.float32
BIG = f32(1e34)
PI = f32(3.14159265358979323846264)  # common.h:8
NONE = 255


# ------------------------------------------------------------------ float32 helpers
def v3(*a):
    return np.array(a, np.float32)


def add(a, b):
    return (a + b).astype(np.float32)


def sub(a, b):
    return (a - b).astype(np.float32)


def mul(a, b):  # float3 * float3 or float3 * float (commutative per lane in IEEE)
    return (np.asarray(a, np.float32) * np.asarray(b, np.float32)).astype(np.float32)


def dot(a, b):  # tmpl8math.h: a.x*b.x + a.y*b.y + a.z*b.z, left to right
    return f32(f32(f32(a[0] * b[0]) + f32(a[1] * b[1])) + f32(a[2] * b[2]))


def length(v):
    return f32(np.sqrt(dot(v, v)))


def normalize(v):  # v * rsqrtf(dot(v, v)), rsqrtf = 1.0f / sqrtf (tmpl8math.h:411-414, 2350-2354)
    return mul(v, f32(f32(1.0) / f32(np.sqrt(dot(v, v)))))


def std_min(a, b):
    return b if b < a else a


def std_max(a, b):
    return b if a < b else a


def trunc_i32(x):  # static_cast<int>(float) on x86 (cvttss2si): INT_MIN out of range / NaN
    x = float(x)
    if not (-2147483904.0 < x < 2147483648.0):
        return -2147483648
    return int(math.trunc(x))


def cr32(exact):
    """The float32 nearest to an exact rational (ties to even)."""
    fr = Fraction(exact)
    g = np.float32(float(fr))
    best = None
    for c in (np.nextafter(g, f32(-np.inf)), g, np.nextafter(g, f32(np.inf))):
        if not np.isfinite(c):
            continue
        d = abs(Fraction(float(c)) - fr)
        key = (d, int(np.asarray(c).view(np.uint32)) & 1)
        if best is None or key < best[0]:
            best = (key, c)
    return f32(best[1])


def cr32_f64(x):
    """float32 rounding of a double result that is within 1 ulp (double) of the true value;
    refuses arguments whose float32 rounding such an error could flip."""
    g = np.float32(x)
    lo, hi = np.nextafter(g, f32(-np.inf)), np.nextafter(g, f32(np.inf))
    for m in ((float(lo) + float(g)) / 2, (float(g) + float(hi)) / 2):
        assert abs(m - x) > 4 * abs(x) * 2.0 ** -52, "double-rounding midpoint: choose another case"
    return g


def sinf(x):
    return cr32_f64(math.sin(float(x)))


def cosf(x):
    return cr32_f64(math.cos(float(x)))


def expf(x):
    return cr32_f64(math.exp(float(x)))


def pow5(x):
    return cr32(Fraction(float(x)) ** 5)


def fbits(x):
    return np.asarray(x, np.float32).view(np.uint32)


# ------------------------------------------------------------------------ RNG
class Rng:  # xorshift32 (13, 17, 5) and RandomFloat (tmpl8math.cpp:119-133)
    def __init__(self, s):
        self.s = int(s) & 0xFFFFFFFF

    def rf(self):
        s = self.s
        s ^= (s << 13) & 0xFFFFFFFF
        s ^= s >> 17
        s ^= (s << 5) & 0xFFFFFFFF
        self.s = s
        return f32(f32(s) * f32(2.3283064365387e-10))

    def sphere_sample(self):  # RandomSphereSample (tmpl8math.h:2502-2511)
        theta = f32(f32(self.rf() * f32(2)) * PI)
        phi = f32(self.rf() * PI)
        r = self.rf()
        x = f32(f32(r * sinf(phi)) * cosf(theta))
        y = f32(f32(r * sinf(phi)) * sinf(theta))
        z = f32(r * cosf(phi))
        return v3(x, y, z)

    def diffuse_reflection(self, n):  # DiffuseReflection (tmpl8math.h:2518-2528), arguments left to right
        while True:
            a = f32(f32(self.rf() * f32(2)) - f32(1))
            b = f32(f32(self.rf() * f32(2)) - f32(1))
            c = f32(f32(self.rf() * f32(2)) - f32(1))
            r = v3(a, b, c)
            if not (dot(r, r) > f32(1)):
                break
        if dot(r, n) < f32(0):
            r = mul(r, f32(-1.0))
        return normalize(r)

    def random_direction(self):  # RandomDirection (tmpl8math.cpp:76-93)
        while True:
            p = v3(self.rf(), self.rf(), self.rf())
            if dot(p, p) < f32(1):
                return normalize(p)


# ------------------------------------------------------------------------ rays
class Ray:  # Ray(origin, direction) (scene.cpp:83-93): D normalised, t = 1e34
    def __init__(self, o, d, t=BIG, inside=False):
        self.O = np.asarray(o, np.float32).copy()
        self.D = normalize(np.asarray(d, np.float32))
        self.t = f32(t)
        self.N = v3(0, 0, 0)
        self.mat = NONE
        self.inside = inside

    def point(self):  # IntersectionPoint: O + t * D
        return add(self.O, mul(self.D, self.t))


def dsign(d):  # ComputeDsign: the sign bit as 0 / 1
    return v3(*[f32(1.0) if np.signbit(x) else f32(0.0) for x in d])


def xform_pos_sse(a, m):  # TransformPosition_SSEM: (x*m0 + y*m1) + (z*m2 + 1*m3) per row
    return v3(*[f32(f32(f32(a[0] * m[4 * j]) + f32(a[1] * m[4 * j + 1])) + f32(f32(a[2] * m[4 * j + 2]) + m[4 * j + 3]))
                for j in range(3)])


def xform_vec_sse(a, m):  # TransformVector_SSEM: (x*m0 + y*m1) + z*m2
    return v3(*[f32(f32(f32(a[0] * m[4 * j]) + f32(a[1] * m[4 * j + 1])) + f32(a[2] * m[4 * j + 2])) for j in range(3)])


def xform_pos(a, m):  # TransformPosition: m0*x + m1*y + m2*z + m3*1, left to right
    return v3(*[f32(f32(f32(f32(m[4 * j] * a[0]) + f32(m[4 * j + 1] * a[1])) + f32(m[4 * j + 2] * a[2]))
                    + f32(m[4 * j + 3] * f32(1))) for j in range(3)])


def xform_vec(a, m):  # TransformVector: ... + m3*0
    return v3(*[f32(f32(f32(f32(m[4 * j] * a[0]) + f32(m[4 * j + 1] * a[1])) + f32(m[4 * j + 2] * a[2]))
                    + f32(m[4 * j + 3] * f32(0))) for j in range(3)])


def offset_ray(p, n):  # OffsetRay (tmpl8math.cpp:473-487): int_scale 256, float_scale 1/65536, origin 1/32
    out = []
    for k in range(3):
        o = trunc_i32(f32(f32(256.0) * n[k]))
        pb = int(np.asarray(p[k], np.float32).view(np.int32))
        pi = np.array([(pb + (-o if p[k] < 0 else o)) & 0xFFFFFFFF], np.uint32).view(np.float32)[0]
        out.append(f32(p[k] + f32(f32(1.0 / 65536.0) * n[k])) if abs(p[k]) < f32(1.0 / 32.0) else pi)
    return v3(*out)


def reflect(d, n):  # Reflect: direction - 2 * normal * dot(normal, direction)
    return sub(d, mul(mul(n, f32(2)), dot(n, d)))


def refract(d, n, ratio):  # Refract (renderer.cpp:917-925)
    c = std_min(dot(-d, n), f32(1.0))
    rper = mul(add(d, mul(n, c)), ratio)
    rpar = mul(n, -f32(np.sqrt(abs(f32(f32(1.0) - dot(rper, rper))))))
    return add(rper, rpar)


def schlick(cosine, ior):  # SchlickReflectance (renderer.cpp:1588-1594)
    r0 = f32(f32(f32(1) - ior) / f32(f32(1) + ior))
    r0 = f32(r0 * r0)
    return f32(r0 + f32(f32(f32(1) - r0) * pow5(f32(f32(1) - cosine))))


def schlick_nonmetal(cosine):  # SchlickReflectanceNonMetal (renderer.cpp:1611-1616)
    r0 = f32(0.04)
    return f32(r0 + f32(f32(f32(1) - r0) * pow5(f32(f32(1) - cosine))))


# ------------------------------------------------------------------------ scene
class Vol:
    """A Scene: u8 grid (x + y*N + z*N^2), cube b0 / b1, matrix / invMatrix (used as given)."""

    def __init__(self, cells, n, matrix=None, inv=None, b0=(0, 0, 0), b1=(1, 1, 1)):
        self.cells, self.n = cells, n
        self.matrix = np.asarray(np.eye(4).reshape(-1) if matrix is None else matrix, np.float32)
        self.inv = np.asarray(np.eye(4).reshape(-1) if inv is None else inv, np.float32)
        self.b0, self.b1 = v3(*b0), v3(*b1)

    def cell(self, x, y, z):
        return int(self.cells[x + y * self.n + z * self.n * self.n])

    def contains(self, p):  # Cube::Contains (scene.cpp:205-210)
        return all(p[k] >= self.b0[k] for k in range(3)) and all(p[k] <= self.b1[k] for k in range(3))

    def intersect(self, O, rD, D):  # Cube::Intersect (scene.cpp:166-202)
        b = (self.b0, self.b1)
        sx, sy, sz = int(D[0] < 0), int(D[1] < 0), int(D[2] < 0)
        tmin_x = f32(f32(b[sx][0] - O[0]) * rD[0])
        tmax_x = f32(f32(b[1 - sx][0] - O[0]) * rD[0])
        tmin_y = f32(f32(b[sy][1] - O[1]) * rD[1])
        tmax_y = f32(f32(b[1 - sy][1] - O[1]) * rD[1])
        if tmin_x > tmax_y or tmin_y > tmax_x:
            return BIG
        tmin_x = std_max(tmin_x, tmin_y)
        tmax_x = std_min(tmax_x, tmax_y)
        tmin_z = f32(f32(b[sz][2] - O[2]) * rD[2])
        tmax_z = f32(f32(b[1 - sz][2] - O[2]) * rD[2])
        if tmin_x > tmax_z or tmin_z > tmax_x:
            return BIG
        tmin_x = std_max(tmin_x, tmin_z)
        return tmin_x if tmin_x > 0 else BIG

    def setup(self, O, D, rD, ds):  # Scene::Setup3DDDA (scene.cpp:719-749); None = ray misses
        t = f32(0)
        if not self.contains(O):
            t = self.intersect(O, rD, D)
            if t > f32(1e33):
                return None
        vmax = sub(self.b1, self.b0)
        g = f32(self.n)
        cell = f32(f32(1.0) / g)
        step = [trunc_i32(f32(f32(1) - f32(ds[k] * f32(2)))) for k in range(3)]
        pos = (mul(add(sub(O, self.b0), mul(D, f32(t + f32(0.00005)))), g) / vmax).astype(np.float32)
        planes = mul(sub(np.ceil(pos).astype(np.float32), ds), cell)
        P = [min(max(trunc_i32(pos[k]), 0), self.n - 1) for k in range(3)]
        tdelta = mul(v3(*[f32(cell * f32(step[k])) for k in range(3)]), rD)
        tmax = mul(sub(mul(planes, vmax), sub(O, self.b0)), rD)
        return dict(t=t, X=P[0], Y=P[1], Z=P[2], step=step, tdelta=tdelta, tmax=tmax)

    @staticmethod
    def advance(s, n, occlusion=False):
        """One step, the axis chosen as scene.cpp:773-802 (strict compares); False = left the grid.
        IsOccluded (scene.cpp:1026-1045) bounds-checks before taking t; the others after."""
        tm = s["tmax"]
        if tm[0] < tm[1]:
            k = 0 if tm[0] < tm[2] else 2
        else:
            k = 1 if tm[1] < tm[2] else 2
        key = "XYZ"[k]
        s[key] = (s[key] + s["step"][k]) & 0xFFFFFFFF  # uint coordinates: -1 wraps
        if s[key] >= n:
            if not occlusion:
                s["t"] = tm[k]
            return False
        s["t"] = tm[k]
        tm[k] = f32(tm[k] + s["tdelta"][k])
        return True

    def normal(self, O, D, t):  # GetNormalVoxel (scene.cpp:121-148), object-space ray
        i1 = mul(add(O, mul(D, t)), f32(self.n))
        fg = sub(i1, np.floor(i1).astype(np.float32))
        d = v3(*[std_min(fg[k], f32(f32(1.0) - fg[k])) for k in range(3)])
        mind = std_min(std_min(d[0], d[1]), d[2])
        sg = sub(mul(dsign(D), f32(2)), f32(1))
        nn = v3(*[sg[k] if mind == d[k] else f32(0.0) for k in range(3)])
        return normalize(xform_vec(nn, self.matrix))


class Scene:
    def __init__(self, vols, mats, points=(), dir_light=(v3(1, 0, 0), v3(0, 0, 0)), sky=(0.392, 0.584, 0.829)):
        self.vols, self.mats = vols, mats
        self.points = list(points)
        self.dir = dir_light
        self.sky = v3(*sky)
        self.cells = 0
        self.shadows = 0
        self.arms = set()  # the random / geometric decisions taken (branch coverage of the KATs)

    def albedo(self, m):
        return v3(*self.mats[m]["albedo"])

    # Scene::FindNearest (scene.cpp:751-811) on an object-space ray; returns (hit, t, N, mat)
    def scene_find_nearest(self, v, O, D, rD, t_in):
        s = v.setup(O, D, rD, dsign(D))
        if s is None:
            return False, t_in, None, None
        while s["t"] < t_in:
            c = v.cell(s["X"], s["Y"], s["Z"])
            self.cells += 1
            if c != NONE and s["t"] < t_in:
                return True, s["t"], v.normal(O, D, s["t"]), c
            if not Vol.advance(s, v.n):
                break
        return False, t_in, None, None

    def find_nearest(self, ray):  # Renderer::FindNearest (renderer.cpp:946-1018)
        vox = -2
        for i, v in enumerate(self.vols):
            O = xform_pos_sse(ray.O, v.inv)
            D = xform_vec_sse(ray.D, v.inv)
            rD = v3(*[f32(f32(1) / D[k]) for k in range(3)])
            hit, t, N, m = self.scene_find_nearest(v, O, D, rD, ray.t)
            if hit:
                ray.t, ray.N, ray.mat, vox = t, N, m, i
        return vox

    def is_occluded(self, ray):  # Renderer::IsOccluded (renderer.cpp:209-243) + Scene::IsOccluded
        self.shadows += 1
        for v in self.vols:
            O = xform_pos(ray.O, v.inv)
            D = xform_vec(ray.D, v.inv)
            rD = v3(*[f32(f32(1) / D[k]) for k in range(3)])
            s = v.setup(O, D, rD, dsign(D))
            if s is None:
                continue
            while s["t"] < ray.t:
                c = v.cell(s["X"], s["Y"], s["Z"])
                self.cells += 1
                if c != NONE:
                    if s["t"] < ray.t:
                        return True
                    break
                if not Vol.advance(s, v.n, occlusion=True):
                    break
        return False

    def exit_march(self, vox, ray, glass):  # FindMaterialExit / FindSmokeExit (scene.cpp:875-1006)
        v = self.vols[vox]
        O = xform_pos(ray.O, v.inv)
        D = xform_vec(ray.D, v.inv)
        rD = v3(*[f32(f32(1) / D[k]) for k in range(3)])
        s = v.setup(O, D, rD, dsign(D))
        if s is None:
            return False
        while True:
            c = v.cell(s["X"], s["Y"], s["Z"])
            self.cells += 1
            leave = (c != 8) if glass else (c > 14 or c < 9)
            if leave:
                ray.t, ray.N, ray.mat = s["t"], v.normal(O, D, s["t"]), c
                return True
            if not Vol.advance(s, v.n):
                break
        ray.t = s["t"]
        return False

    def illumination(self, ray, g):  # Illumination (renderer.cpp:738-764), point + directional
        lc = len(self.points) + 1
        idx = int(f32(g.rf() * f32(lc)))
        ip, n = ray.point(), ray.N
        inc = v3(0, 0, 0)
        if idx < len(self.points):  # PointLightEvaluate (renderer.cpp:102-131)
            pos, col = self.points[idx]
            dr = sub(pos, ip)
            dst = length(dr)
            dn = mul(dr, f32(f32(1.0) / dst))
            c = dot(dn, n)
            if not (c <= f32(0.0)):
                li = mul(mul(col, std_max(f32(0.0), c)), f32(f32(1.0) / f32(dst * dst)))
                sh = Ray(offset_ray(ip, n), dn)
                sh.t = dst
                if not self.is_occluded(sh):
                    inc = mul(li, self.albedo(ray.mat))
        else:  # DirectionalLightEvaluate (renderer.cpp:315-338)
            dr = -self.dir[0]
            c = dot(dr, n)
            if not (c <= f32(0)):
                li = mul(self.dir[1], std_max(f32(0.0), c))
                sh = Ray(offset_ray(ip, n), dr)
                if not self.is_occluded(sh):
                    inc = mul(li, self.albedo(ray.mat))
        return mul(inc, f32(lc))

    def trace(self, ray, depth, g):  # Renderer::Trace (renderer.cpp:1076-1328)
        if depth < 0:
            return v3(0, 0, 0)
        vox = self.find_nearest(ray)
        m = ray.mat
        if m == NONE:
            return self.sky.copy()
        mat = self.mats[m]
        if 5 <= m <= 7:  # metal :1103-1114
            refl = reflect(ray.D, ray.N)
            o = offset_ray(ray.point(), ray.N)
            nr = Ray(o, add(refl, mul(g.sphere_sample(), f32(mat["roughness"]))))
            return mul(self.trace(nr, depth - 1, g), self.albedo(m))
        if m <= 4:  # non-metal :1117-1144
            diffuse = g.rf() > schlick_nonmetal(dot(-ray.D, ray.N))
            self.arms.add(("non_metal", "diffuse" if diffuse else "specular"))
            if diffuse:
                rdir = add(ray.N, g.sphere_sample())  # RandomLambertianReflectionVector
                inc = self.illumination(ray, g)
                nr = Ray(offset_ray(ray.point(), ray.N), rdir)
                color = add(v3(0, 0, 0), inc)
                return add(color, mul(self.trace(nr, depth - 1, g), self.albedo(m)))
            refl = reflect(ray.D, ray.N)
            o = offset_ray(ray.point(), ray.N)
            nr = Ray(o, add(refl, mul(g.sphere_sample(), f32(mat["roughness"]))))
            return self.trace(nr, depth - 1, g)
        if m == 8:  # glass :1146-1209
            color = v3(1, 1, 1)
            in_glass = ray.inside
            ior = f32(mat["ior"])
            ratio = ior if in_glass else f32(f32(1.0) / ior)
            inside_volume = True
            if in_glass:
                color = self.albedo(m)
                inside_volume = self.exit_march(vox, ray, glass=True)
            if not inside_volume:
                ray.O = add(ray.O, mul(ray.D, ray.t))
                ray.t = f32(0)
            c = std_min(dot(-ray.D, ray.N), f32(1.0))
            s = f32(np.sqrt(f32(f32(1.0) - f32(c * c))))
            cannot = f32(ratio * s) > f32(1.0)
            refl = cannot or schlick(c, ratio) > g.rf()
            self.arms.add(("glass", "inside" if ray.inside else "outside", "reflect" if refl else "refract",
                           "exit" if inside_volume else "left grid"))
            if refl:
                rdir, rn = reflect(ray.D, ray.N), ray.N
            else:
                rdir, rn = refract(ray.D, ray.N, ratio), -ray.N
                in_glass = not in_glass
            nr = Ray(offset_ray(ray.point(), rn), rdir)
            nr.inside = in_glass
            return mul(self.trace(nr, depth - 1, g), color)
        if m <= 14:  # smoke :1210-1314
            color = v3(1, 1, 1)
            in_glass = ray.inside
            inside_volume = True
            intensity, dist = f32(0), f32(0)
            if vox == 0:
                self.illumination(ray, g)  # the player light probe (result only printed)
            if in_glass:
                intensity = f32(mat["emissive"])
                color = self.albedo(m)
                inside_volume = self.exit_march(vox, ray, glass=False)
                dist = ray.t
            threshold = f32(f32(g.rf() * f32(100)) - intensity)
            scatter = f32(g.rf() * dist) > threshold
            self.arms.add(("smoke", "inside" if ray.inside else "outside", "scatter" if scatter else "pass"))
            if scatter:
                lo, hi = f32(ray.t * f32(0.45)), ray.t
                tt = f32(lo + f32(g.rf() * f32(hi - lo)))  # Rand(min, max)
                ray.O = add(ray.O, mul(ray.D, tt))
                ray.D = g.random_direction()
                ray.t = f32(0)
            flipped = sub(v3(1, 1, 1), color)
            e = mul(flipped, f32(f32(-dist) * intensity))
            color = v3(expf(e[0]), expf(e[1]), expf(e[2]))  # Absorption (renderer.cpp:1596-1608)
            if not inside_volume:
                ray.O = add(ray.O, mul(ray.D, ray.t))
                ray.t = f32(0)
            rdir = refract(ray.D, ray.N, f32(1.0))
            nr = Ray(offset_ray(ray.point(), -ray.N), rdir)
            nr.inside = not in_glass
            return mul(self.trace(nr, depth - 1, g), color)
        if m == 15:  # emissive :1315-1316
            return mul(self.albedo(m), f32(mat["emissive"]))
        rdir = g.diffuse_reflection(ray.N)  # default :1319-1326
        inc = self.illumination(ray, g)
        nr = Ray(offset_ray(ray.point(), ray.N), rdir)
        return mul(add(self.trace(nr, depth - 1, g), inc), self.albedo(m))


# --------------------------------------------------------------- KAT scenes
N = 16


def room_cells():
    """A 16^3 room: a floor (y < 2, default material 20), a back wall (z = 12..13) of the
    material under test in x, y in [3, 12], a glass block and a smoke block beside it."""
    c = np.full(N * N * N, NONE, np.uint8)
    idx = lambda x, y, z: x + y * N + z * N * N
    for x in range(N):
        for z in range(N):
            for y in range(2):
                c[idx(x, y, z)] = 20
    return c, idx


MATS = {
    0: dict(albedo=(0.8, 0.7, 0.6), roughness=0.3, emissive=0.0, ior=1.5),   # NON_METAL_WHITE
    6: dict(albedo=(0.9, 0.6, 0.3), roughness=0.25, emissive=0.0, ior=1.5),  # METAL_MID
    8: dict(albedo=(0.7, 0.9, 0.95), roughness=0.0, emissive=0.0, ior=1.45), # GLASS (MaterialSetUp IOR 1.45)
    11: dict(albedo=(0.5, 0.55, 0.6), roughness=1.0, emissive=7.0, ior=1.0), # SMOKE_MID_DENSITY
    15: dict(albedo=(1.0, 0.9, 0.5), roughness=1.0, emissive=5.0, ior=1.0),  # EMISSIVE (emissive 5)
    20: dict(albedo=(0.45, 0.6, 0.35), roughness=1.0, emissive=0.0, ior=1.5),  # a model palette colour
}


def kat_scene(wall_mat):
    c, idx = room_cells()
    for x in range(3, 13):
        for y in range(3, 13):
            for z in (12, 13):
                c[idx(x, y, z)] = wall_mat
    for x in range(3, 6):  # a glass block and a smoke block in front of the wall
        for y in range(2, 5):
            for z in range(6, 9):
                c[idx(x, y, z)] = 8
                c[idx(x + 6, y, z)] = 11
    mats = {m: MATS[m] for m in MATS}
    points = [(v3(0.5, 0.9, 0.2), v3(1.0, 0.95, 0.9))]
    d = (v3(-0.3, -1.0, 0.4), v3(0.6, 0.6, 0.7))
    return c, mats, points, d


def to_oracle(pkg, orc, cells, mats, points, d, vols):
    """The same scene as the oracle's (and the device's) SceneDesc."""
    abi, sc = pkg.abi, pkg.scene
    m = (abi.Material * 256)()
    for i in range(256):
        m[i].albedo[:] = [1.0, 1.0, 1.0]
        m[i].roughness, m[i].emissive, m[i].ior = 1.0, 0.0, 1.5
    for i, e in mats.items():
        m[i].albedo[:] = [float(f32(a)) for a in e["albedo"]]
        m[i].roughness, m[i].emissive, m[i].ior = float(f32(e["roughness"])), float(f32(e["emissive"])), float(f32(e["ior"]))
    vs = []
    for v in vols:
        vol = abi.Volume()
        vol.grid_id = 0
        vol.matrix[:] = [float(x) for x in v.matrix]
        vol.inv_matrix[:] = [float(x) for x in v.inv]
        vol.b0[:] = [float(x) for x in v.b0]
        vol.b1[:] = [float(x) for x in v.b1]
        vs.append(vol)
    desc = sc._scene("kat", [sc.GridSpec(n=N, dense=cells)], vs, m,
                     [sc.point_light(tuple(map(float, p)), tuple(map(float, c))) for p, c in points], [], [],
                     sc.dir_light(tuple(map(float, d[0])), tuple(map(float, d[1]))), (0.5, 0.5, -1.0), (0.5, 0.5, 0.5),
                     16, 16)
    return desc


def api_rays(abi, rays):
    arr = (abi.Ray * len(rays))()
    for i, (o, dd, tmax, inside) in enumerate(rays):
        arr[i].origin[:] = [float(x) for x in o]
        arr[i].direction[:] = [float(x) for x in dd]
        arr[i].tmax = float(tmax)
        arr[i].inside_glass = 1 if inside else 0
    return arr


# (origin, direction, inside_glass, material it must reach first, seeds, depth-1 branches
# the seed set must cover).  Rays start outside the unit cube (Setup3DDDA's Cube::Intersect
# entry) and travel in -y / +z / -x directions (negative steps and Dsign = 1 axes).
CASES = [
    ("default", 20, ((0.37, 1.3, 0.31), (0.11, -1.0, 0.23), False)),
    ("non_metal", 0, ((0.41, 0.47, -0.8), (0.05, 0.03, 1.0), False)),
    ("metal", 6, ((0.66, 0.52, -0.7), (-0.07, -0.02, 1.0), False)),
    ("emissive", 15, ((0.52, 0.61, -0.9), (0.02, -0.05, 1.0), False)),
    ("glass_outside", 8, ((0.27, 0.23, -0.5), (0.02, -0.03, 1.0), False)),
    ("glass_inside", 8, ((0.27, 0.22, 0.45), (0.31, 0.05, 1.0), True)),
    ("smoke_outside", 11, ((0.65, 0.24, -0.5), (0.01, 0.0, 1.0), False)),
    ("smoke_inside", 11, ((0.65, 0.2, 0.47), (0.1, 0.35, 0.9), True)),
]
SEEDS = [0x12345678 + 977 * k for k in range(24)]


def _expected(cells, mats, points, d, vols, o, dd, inside, seed, depth):
    s = Scene(vols, mats, points, d)
    r = Ray(v3(*o), v3(*dd), inside=inside)
    v = s.trace(r, depth, Rng(seed))
    return v, s


@pytest.mark.parametrize("name,wall,ray", CASES, ids=[c[0] for c in CASES])
def test_trace_depth1_every_branch(pkg, orc, name, wall, ray):
    """Trace(ray, 1) over 24 seeds per case: the oracle's radiance equals the numpy
    restatement's bit for bit, and so do the shadow-ray and DDA-cell counts."""
    wall_mat = {"default": 20, "non_metal": 0, "metal": 6, "emissive": 15}.get(name, 0)
    cells, mats, points, d = kat_scene(wall_mat)
    vols = [Vol(cells, N)]
    desc = to_oracle(pkg, orc, cells, mats, points, d, vols)
    o = orc.Oracle(pkg.abi, desc)
    org, dirn, inside = ray
    # the ray reaches the material under test first
    h = o.find_nearest(api_rays(pkg.abi, [(org, dirn, 1e34, inside)]))[0]
    assert h.material == wall, (name, h.material)
    rays = api_rays(pkg.abi, [(org, dirn, 1e34, inside)] * len(SEEDS))
    got, st = o.trace(rays, np.array(SEEDS, np.uint32), 1, (0.392, 0.584, 0.829), 3)
    shadows = cells_n = 0
    for i, seed in enumerate(SEEDS):
        exp, s = _expected(cells, mats, points, d, vols, org, dirn, inside, seed, 1)
        assert np.array_equal(fbits(got[i]), fbits(exp)), (name, hex(seed), got[i], exp)
        shadows += s.shadows
        cells_n += s.cells
    assert (st.shadow_rays, st.dda_cells) == (shadows, cells_n)


def test_branch_arms_are_covered():
    """The seeds above take both arms of the random decisions the KATs exist for: the
    non-metal Schlick draw (diffuse / specular), glass reflect and refract from outside and
    from inside after FindMaterialExit, and the smoke scatter draw after FindSmokeExit."""
    arms = set()
    for name, wall, (org, dirn, inside) in CASES:
        wall_mat = {"default": 20, "non_metal": 0, "metal": 6, "emissive": 15}.get(name, 0)
        cells, mats, points, d = kat_scene(wall_mat)
        for seed in SEEDS:
            s = Scene([Vol(cells, N)], mats, points, d)
            s.trace(Ray(v3(*org), v3(*dirn), inside=inside), 1, Rng(seed))
            arms |= s.arms
    need = {("non_metal", "diffuse"), ("non_metal", "specular"),
            ("glass", "outside", "reflect", "exit"), ("glass", "outside", "refract", "exit"),
            ("glass", "inside", "refract", "exit"), ("glass", "inside", "reflect", "exit"),
            ("smoke", "inside", "scatter"), ("smoke", "inside", "pass"), ("smoke", "outside", "pass")}
    assert need <= arms, sorted(need - arms)


def _messy_volume(cells):
    """A rotated, non-uniformly scaled, translated volume whose invMatrix has many-bit
    entries (pairwise and left-to-right sums differ) and a cube off the origin."""
    a, b = 0.43, -0.29
    ca, sa, cb, sb = math.cos(a), math.sin(a), math.cos(b), math.sin(b)
    R = np.array([[ca, -sa, 0], [sa, ca, 0], [0, 0, 1]]) @ np.array([[cb, 0, sb], [0, 1, 0], [-sb, 0, cb]])
    S = np.diag([0.8, 1.3, 0.95])
    Mo = np.eye(4)
    Mo[:3, :3] = R @ S
    Mo[:3, 3] = [0.137, -0.211, 0.093]
    inv = np.linalg.inv(Mo)
    return Vol(cells, N, matrix=Mo.reshape(-1).astype(np.float32), inv=inv.reshape(-1).astype(np.float32),
               b0=(0.0625, -0.125, 0.03125), b1=(1.0625, 0.875, 1.03125))


def test_setup3ddda_general_and_sse_sum_order(pkg, orc):
    """Renderer::FindNearest / IsOccluded in a rotated, scaled, offset volume, from inside and
    outside the cube, every direction octant: t, normal, material and cells equal the numpy
    restatement (Setup3DDDA's general tmax / tdelta with the 5e-5 nudge and the clamp), with
    the SSE pairwise sums for FindNearest and left-to-right sums for IsOccluded — and the
    case set contains rays where the other sum order changes the object-space origin."""
    cells, mats, points, d = kat_scene(20)
    vol = _messy_volume(cells)
    desc = to_oracle(pkg, orc, cells, mats, points, d, [vol])
    o = orc.Oracle(pkg.abi, desc)
    rng = np.random.default_rng(7)
    rays, exp, exp_scalar = [], [], []
    differs = 0
    for k in range(160):
        org = rng.uniform(-0.7, 1.7, 3) if k % 3 else rng.uniform(0.15, 0.85, 3)
        dd = rng.normal(size=3)
        r = Ray(v3(*org), v3(*dd))
        if np.any(xform_pos_sse(r.O, vol.inv) != xform_pos(r.O, vol.inv)):
            differs += 1
        s = Scene([vol], mats, points, d)
        vox = s.find_nearest(r)
        rays.append((org, dd, 1e34, False))
        exp.append((r.t, r.N if vox >= 0 else v3(0, 0, 0), r.mat, vox, s.cells))
        # the same walk with left-to-right sums (what the SSE order must NOT give)
        rs, ss = Ray(v3(*org), v3(*dd)), Scene([vol], mats, points, d)
        ss.find_nearest_scalar = True
        for i, v in enumerate(ss.vols):
            O, D = xform_pos(rs.O, v.inv), xform_vec(rs.D, v.inv)
            rD = v3(*[f32(f32(1) / D[k2]) for k2 in range(3)])
            hit, t, _, _ = ss.scene_find_nearest(v, O, D, rD, rs.t)
            exp_scalar.append((fbits(t), ss.cells))
    assert differs >= 20
    hits = o.find_nearest(api_rays(pkg.abi, rays))
    # the case set is sensitive to the sum order: left-to-right sums change t / cells somewhere
    assert sum((fbits(h.t), h.cells) != e for h, e in zip(hits, exp_scalar)) >= 1
    nhit = 0
    for h, (t, n, m, vox, cn) in zip(hits, exp):
        assert fbits(h.t) == fbits(t) and h.material == m and h.vox_index == vox and h.cells == cn
        if vox >= 0:
            nhit += 1
            assert np.array_equal(fbits(np.array(h.normal[:], np.float32)), fbits(n))
    assert nhit >= 15
    # IsOccluded: the same rays bounded at a distance, scalar transforms
    occ_rays, occ_exp = [], []
    for (org, dd, _, _), (t, *_rest) in zip(rays, exp):
        bound = f32(0.6)
        r = Ray(v3(*org), v3(*dd), t=bound)
        s = Scene([vol], mats, points, d)
        occ_exp.append((s.is_occluded(r), s.cells))
        occ_rays.append((org, dd, bound, False))
    occ, ocells = o.is_occluded(api_rays(pkg.abi, occ_rays))
    assert [bool(x) for x in occ] == [e[0] for e in occ_exp]
    assert [int(x) for x in ocells] == [e[1] for e in occ_exp]
    assert 10 <= sum(e[0] for e in occ_exp) <= len(occ_exp) - 10


@pytest.mark.gpu
def test_kat_paths_on_device(pkg):
    """The same depth-1 KATs through the library's vpx_trace on the GPU: bit for bit equal
    to the numpy restatement (no oracle in between)."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    for name, wall, (org, dirn, inside) in CASES:
        wall_mat = {"default": 20, "non_metal": 0, "metal": 6, "emissive": 15}.get(name, 0)
        cells, mats, points, d = kat_scene(wall_mat)
        vols = [Vol(cells, N)]
        desc = to_oracle(pkg, None, cells, mats, points, d, vols)
        ctx = pkg.context.Context(0)
        ctx.load_scene(desc)
        rays = api_rays(pkg.abi, [(org, dirn, 1e34, inside)] * len(SEEDS))
        got = ctx.trace(rays, np.array(SEEDS, np.uint32), 1, (0.392, 0.584, 0.829), 3)
        got = got[0] if isinstance(got, tuple) else got
        ctx.close()
        for i, seed in enumerate(SEEDS):
            exp, _ = _expected(cells, mats, points, d, vols, org, dirn, inside, seed, 1)
            assert np.array_equal(fbits(np.asarray(got[i], np.float32)), fbits(exp)), (name, hex(seed))
