/*
 * vpx_oracle.c — CPU restatement of the reference per-pixel voxel ray-trace path.
 *
 * TEST INFRASTRUCTURE ONLY (the checker, never the product).  See vpx_oracle.h for
 * the parity status ("parity unpinned" for the trace path; the .vox decode is pinned).
 *
 * Every function names the reference file:line it restates.  Expressions keep the
 * reference's operand order; the file is compiled with -ffp-contract=off -fno-fast-math
 * and runs with FTZ|DAZ set (template/template.cpp:130).  Decisions on the reference's
 * platform-dependent operations:
 *   - FastReciprocal (rcpps + Newton, renderer.cpp:929-934) and _mm_rsqrt_ps
 *     (tmpl8math.h:2356-2360) -> exact 1/x and 1/sqrtf(x);
 *   - unspecified argument evaluation order (make_float3(RandomFloat(), ...)) -> left
 *     to right;
 *   - sinf/cosf/powf/expf/SVML -> correctly rounded float results, computed as
 *     (float)f((double)x);
 *   - GetVoxel's 32-bit index arithmetic (scene.h:246) -> 64-bit (wraps at N >= 2048).
 */
#include "vpx_oracle.h"

#include <limits.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#if defined(__x86_64__) || defined(__i386__)
#include <xmmintrin.h>
#define ORACLE_X86 1
#endif

#define NONE_MAT 255u
#define PI_F 3.14159265358979323846264f /* common.h:8 */
#define BIG_T 1e34f

/* ------------------------------------------------------------------ vector math -- */
/* float3 operators of template/tmpl8math.h (operator+ :913, operator- :1361, ...). */
typedef struct { float x, y, z; } v3;

static inline v3 V3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 v3f(const float* p) { return V3(p[0], p[1], p[2]); }
static inline v3 vadd(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vmul(v3 a, v3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 vdiv(v3 a, v3 b) { return V3(a.x / b.x, a.y / b.y, a.z / b.z); }
static inline v3 vmuls(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
static inline v3 vdivs(v3 a, float s) { return V3(a.x / s, a.y / s, a.z / s); }
static inline v3 vneg(v3 a) { return V3(-a.x, -a.y, -a.z); }
static inline float vdot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; } /* :2259 */
static inline float vlength(v3 a) { return sqrtf(vdot(a, a)); }                   /* :2319 */
static inline v3 vnormalize(v3 v) /* tmpl8math.h:2350-2354, rsqrtf = 1/sqrtf (:411) */
{
    const float inv = 1.0f / sqrtf(vdot(v, v));
    return vmuls(v, inv);
}
static inline v3 vcross(v3 a, v3 b) /* tmpl8math.h:2494 */
{
    return V3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
/* std::min / std::max as libstdc++/MSVC define them (NaN and signed-zero exact). */
static inline float smin(float a, float b) { return (b < a) ? b : a; }
static inline float smax(float a, float b) { return (a < b) ? b : a; }

static inline uint32_t f2u_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f_bits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* static_cast<int>(float) as x86 cvttss2si evaluates it (out of range / NaN -> INT_MIN). */
static inline int f2i_trunc(float f)
{
    if (!(f > -2147483904.0f && f < 2147483648.0f)) return INT_MIN;
    return (int)f;
}

/* sinf / cosf / expf / powf(x, 5) (tmpl8math.h:2506-2508, renderer.cpp:1593, 1607, 1615):
 * the float result of one fixed double-precision evaluation (Cody-Waite reduction, fdlibm
 * kernel polynomials), within 1 ulp (double) of the true value, hence the correctly rounded
 * float except at double-rounding midpoints.  tests/test_cpu_oracle.py checks these against
 * (float)libm(double) on 4M arguments each.  The device evaluates the same operations in the
 * same order (csrc/vpx_trace.hpp namespace dm), so the two agree bit for bit by construction
 * -- the MSVC powf/sinf the reference links are unknowable here (parity hazard 4). */
static const double dm_S1 = -1.66666666666666324348e-01, dm_S2 = 8.33333333332248946124e-03,
                    dm_S3 = -1.98412698298579493134e-04, dm_S4 = 2.75573137070700676789e-06,
                    dm_S5 = -2.50507602534068634195e-08, dm_S6 = 1.58969099521155010221e-10;
static const double dm_C1 = 4.16666666666666019037e-02, dm_C2 = -1.38888888888741095749e-03,
                    dm_C3 = 2.48015872894767294178e-05, dm_C4 = -2.75573143513906633035e-07,
                    dm_C5 = 2.08757232129817482790e-09, dm_C6 = -1.13596475577881948265e-11;
static const double dm_invpio2 = 6.36619772367581382433e-01, dm_pio2_1 = 1.57079632673412561417e+00,
                    dm_pio2_1t = 6.07710050650619224932e-11;
static const double dm_ln2hi = 6.93147180369123816490e-01, dm_ln2lo = 1.90821492927058770002e-10,
                    dm_invln2 = 1.44269504088896338700e+00;
static const double dm_P1 = 1.66666666666666019037e-01, dm_P2 = -2.77777777770155933842e-03,
                    dm_P3 = 6.61375632143793436117e-05, dm_P4 = -1.65339022054652515390e-06,
                    dm_P5 = 4.13813679705723846039e-08;
static inline double dm_ksin(double x)
{
    const double z = x * x, v = z * x;
    const double r = dm_S2 + z * (dm_S3 + z * (dm_S4 + z * (dm_S5 + z * dm_S6)));
    return x + v * (dm_S1 + z * r);
}
static inline double dm_kcos(double x)
{
    const double z = x * x;
    const double r = z * (dm_C1 + z * (dm_C2 + z * (dm_C3 + z * (dm_C4 + z * (dm_C5 + z * dm_C6)))));
    const double hz = 0.5 * z, w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + z * r);
}
/* |x| < 2^20: k * dm_pio2_1 is exact (33-bit constant) */
static inline void dm_sincosf(float xf, float* sf, float* cf)
{
    const double x = (double)xf;
    const double k = rint(x * dm_invpio2);
    const double r = (x - k * dm_pio2_1) - k * dm_pio2_1t;
    const int n = (int)k & 3;
    const double s = dm_ksin(r), c = dm_kcos(r);
    *sf = (float)(n == 0 ? s : n == 1 ? c : n == 2 ? -s : -c);
    *cf = (float)(n == 0 ? c : n == 1 ? -s : n == 2 ? -c : s);
}
static inline float cr_sinf(float x) { float s, c; dm_sincosf(x, &s, &c); return s; }
static inline float cr_cosf(float x) { float s, c; dm_sincosf(x, &s, &c); return c; }
static inline float cr_expf(float xf)
{
    if (xf != xf) return xf;
    double x = (double)xf;
    x = x < -800.0 ? -800.0 : (x > 800.0 ? 800.0 : x);
    const double k = rint(x * dm_invln2);
    const double hi = x - k * dm_ln2hi, lo = k * dm_ln2lo;
    const double r = hi - lo, t = r * r;
    const double c = r - t * (dm_P1 + t * (dm_P2 + t * (dm_P3 + t * (dm_P4 + t * dm_P5))));
    const double y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);
    return (float)ldexp(y, (int)k);
}
static inline float cr_pow5f(float xf)
{
    const double x = (double)xf, x2 = x * x, x4 = x2 * x2;
    return (float)(x4 * x);
}
/* for the CPU pin test: fn 0 sin, 1 cos, 2 exp, 3 pow5 over n arguments */
void oracle_dm_eval(int fn, const float* x, float* out, uint32_t n)
{
    for (uint32_t i = 0; i < n; ++i)
        out[i] = fn == 0 ? cr_sinf(x[i]) : fn == 1 ? cr_cosf(x[i]) : fn == 2 ? cr_expf(x[i]) : cr_pow5f(x[i]);
}

/* ----------------------------------------------------------------------- RNG -- */
/* WangHash, template/tmpl8math.cpp:20-27 */
uint32_t oracle_wang_hash(uint32_t s)
{
    s = (s ^ 61u) ^ (s >> 16);
    s *= 9u, s = s ^ (s >> 4);
    s *= 0x27d4eb2du;
    s = s ^ (s >> 15);
    return s;
}

/* RandomUInt, template/tmpl8math.cpp:119-125 (Marsaglia xorshift32, 13/17/5) */
uint32_t oracle_xorshift32(uint32_t* seed)
{
    uint32_t s = *seed;
    s ^= s << 13;
    s ^= s >> 17;
    s ^= s << 5;
    *seed = s;
    return s;
}

/* RandomFloat, template/tmpl8math.cpp:130-133 */
float oracle_random_float(uint32_t* seed)
{
    return (float)oracle_xorshift32(seed) * 2.3283064365387e-10f;
}

/* InitSeed on a fresh thread-local seed (tmpl8math.cpp:16, 35-38) keyed by pixel. */
uint32_t oracle_pixel_seed(uint32_t seed_base, uint32_t frame_index, uint32_t width,
                           uint32_t height, uint32_t x, uint32_t y)
{
    const uint32_t k = seed_base + frame_index * (width * height) + y * width + x;
    return 0x12345678u + oracle_wang_hash((k + 1u) * 17u);
}

/* ---------------------------------------------------------------------- Ray -- */
/* Ray, template/scene.h:64-155 */
typedef struct {
    v3 O, D, rD, Dsign, N;
    float t;
    int inside;   /* isInsideGlass */
    uint32_t mat; /* indexMaterial */
} ray_t;

/* Ray::ComputeDsign, template/scene.cpp:49-57 (== ComputeDsign_SSE :59-80) */
static inline v3 compute_dsign(v3 d)
{
    const float sx = (float)(f2u_bits(d.x) >> 31), sy = (float)(f2u_bits(d.y) >> 31),
                sz = (float)(f2u_bits(d.z) >> 31);
    return vmuls(vadd(V3(sx * 2 - 1, sy * 2 - 1, sz * 2 - 1), V3(1, 1, 1)), 0.5f);
}

/* Ray::Ray(origin, direction, rayLength = 1e34), template/scene.cpp:83-93 */
static ray_t make_ray(v3 o, v3 dir)
{
    ray_t r;
    r.O = o;
    r.t = BIG_T;
    r.D = vnormalize(dir);
    r.rD = V3(1 / r.D.x, 1 / r.D.y, 1 / r.D.z);
    r.Dsign = compute_dsign(r.D);
    r.N = V3(0, 0, 0);
    r.inside = 0;
    r.mat = NONE_MAT;
    return r;
}

static inline v3 ray_point(const ray_t* r) { return vadd(r->O, vmuls(r->D, r->t)); } /* scene.h:80-83 */

/* ----------------------------------------------------------------- transforms -- */
/* TransformPosition_SSEM, template/tmpl8math.cpp:369-380: pairwise (a0m0+a1m1)+(a2m2+m3) */
static inline v3 xform_pos_ssem(v3 a, const float* m)
{
    return V3((a.x * m[0] + a.y * m[1]) + (a.z * m[2] + m[3]),
              (a.x * m[4] + a.y * m[5]) + (a.z * m[6] + m[7]),
              (a.x * m[8] + a.y * m[9]) + (a.z * m[10] + m[11]));
}
/* TransformVector_SSEM, template/tmpl8math.cpp:393-402 */
static inline v3 xform_vec_ssem(v3 a, const float* m)
{
    return V3((a.x * m[0] + a.y * m[1]) + a.z * m[2], (a.x * m[4] + a.y * m[5]) + a.z * m[6],
              (a.x * m[8] + a.y * m[9]) + a.z * m[10]);
}
/* TransformPosition, template/tmpl8math.cpp:345-348 with operator*(float4, mat4) :337-343 */
static inline v3 xform_pos(v3 a, const float* m)
{
    return V3(m[0] * a.x + m[1] * a.y + m[2] * a.z + m[3] * 1.0f,
              m[4] * a.x + m[5] * a.y + m[6] * a.z + m[7] * 1.0f,
              m[8] * a.x + m[9] * a.y + m[10] * a.z + m[11] * 1.0f);
}
/* TransformVector, template/tmpl8math.cpp:350-353 */
static inline v3 xform_vec(v3 a, const float* m)
{
    return V3(m[0] * a.x + m[1] * a.y + m[2] * a.z + m[3] * 0.0f,
              m[4] * a.x + m[5] * a.y + m[6] * a.z + m[7] * 0.0f,
              m[8] * a.x + m[9] * a.y + m[10] * a.z + m[11] * 0.0f);
}

/* OffsetRay, template/tmpl8math.cpp:473-487 (Ray Tracing Gems ch. 6) */
static v3 offset_ray(v3 p, v3 n)
{
    const int ox = f2i_trunc(256.0f * n.x), oy = f2i_trunc(256.0f * n.y), oz = f2i_trunc(256.0f * n.z);
    const float pix = u2f_bits(f2u_bits(p.x) + (uint32_t)((p.x < 0) ? -ox : ox));
    const float piy = u2f_bits(f2u_bits(p.y) + (uint32_t)((p.y < 0) ? -oy : oy));
    const float piz = u2f_bits(f2u_bits(p.z) + (uint32_t)((p.z < 0) ? -oz : oz));
    const float origin = 1.0f / 32.0f, fs = 1.0f / 65536.0f;
    return V3(fabsf(p.x) < origin ? p.x + fs * n.x : pix, fabsf(p.y) < origin ? p.y + fs * n.y : piy,
              fabsf(p.z) < origin ? p.z + fs * n.z : piz);
}

void oracle_offset_ray(const float p[3], const float n[3], float out[3])
{
    const v3 r = offset_ray(v3f(p), v3f(n));
    out[0] = r.x, out[1] = r.y, out[2] = r.z;
}

/* --------------------------------------------------------------------- voxels -- */
typedef struct {
    const oracle_scene* sc;
    uint32_t rng;
    float sky[3];
    int sky_tex; /* activateSky with a texture: SampleSky reads sc->sky_pixels */
    int area_samples;
    uint64_t shadow_rays, nearest_calls, dda_cells;
} tctx;

/* atan2_approximation2, template/tmpl8math.cpp:405-426 (ONEQTR_PI = PI / 4.0 in double,
   stored as float). */
static float atan2_approximation2(float y, float x)
{
    const float ONEQTR_PI = (float)((double)PI_F / 4.0);
    const float THRQTR_PI = (float)(3.0 * (double)PI_F / 4.0);
    float r, angle;
    const float abs_y = fabsf(y) + 1e-10f;
    if (x < 0.0f) {
        r = (x + abs_y) / (abs_y - x);
        angle = THRQTR_PI;
    } else {
        r = (x - abs_y) / (x + abs_y);
        angle = ONEQTR_PI;
    }
    angle += (0.1963f * r * r - 0.9817f) * r;
    return y < 0.0f ? -angle : angle;
}

/* FastAcos, template/tmpl8math.cpp:429-443 */
static float fast_acos(float x)
{
    const float negate = (float)(x < 0);
    x = fabsf(x);
    float ret = (float)-0.0187293;
    ret = ret * x;
    ret = ret + 0.0742610f;
    ret = ret * x;
    ret = ret - 0.2121144f;
    ret = ret * x;
    ret = ret + 1.5707288f;
    ret = ret * sqrtf(1.0f - x);
    ret = ret - 2 * negate * ret;
    return negate * 3.14159265358979f + ret;
}

/* Renderer::SampleSky, renderer.cpp:2308-2326 (INV2PI / INVPI: common.h:13-14).  The
   int arithmetic wraps as on x86; an index past the image (only from a NaN direction)
   is clamped to the last texel instead of reading outside it (reference: UB). */
static v3 sample_sky(const tctx* c, v3 d)
{
    if (!c->sky_tex) return V3(c->sky[0], c->sky[1], c->sky[2]);
    const oracle_scene* sc = c->sc;
    const float uf = (float)sc->sky_w * atan2_approximation2(d.z, d.x) * 0.15915494309189533576888f - 0.5f;
    const int u = f2i_trunc(uf);
    const float vf = (float)sc->sky_h * fast_acos(d.y) * 0.31830988618379067153777f - 0.5f;
    const int v = f2i_trunc(vf);
    const int32_t lin = (int32_t)((uint32_t)u + (uint32_t)v * sc->sky_w);
    uint32_t idx = lin > 0 ? (uint32_t)lin : 0u;
    const uint32_t last = sc->sky_w * sc->sky_h - 1u;
    if (idx > last) idx = last;
    const float* px = sc->sky_pixels + 3u * (uint64_t)idx;
    const float h = sc->sky_hdr;
    return V3(h * px[0], h * px[1], h * px[2]);
}

typedef struct {
    int sx, sy, sz;  /* step */
    uint32_t X, Y, Z;
    float t;
    v3 tdelta, tmax;
} dda_t;

/* Cube::Intersect, template/scene.cpp:166-202 */
static float cube_intersect(v3 b0, v3 b1, const ray_t* r)
{
    const int signx = r->D.x < 0, signy = r->D.y < 0, signz = r->D.z < 0;
    const float bx[2] = {b0.x, b1.x}, by[2] = {b0.y, b1.y}, bz[2] = {b0.z, b1.z};
    float tmin_x = (bx[signx] - r->O.x) * r->rD.x;
    float tmax_x = (bx[1 - signx] - r->O.x) * r->rD.x;
    const float tmin_y = (by[signy] - r->O.y) * r->rD.y;
    const float tmax_y = (by[1 - signy] - r->O.y) * r->rD.y;
    if (tmin_x > tmax_y || tmin_y > tmax_x) return BIG_T;
    tmin_x = smax(tmin_x, tmin_y);
    tmax_x = smin(tmax_x, tmax_y);
    const float tmin_z = (bz[signz] - r->O.z) * r->rD.z;
    const float tmax_z = (bz[1 - signz] - r->O.z) * r->rD.z;
    if (tmin_x > tmax_z || tmin_z > tmax_x) return BIG_T;
    tmin_x = smax(tmin_x, tmin_z);
    if (tmin_x > 0) return tmin_x;
    return BIG_T;
}

float oracle_cube_intersect(const float b0[3], const float b1[3], const float o[3],
                            const float d[3], const float rd[3])
{
    ray_t r;
    r.O = v3f(o), r.D = v3f(d), r.rD = v3f(rd);
    return cube_intersect(v3f(b0), v3f(b1), &r);
}

/* Cube::Contains, template/scene.cpp:205-210 */
static inline int cube_contains(v3 b0, v3 b1, v3 p)
{
    return p.x >= b0.x && p.y >= b0.y && p.z >= b0.z && p.x <= b1.x && p.y <= b1.y && p.z <= b1.z;
}

/* Scene::Setup3DDDA, template/scene.cpp:719-749 */
static int setup_dda(const vpx_volume* vol, uint32_t n, const ray_t* r, dda_t* s)
{
    const v3 b0 = v3f(vol->b0), b1 = v3f(vol->b1);
    s->t = 0;
    if (!cube_contains(b0, b1, r->O)) {
        s->t = cube_intersect(b0, b1, r);
        if (s->t > 1e33f) return 0;
    }
    const v3 vmin = b0;
    const v3 vmax = vsub(b1, b0);
    const float g = (float)n;
    const float cell = 1.0f / g;
    const v3 stepf = vsub(V3(1, 1, 1), vmuls(r->Dsign, 2)); /* 1 - Dsign*2 */
    s->sx = f2i_trunc(stepf.x), s->sy = f2i_trunc(stepf.y), s->sz = f2i_trunc(stepf.z);
    const v3 pos = vdiv(vmuls(vadd(vsub(r->O, vmin), vmuls(r->D, s->t + 0.00005f)), g), vmax);
    const v3 planes = vmuls(vsub(V3(ceilf(pos.x), ceilf(pos.y), ceilf(pos.z)), r->Dsign), cell);
    const int hi = (int)(n - 1);
    int px = f2i_trunc(pos.x), py = f2i_trunc(pos.y), pz = f2i_trunc(pos.z);
    px = px < 0 ? 0 : (px > hi ? hi : px); /* clamp(int3, 0, gridsize-1), tmpl8math.h:2110-2113 */
    py = py < 0 ? 0 : (py > hi ? hi : py);
    pz = pz < 0 ? 0 : (pz > hi ? hi : pz);
    s->X = (uint32_t)px, s->Y = (uint32_t)py, s->Z = (uint32_t)pz;
    s->tdelta = vmul(V3(cell * (float)s->sx, cell * (float)s->sy, cell * (float)s->sz), r->rD);
    s->tmax = vmul(vsub(vmul(planes, vmax), vsub(r->O, vmin)), r->rD);
    return 1;
}

static inline uint8_t grid_at(const oracle_grid* g, uint32_t x, uint32_t y, uint32_t z)
{
    const uint64_t n = g->n;
    return g->cells[(uint64_t)x + (uint64_t)y * n + (uint64_t)z * n * n];
}

/* One Amanatides-Woo step, shared by FindNearest/FindMaterialExit/FindSmokeExit
   (scene.cpp:773-802).  Returns 0 when the walk leaves the grid. */
static inline int dda_step(dda_t* s, uint32_t n)
{
    if (s->tmax.x < s->tmax.y) {
        if (s->tmax.x < s->tmax.z) {
            s->t = s->tmax.x, s->X += (uint32_t)s->sx;
            if (s->X >= n) return 0;
            s->tmax.x += s->tdelta.x;
        } else {
            s->t = s->tmax.z, s->Z += (uint32_t)s->sz;
            if (s->Z >= n) return 0;
            s->tmax.z += s->tdelta.z;
        }
    } else {
        if (s->tmax.y < s->tmax.z) {
            s->t = s->tmax.y, s->Y += (uint32_t)s->sy;
            if (s->Y >= n) return 0;
            s->tmax.y += s->tdelta.y;
        } else {
            s->t = s->tmax.z, s->Z += (uint32_t)s->sz;
            if (s->Z >= n) return 0;
            s->tmax.z += s->tdelta.z;
        }
    }
    return 1;
}

/* Ray::GetNormalVoxel, template/scene.cpp:121-148 */
static v3 normal_voxel(const ray_t* r, uint32_t n, const float* matrix)
{
    const v3 i1 = vmuls(ray_point(r), (float)n);
    const v3 fg = V3(i1.x - floorf(i1.x), i1.y - floorf(i1.y), i1.z - floorf(i1.z));
    const v3 d = V3(smin(fg.x, 1.0f - fg.x), smin(fg.y, 1.0f - fg.y), smin(fg.z, 1.0f - fg.z));
    const float mind = smin(smin(d.x, d.y), d.z);
    const v3 sign = vsub(vmuls(r->Dsign, 2), V3(1, 1, 1));
    const v3 nn = V3(mind == d.x ? sign.x : 0.0f, mind == d.y ? sign.y : 0.0f, mind == d.z ? sign.z : 0.0f);
    return vnormalize(xform_vec(nn, matrix));
}

/* Scene::FindNearest, template/scene.cpp:751-811 */
static int scene_find_nearest(tctx* c, const vpx_volume* vol, ray_t* r)
{
    const oracle_grid* g = &c->sc->grids[vol->grid_id];
    dda_t s;
    if (!setup_dda(vol, g->n, r, &s)) return 0;
    while (s.t < r->t) {
        const uint8_t cell = grid_at(g, s.X, s.Y, s.Z);
        c->dda_cells++;
        if (cell != NONE_MAT && s.t < r->t) {
            r->t = s.t;
            r->N = normal_voxel(r, g->n, vol->matrix);
            r->mat = cell;
            return 1;
        }
        if (!dda_step(&s, g->n)) break;
    }
    return 0;
}

/* Scene::FindMaterialExit (:875-939) and Scene::FindSmokeExit (:941-1006). */
static int scene_find_exit(tctx* c, const vpx_volume* vol, ray_t* r, int smoke)
{
    const oracle_grid* g = &c->sc->grids[vol->grid_id];
    dda_t s;
    if (!setup_dda(vol, g->n, r, &s)) return 0;
    for (;;) {
        const uint8_t cell = grid_at(g, s.X, s.Y, s.Z);
        c->dda_cells++;
        const int leave = smoke ? (cell > VPX_MAT_SMOKE_PLAYER || cell < VPX_MAT_SMOKE_LOW_DENSITY)
                                : (cell != VPX_MAT_GLASS);
        if (leave) {
            r->t = s.t;
            r->N = normal_voxel(r, g->n, vol->matrix);
            r->mat = cell;
            return 1;
        }
        if (!dda_step(&s, g->n)) break;
    }
    r->t = s.t;
    return 0;
}

/* Scene::IsOccluded, template/scene.cpp:1009-1047 */
static int scene_is_occluded(tctx* c, const vpx_volume* vol, const ray_t* r)
{
    const oracle_grid* g = &c->sc->grids[vol->grid_id];
    const uint32_t n = g->n;
    dda_t s;
    if (!setup_dda(vol, n, r, &s)) return 0;
    while (s.t < r->t) {
        const uint8_t cell = grid_at(g, s.X, s.Y, s.Z);
        c->dda_cells++;
        if (cell != NONE_MAT) return s.t < r->t;
        if (s.tmax.x < s.tmax.y) {
            if (s.tmax.x < s.tmax.z) {
                if ((s.X += (uint32_t)s.sx) >= n) return 0;
                s.t = s.tmax.x, s.tmax.x += s.tdelta.x;
            } else {
                if ((s.Z += (uint32_t)s.sz) >= n) return 0;
                s.t = s.tmax.z, s.tmax.z += s.tdelta.z;
            }
        } else {
            if (s.tmax.y < s.tmax.z) {
                if ((s.Y += (uint32_t)s.sy) >= n) return 0;
                s.t = s.tmax.y, s.tmax.y += s.tdelta.y;
            } else {
                if ((s.Z += (uint32_t)s.sz) >= n) return 0;
                s.t = s.tmax.z, s.tmax.z += s.tdelta.z;
            }
        }
    }
    return 0;
}

/* ------------------------------------------------------------------ analytic -- */
/* Sphere::Hit, src/BVH/Shapes.h:12-42 */
static void sphere_hit(const vpx_sphere* sp, ray_t* r)
{
    const v3 center = v3f(sp->center);
    const v3 to = vsub(r->O, center);
    const float b = vdot(to, r->D);
    const float c = vdot(to, to) - (sp->radius * sp->radius);
    const float disc = b * b - c;
    if (c > 0.0f && b > 0.0f) return;
    if (disc < 0) return;
    const float len = -b - sqrtf(disc);
    if (len > r->t) return;
    if (len < 0) return;
    const v3 ip = vadd(r->O, vmuls(r->D, len));
    const v3 outn = vdivs(vsub(ip, center), sp->radius);
    const int outside = vdot(r->D, outn) < 0;
    r->N = outside ? outn : vneg(outn);
    r->inside = !outside;
    r->t = len;
    r->mat = sp->material;
}

/* Sphere::IsHit, src/BVH/Shapes.h:44-63 */
static int sphere_is_hit(const vpx_sphere* sp, const ray_t* r)
{
    const v3 center = v3f(sp->center);
    const v3 to = vsub(r->O, center);
    const float b = vdot(to, r->D);
    const float c = vdot(to, to) - (sp->radius * sp->radius);
    const float disc = b * b - c;
    if (c > 0.0f && b > 0.0f) return 0;
    if (disc < 0) return 0;
    const float len = -b - sqrtf(disc);
    if (len < 0) return 0;
    if (len > r->t) return 0;
    return 1;
}

/* Triangle::Hit / IsHit, src/BVH/Shapes.h:79-139 (Moller-Trumbore). */
static int tri_core(const vpx_triangle* tr, const ray_t* r, float* tout, v3* e1o, v3* e2o)
{
    const v3 pos = v3f(tr->position);
    const v3 p1 = vadd(pos, v3f(tr->v0)), p2 = vadd(pos, v3f(tr->v1)), p3 = vadd(pos, v3f(tr->v2));
    const v3 e1 = vsub(p2, p1), e2 = vsub(p3, p1);
    const v3 h = vcross(r->D, e2);
    const float a = vdot(e1, h);
    if (a > -0.0001f && a < 0.0001f) return 0;
    const float f = 1 / a;
    const v3 s = vsub(r->O, p1);
    const float u = f * vdot(s, h);
    if (u < 0 || u > 1) return 0;
    const v3 q = vcross(s, e1);
    const float v = f * vdot(r->D, q);
    if (v < 0 || u + v > 1) return 0;
    *tout = f * vdot(e2, q);
    *e1o = e1, *e2o = e2;
    return 1;
}

static void tri_hit(const vpx_triangle* tr, ray_t* r)
{
    float t;
    v3 e1, e2;
    if (!tri_core(tr, r, &t, &e1, &e2)) return;
    if (t > 0.0001f) {
        if (r->t > t) {
            r->t = t;
            r->mat = tr->material;
            const v3 nrm = vnormalize(vcross(e1, e2));
            const int outside = vdot(r->D, nrm) < 0;
            r->N = outside ? nrm : vneg(nrm);
        }
    }
}

static int tri_is_hit(const vpx_triangle* tr, const ray_t* r)
{
    float t;
    v3 e1, e2;
    if (!tri_core(tr, r, &t, &e1, &e2)) return 0;
    if (t < 0.0001f) return 0;
    if (t > r->t) return 0;
    return 1;
}

/* ------------------------------------------------- the reference's x86 approximations -- */
/* Off by default (the build's decision: exact 1/x and 1/sqrtf).  On,
   the restatement uses the reference's own operations where it uses them:
   FastReciprocal (rcpps + one Newton step, renderer.cpp:929-934) for the object-space rD of
   Renderer::FindNearest (:969), and normalize(__m128) = v * rsqrtps(dpps(v, v, 0x7F))
   (tmpl8math.h:2356-2360) for the primary direction of Renderer::Update (:1735-1765, rD
   from the unnormalised D, :1734).  rcpps / rsqrtps are approximations whose bits differ
   between CPU vendors: results hold for the CPU this runs on.  Used only to measure how far
   the exact decision moves the image (tests/test_cpu_oracle.py). */
static int g_x86_approx = 0;
int oracle_set_x86_approx(int on)
{
#ifdef ORACLE_X86
    g_x86_approx = on != 0;
    return 0;
#else
    return on ? -1 : 0;
#endif
}
#ifdef ORACLE_X86
static inline float rcp_approx(float x) { return _mm_cvtss_f32(_mm_rcp_ss(_mm_set_ss(x))); }
static inline float rsqrt_approx(float x) { return _mm_cvtss_f32(_mm_rsqrt_ss(_mm_set_ss(x))); }
static inline float fast_reciprocal1(float x)
{
    const float r = rcp_approx(x);
    const float muls = x * (r * r);
    return (r + r) - muls;
}
static v3 fast_reciprocal(v3 d) { return V3(fast_reciprocal1(d.x), fast_reciprocal1(d.y), fast_reciprocal1(d.z)); }
/* primary ray of the AVX loop: rD = SlowReciprocal(D), D = normalize(D) (rsqrtps), Dsign */
static void primary_rsqrt(ray_t* r, v3 dir)
{
    const float dp = (dir.x * dir.x + dir.y * dir.y) + dir.z * dir.z; /* dpps 0x7F */
    const float inv = rsqrt_approx(dp);
    r->rD = V3(1.0f / dir.x, 1.0f / dir.y, 1.0f / dir.z);
    r->D = V3(dir.x * inv, dir.y * inv, dir.z * inv);
    r->Dsign = compute_dsign(r->D);
}
#endif

/* ------------------------------------------------------------- renderer level -- */
/* Renderer::FindNearest, renderer.cpp:946-1018 */
static int32_t renderer_find_nearest(tctx* c, ray_t* r)
{
    const oracle_scene* sc = c->sc;
    int32_t vox = -2;
    c->nearest_calls++;
    for (uint32_t i = 0; i < sc->num_volumes; i++) {
        const ray_t backup = *r;
        const float* inv = sc->volumes[i].inv_matrix;
        r->O = xform_pos_ssem(backup.O, inv);
        r->D = xform_vec_ssem(backup.D, inv);
        r->rD = V3(1.0f / r->D.x, 1.0f / r->D.y, 1.0f / r->D.z); /* FastReciprocal -> exact */
#ifdef ORACLE_X86
        if (g_x86_approx) r->rD = fast_reciprocal(r->D);
#endif
        r->Dsign = compute_dsign(r->D);
        if (scene_find_nearest(c, &sc->volumes[i], r)) vox = (int32_t)i;
        r->O = backup.O, r->D = backup.D, r->rD = backup.rD, r->Dsign = backup.Dsign;
    }
    if (sc->num_spheres || sc->num_triangles) {
        ray_t sh = make_ray(r->O, r->D);
        for (uint32_t i = 0; i < sc->num_spheres; i++) sphere_hit(&sc->spheres[i], &sh);
        for (uint32_t i = 0; i < sc->num_triangles; i++) tri_hit(&sc->triangles[i], &sh);
        if (r->t > sh.t) {
            r->t = sh.t;
            r->mat = sh.mat;
            r->N = sh.N;
            r->inside = sh.inside;
            vox = -1;
        }
    }
    return vox;
}

/* Renderer::IsOccluded, renderer.cpp:209-243 */
static int renderer_is_occluded(tctx* c, ray_t* r)
{
    const oracle_scene* sc = c->sc;
    for (uint32_t i = 0; i < sc->num_volumes; i++) {
        const ray_t backup = *r;
        const float* inv = sc->volumes[i].inv_matrix;
        r->O = xform_pos(backup.O, inv);
        r->D = xform_vec(backup.D, inv);
        r->rD = V3(1 / r->D.x, 1 / r->D.y, 1 / r->D.z);
        r->Dsign = compute_dsign(r->D);
        const int occ = scene_is_occluded(c, &sc->volumes[i], r);
        r->O = backup.O, r->D = backup.D, r->rD = backup.rD, r->Dsign = backup.Dsign;
        if (occ) return 1;
    }
    for (uint32_t i = 0; i < sc->num_spheres; i++)
        if (sphere_is_hit(&sc->spheres[i], r)) return 1;
    for (uint32_t i = 0; i < sc->num_triangles; i++)
        if (tri_is_hit(&sc->triangles[i], r)) return 1;
    return 0;
}

static int shadow_occluded(tctx* c, ray_t* r)
{
    c->shadow_rays++;
    return renderer_is_occluded(c, r);
}

static inline v3 albedo_of(tctx* c, uint32_t m) { return v3f(c->sc->materials[m].albedo); }
static inline float rf(tctx* c) { return oracle_random_float(&c->rng); }

/* RandomDirection, template/tmpl8math.cpp:76-93 (positive octant only) */
static v3 random_direction(tctx* c)
{
    for (;;) {
        const float a = rf(c), b = rf(c), d = rf(c); /* brace-init: left to right */
        const v3 p = V3(a, b, d);
        if (vdot(p, p) < 1) return vnormalize(p);
    }
}

/* RandomSphereSample, template/tmpl8math.h:2502-2511 */
static v3 random_sphere_sample(tctx* c)
{
    const float theta = rf(c) * 2 * PI_F;
    const float phi = rf(c) * PI_F;
    const float r = rf(c);
    const float x = r * cr_sinf(phi) * cr_cosf(theta);
    const float y = r * cr_sinf(phi) * cr_sinf(theta);
    const float z = r * cr_cosf(phi);
    return V3(x, y, z);
}

/* DiffuseReflection, template/tmpl8math.h:2518-2528 (argument order: left to right) */
static v3 diffuse_reflection(tctx* c, v3 n)
{
    v3 r;
    do {
        const float a = rf(c) * 2 - 1;
        const float b = rf(c) * 2 - 1;
        const float d = rf(c) * 2 - 1;
        r = V3(a, b, d);
    } while (vdot(r, r) > 1);
    if (vdot(r, n) < 0) r = vmuls(r, -1.0f);
    return vnormalize(r);
}

/* Renderer::Reflect / Refract, renderer.cpp:913-925 */
static inline v3 reflect(v3 d, v3 n) { return vsub(d, vmuls(vmuls(n, 2.0f), vdot(n, d))); }
static inline v3 refract(v3 d, v3 n, float ratio)
{
    const float cos_t = smin(vdot(vneg(d), n), 1.0f);
    const v3 rper = vmuls(vadd(d, vmuls(n, cos_t)), ratio);
    const v3 rpar = vmuls(n, -sqrtf(fabsf(1.0f - vdot(rper, rper))));
    return vadd(rper, rpar);
}

/* SchlickReflectance (renderer.cpp:1588-1594), SchlickReflectanceNonMetal (:1611-1616) */
static inline float schlick(float cosine, float ior)
{
    float r0 = (1 - ior) / (1 + ior);
    r0 = r0 * r0;
    return r0 + (1 - r0) * cr_pow5f(1 - cosine);
}
static inline float schlick_nonmetal(float cosine)
{
    const float r0 = 0.04f;
    return r0 + (1 - r0) * cr_pow5f(1 - cosine);
}

/* Renderer::Absorption, renderer.cpp:1596-1608 */
static inline v3 absorption(v3 color, float intensity, float dist)
{
    const v3 flipped = vsub(V3(1, 1, 1), color);
    const v3 e = vmuls(flipped, (-dist) * intensity);
    return V3(cr_expf(e.x), cr_expf(e.y), cr_expf(e.z));
}

/* PointLightEvaluate, renderer.cpp:102-131 */
static v3 point_light(tctx* c, const ray_t* r, const vpx_point_light* l)
{
    const v3 ip = ray_point(r);
    const v3 dir = vsub(v3f(l->position), ip);
    const float dst = vlength(dir);
    const v3 dn = vmuls(dir, 1.0f / dst);
    const v3 n = r->N;
    const float cos_t = vdot(dn, n);
    if (cos_t <= 0.0f) return V3(0, 0, 0);
    const v3 li = vmuls(vmuls(v3f(l->color), smax(0.0f, cos_t)), 1.0f / (dst * dst));
    const v3 origin = offset_ray(ip, n);
    const v3 k = albedo_of(c, r->mat);
    ray_t sh = make_ray(origin, dn);
    sh.t = dst;
    if (shadow_occluded(c, &sh)) return V3(0, 0, 0);
    return vmul(li, k);
}

/* SpotLightEvaluate, renderer.cpp:133-159 (no N.L term) */
static v3 spot_light(tctx* c, const ray_t* r, const vpx_spot_light* l)
{
    const v3 ip = ray_point(r);
    const v3 dir = vsub(v3f(l->position), ip);
    const float dst = vlength(dir);
    const v3 dn = vdivs(dir, dst);
    const v3 n = r->N;
    const float cos_t = vdot(dn, v3f(l->direction));
    if (cos_t <= l->angle) return V3(0, 0, 0);
    const float alpha = 1.0f - (1.0f - cos_t) * 1.0f / (1.0f - l->angle);
    const v3 li = vdivs(vmuls(v3f(l->color), smax(0.0f, cos_t)), dst * dst);
    const v3 k = albedo_of(c, r->mat);
    ray_t sh = make_ray(offset_ray(ip, n), dn);
    sh.t = dst;
    if (shadow_occluded(c, &sh)) return V3(0, 0, 0);
    return vmuls(vmul(li, k), alpha);
}

/* AreaLightEvaluation, renderer.cpp:161-207 (PI4 expands textually: *PI*4.0f) */
static v3 area_light(tctx* c, const ray_t* r, const vpx_area_light* l)
{
    const v3 ip = ray_point(r);
    const v3 n = r->N;
    const v3 center = v3f(l->position);
    const float radius = l->radius;
    v3 inc = V3(0, 0, 0);
    const v3 k = albedo_of(c, r->mat);
    const v3 point = offset_ray(ip, n);
    for (int i = 0; i < c->area_samples; i++) {
        v3 rp = random_direction(c);
        rp = vmuls(rp, radius);
        rp = vadd(rp, center);
        const v3 dir = vsub(rp, ip);
        const float dst = vlength(dir);
        const v3 dn = vmuls(dir, 1 / dst);
        const float cos_t = vdot(dn, n);
        if (cos_t <= 0) continue;
        ray_t sh = make_ray(point, dn);
        sh.t = dst;
        if (shadow_occluded(c, &sh)) continue;
        v3 li = vmuls(v3f(l->color), cos_t);
        li = vmuls(li, l->color_multiplier);
        li = vmuls(li, radius * radius);
        li = vmuls(li, PI_F);
        li = vmuls(li, 4.0f);
        li = vdivs(li, dst * dst);
        inc = vadd(inc, li);
    }
    inc = vdivs(inc, (float)c->area_samples);
    return vmul(inc, k);
}

/* DirectionalLightEvaluate, renderer.cpp:315-338 (direction not normalised) */
static v3 dir_light(tctx* c, const ray_t* r, const vpx_dir_light* l)
{
    const v3 ip = ray_point(r);
    const v3 dir = vneg(v3f(l->direction));
    const v3 n = r->N;
    const float cos_t = vdot(dir, n);
    if (cos_t <= 0) return V3(0, 0, 0);
    const v3 li = vmuls(v3f(l->color), smax(0.0f, cos_t));
    const v3 k = albedo_of(c, r->mat);
    ray_t sh = make_ray(offset_ray(ip, n), dir);
    if (shadow_occluded(c, &sh)) return V3(0, 0, 0);
    return vmul(li, k);
}

/* Renderer::Illumination, renderer.cpp:738-764 */
static v3 illumination(tctx* c, const ray_t* r)
{
    const oracle_scene* sc = c->sc;
    const uint64_t pc = sc->num_points, sc_ = sc->num_spots, ac = sc->num_areas;
    const uint64_t light_count = pc + sc_ + ac + 1;
    const float rnd = rf(c) * (float)light_count;
    const uint64_t idx = (uint64_t)rnd;
    v3 inc;
    if (idx < pc)
        inc = point_light(c, r, &sc->points[idx]);
    else if (idx < ac + pc)
        inc = area_light(c, r, &sc->areas[idx - pc]);
    else if (idx < ac + sc_ + pc)
        inc = spot_light(c, r, &sc->spots[idx - ac - pc]);
    else
        inc = dir_light(c, r, &sc->dir);
    return vmuls(inc, (float)light_count);
}

/* Object-space helper of the glass/smoke branches (renderer.cpp:1160-1173, 1266-1279). */
static int exit_march(tctx* c, ray_t* r, int32_t vox, int smoke)
{
    const vpx_volume* vol = &c->sc->volumes[vox];
    const ray_t backup = *r;
    r->O = xform_pos(backup.O, vol->inv_matrix);
    r->D = xform_vec(backup.D, vol->inv_matrix);
    r->rD = V3(1 / r->D.x, 1 / r->D.y, 1 / r->D.z);
    r->Dsign = compute_dsign(r->D);
    const int res = scene_find_exit(c, vol, r, smoke);
    r->O = backup.O, r->D = backup.D, r->rD = backup.rD, r->Dsign = backup.Dsign;
    return res;
}

/* Renderer::Trace, renderer.cpp:1076-1328 */
static v3 trace(tctx* c, ray_t* r, int depth)
{
    if (depth < 0) return V3(0, 0, 0);
    const int32_t vox = renderer_find_nearest(c, r);
    if (r->mat == NONE_MAT) return sample_sky(c, r->D); /* SampleSky :1092-1095 */
    const vpx_material* mat = &c->sc->materials[r->mat];
    switch (r->mat) {
    case 5: case 6: case 7: { /* metals :1103-1114 */
        const v3 refl = reflect(r->D, r->N);
        const v3 o = offset_ray(ray_point(r), r->N);
        const v3 d = vadd(refl, vmuls(random_sphere_sample(c), mat->roughness));
        ray_t nr = make_ray(o, d);
        return vmul(trace(c, &nr, depth - 1), albedo_of(c, r->mat));
    }
    case 0: case 4: case 1: case 2: case 3: { /* non-metals :1117-1144 */
        v3 color = V3(0, 0, 0);
        if (rf(c) > schlick_nonmetal(vdot(vneg(r->D), r->N))) {
            const v3 rdir = vadd(r->N, random_sphere_sample(c));
            const v3 inc = illumination(c, r);
            ray_t nr = make_ray(offset_ray(ray_point(r), r->N), rdir);
            color = vadd(color, inc);
            color = vadd(color, vmul(trace(c, &nr, depth - 1), albedo_of(c, r->mat)));
        } else {
            const v3 refl = reflect(r->D, r->N);
            const v3 o = offset_ray(ray_point(r), r->N);
            const v3 d = vadd(refl, vmuls(random_sphere_sample(c), mat->roughness));
            ray_t nr = make_ray(o, d);
            color = trace(c, &nr, depth - 1);
        }
        return color;
    }
    case VPX_MAT_GLASS: { /* :1146-1209 */
        v3 color = V3(1, 1, 1);
        int in_glass = r->inside;
        const float ior = mat->ior;
        const float ratio = in_glass ? ior : 1.0f / ior;
        int inside_volume = 1;
        if (in_glass) {
            color = albedo_of(c, r->mat);
            if (vox >= 0) inside_volume = exit_march(c, r, vox, 0); /* vox < 0: UB guard */
        }
        if (!inside_volume) {
            r->O = vadd(r->O, vmuls(r->D, r->t));
            r->t = 0;
        }
        const float cos_t = smin(vdot(vneg(r->D), r->N), 1.0f);
        const float sin_t = sqrtf(1.0f - cos_t * cos_t);
        const int cannot = ratio * sin_t > 1.0f;
        v3 rdir, rn;
        if (cannot || schlick(cos_t, ratio) > rf(c)) {
            rdir = reflect(r->D, r->N);
            rn = r->N;
        } else {
            rdir = refract(r->D, r->N, ratio);
            in_glass = !in_glass;
            rn = vneg(r->N);
        }
        ray_t nr = make_ray(offset_ray(ray_point(r), rn), rdir);
        nr.inside = in_glass;
        return vmul(trace(c, &nr, depth - 1), color);
    }
    case 9: case 10: case 11: case 12: case 13: case 14: { /* smoke :1210-1314 */
        v3 color = V3(1, 1, 1);
        int in_glass = r->inside;
        const float ratio = 1.0f;
        int inside_volume = 1;
        float intensity = 0, dist = 0;
        if (vox == 0) (void)illumination(c, r); /* player light probe :1228-1240 */
        if (in_glass) {
            intensity = mat->emissive;
            color = albedo_of(c, r->mat);
            if (vox >= 0) inside_volume = exit_march(c, r, vox, 1);
            dist = r->t;
        }
        const float threshold = rf(c) * 100 - intensity;
        if (rf(c) * dist > threshold) {
            const float lo = r->t * .45f, hi = r->t;
            const float tt = lo + rf(c) * (hi - lo); /* Rand(min, max), tmpl8math.cpp:154 */
            r->O = vadd(r->O, vmuls(r->D, tt));
            r->D = random_direction(c);
            r->t = 0;
        }
        color = absorption(color, intensity, dist);
        if (!inside_volume) {
            r->O = vadd(r->O, vmuls(r->D, r->t));
            r->t = 0;
        }
        const v3 rdir = refract(r->D, r->N, ratio);
        in_glass = !in_glass;
        const v3 rn = vneg(r->N);
        ray_t nr = make_ray(offset_ray(ray_point(r), rn), rdir);
        nr.inside = in_glass;
        return vmul(trace(c, &nr, depth - 1), color);
    }
    case VPX_MAT_EMISSIVE: /* :1315-1316 */
        return vmuls(albedo_of(c, r->mat), mat->emissive);
    default: { /* model materials :1319-1326 */
        const v3 rdir = diffuse_reflection(c, r->N);
        const v3 inc = illumination(c, r);
        ray_t nr = make_ray(offset_ray(ray_point(r), r->N), rdir);
        return vmul(vadd(trace(c, &nr, depth - 1), inc), albedo_of(c, r->mat));
    }
    }
}

/* ------------------------------------------------------------------ FTZ/DAZ -- */
typedef struct { unsigned int csr; } fpstate;
static inline fpstate fp_enter(void)
{
    fpstate s = {0};
#ifdef ORACLE_X86
    s.csr = _mm_getcsr();
    _mm_setcsr(s.csr | 0x8040u); /* FTZ | DAZ, template/template.cpp:130 */
#endif
    return s;
}
static inline void fp_leave(fpstate s)
{
#ifdef ORACLE_X86
    _mm_setcsr(s.csr);
#else
    (void)s;
#endif
}

static ray_t ray_from_api(const vpx_ray* in)
{
    ray_t r = make_ray(v3f(in->origin), v3f(in->direction));
    r.t = in->tmax;
    r.inside = in->inside_glass ? 1 : 0;
    return r;
}

static void tctx_init(tctx* c, const oracle_scene* sc)
{
    memset(c, 0, sizeof(*c));
    c->sc = sc;
    c->sky[0] = 0.392f, c->sky[1] = 0.584f, c->sky[2] = 0.829f;
    c->area_samples = 3;
}

/* ------------------------------------------------------------ known-answer hooks -- */
/* Single reference functions evaluated on given inputs, for the hand-derived known-answer
   tests (tests/test_kat_reference.py).  Ray built with the Ray ctor (normalised D, Dsign). */
int oracle_kat_normal(const float o[3], const float d[3], float t, uint32_t n, const float m[16], float out[3])
{
    const fpstate fs = fp_enter();
    ray_t r = make_ray(v3f(o), v3f(d));
    r.t = t;
    const v3 v = normal_voxel(&r, n, m);
    out[0] = v.x, out[1] = v.y, out[2] = v.z;
    fp_leave(fs);
    return VPX_OK;
}

/* One light evaluator (kind 0 point, 1 spot, 2 area, 3 directional; light `index` of that
   kind in sc) at the hit O + t*D with normal N on material `mat`; the IsOccluded calls run
   against sc.  *rng is the xorshift32 state (area samples draw from it). */
int oracle_kat_light(const oracle_scene* sc, int kind, uint32_t index, const float o[3], const float d[3], float t,
                     const float nrm[3], uint32_t mat, int32_t area_samples, uint32_t* rng, float out[3])
{
    if (!sc || !rng) return VPX_E_INVALID;
    const fpstate fs = fp_enter();
    tctx c;
    tctx_init(&c, sc);
    c.area_samples = area_samples;
    c.rng = *rng;
    ray_t r = make_ray(v3f(o), v3f(d));
    r.t = t;
    r.N = v3f(nrm);
    r.mat = (uint8_t)mat;
    v3 v = V3(0, 0, 0);
    if (kind == 0) v = point_light(&c, &r, &sc->points[index]);
    else if (kind == 1) v = spot_light(&c, &r, &sc->spots[index]);
    else if (kind == 2) v = area_light(&c, &r, &sc->areas[index]);
    else v = dir_light(&c, &r, &sc->dir);
    out[0] = v.x, out[1] = v.y, out[2] = v.z;
    *rng = c.rng;
    fp_leave(fs);
    return VPX_OK;
}

/* fn 0 SchlickReflectance(in0, in1); 1 SchlickReflectanceNonMetal(in0); 2 Refract(in0..2,
   in3..5, in6); 3 Absorption(in0..2, in3, in4); 4 Reflect(in0..2, in3..5). */
int oracle_kat_shading(int fn, const float* in, float* out)
{
    const fpstate fs = fp_enter();
    v3 v;
    switch (fn) {
    case 0: out[0] = schlick(in[0], in[1]); break;
    case 1: out[0] = schlick_nonmetal(in[0]); break;
    case 2: v = refract(V3(in[0], in[1], in[2]), V3(in[3], in[4], in[5]), in[6]);
            out[0] = v.x, out[1] = v.y, out[2] = v.z; break;
    case 3: v = absorption(V3(in[0], in[1], in[2]), in[3], in[4]);
            out[0] = v.x, out[1] = v.y, out[2] = v.z; break;
    case 4: v = reflect(V3(in[0], in[1], in[2]), V3(in[3], in[4], in[5]));
            out[0] = v.x, out[1] = v.y, out[2] = v.z; break;
    default: fp_leave(fs); return VPX_E_INVALID;
    }
    fp_leave(fs);
    return VPX_OK;
}

int oracle_find_nearest(const oracle_scene* sc, const vpx_ray* rays, uint32_t n, vpx_hit* hits)
{
    if (!sc || (!rays && n) || (!hits && n)) return VPX_E_INVALID;
    const fpstate fs = fp_enter();
    tctx c;
    tctx_init(&c, sc);
    for (uint32_t i = 0; i < n; i++) {
        ray_t r = ray_from_api(&rays[i]);
        const uint64_t before = c.dda_cells;
        const int32_t vox = renderer_find_nearest(&c, &r);
        hits[i].t = r.t;
        hits[i].normal[0] = r.N.x, hits[i].normal[1] = r.N.y, hits[i].normal[2] = r.N.z;
        hits[i].vox_index = vox;
        hits[i].material = r.mat;
        hits[i].cells = (uint32_t)(c.dda_cells - before);
        hits[i].inside_glass = (uint32_t)r.inside;
    }
    fp_leave(fs);
    return VPX_OK;
}

int oracle_is_occluded(const oracle_scene* sc, const vpx_ray* rays, uint32_t n, uint8_t* occluded,
                       uint32_t* cells)
{
    if (!sc || (!rays && n) || (!occluded && n)) return VPX_E_INVALID;
    const fpstate fs = fp_enter();
    tctx c;
    tctx_init(&c, sc);
    for (uint32_t i = 0; i < n; i++) {
        ray_t r = ray_from_api(&rays[i]);
        const uint64_t before = c.dda_cells;
        occluded[i] = (uint8_t)renderer_is_occluded(&c, &r);
        if (cells) cells[i] = (uint32_t)(c.dda_cells - before);
    }
    fp_leave(fs);
    return VPX_OK;
}

int oracle_trace(const oracle_scene* sc, const vpx_ray* rays, const uint32_t* seeds, uint32_t n,
                 int32_t depth, const float sky[3], int32_t area_samples, float* radiance,
                 vpx_stats* stats)
{
    if (!sc || (!rays && n) || (!seeds && n) || (!radiance && n)) return VPX_E_INVALID;
    if (!sky && !sc->sky_pixels) return VPX_E_STATE;
    const fpstate fs = fp_enter();
    tctx c;
    tctx_init(&c, sc);
    if (sky) c.sky[0] = sky[0], c.sky[1] = sky[1], c.sky[2] = sky[2];
    c.sky_tex = sky == NULL;
    c.area_samples = area_samples;
    for (uint32_t i = 0; i < n; i++) {
        ray_t r = ray_from_api(&rays[i]);
        c.rng = seeds[i];
        const v3 v = trace(&c, &r, depth);
        radiance[3 * i] = v.x, radiance[3 * i + 1] = v.y, radiance[3 * i + 2] = v.z;
    }
    if (stats) {
        memset(stats, 0, sizeof(*stats));
        stats->primary_rays = n;
        stats->shadow_rays = c.shadow_rays;
        stats->bounce_rays = c.nearest_calls - (c.nearest_calls ? n : 0);
        stats->dda_cells = c.dda_cells;
    }
    fp_leave(fs);
    return VPX_OK;
}

/* ------------------------------------------------------------------- pixels -- */
/* Primary ray: Camera::GetPrimaryRayNoDOF (camera.h:103-110) or GetPrimaryRay with the
   thin-lens jitter (camera.h:68-83) when VPX_FLAG_DOF; sub-pixel jitter as the AVX path
   computes it, fma(rand, aa, x) (renderer.cpp:1699-1708).  The primary D is normalised
   exactly (the reference's _mm_rsqrt_ps normalize is vendor-specific).
   Per-pixel stream order: [AA: rx, ry] [DOF: r, theta] then Trace. */
static v3 pixel_sample(tctx* c, const vpx_frame_params* p, uint32_t x, uint32_t y)
{
    const vpx_camera* cam = &c->sc->camera;
    c->rng = oracle_pixel_seed(p->seed_base, p->frame_index, p->width, p->height, x, y);
    float fx = (float)x, fy = (float)y;
    if (p->flags & VPX_FLAG_AA) {
        const float rx = rf(c), ry = rf(c);
        fx = fmaf(rx, p->aa_strength, fx);
        fy = fmaf(ry, p->aa_strength, fy);
    }
    const float u = fx * (1.0f / (float)p->width);
    const float v = fy * (1.0f / (float)p->height);
    const v3 tl = v3f(cam->top_left), tr = v3f(cam->top_right), bl = v3f(cam->bottom_left);
    const v3 P = vadd(vadd(tl, vmuls(vsub(tr, tl), u)), vmuls(vsub(bl, tl), v));
    const v3 cp = v3f(cam->cam_pos);
    ray_t r;
    if (p->flags & VPX_FLAG_DOF) {
        const float rr = sqrtf(rf(c));
        const float theta = rf(c) * (2 * PI_F);
        const float cx = cr_cosf(theta) * rr, cy = cr_sinf(theta) * rr;
        const float jx = cx * cam->defocus_jitter / (float)p->width;
        const float jy = cy * cam->defocus_jitter / (float)p->width;
        const v3 focal = vadd(cp, vmuls(vnormalize(vsub(P, cp)), cam->focal_distance));
        const v3 o = vadd(vadd(cp, vmuls(v3f(cam->right), jx)), vmuls(v3f(cam->up), jy));
        r = make_ray(o, vsub(focal, o));
#ifdef ORACLE_X86
        if (g_x86_approx) primary_rsqrt(&r, vsub(focal, o));
#endif
    } else {
        r = make_ray(cp, vsub(P, cp));
#ifdef ORACLE_X86
        if (g_x86_approx) primary_rsqrt(&r, vsub(P, cp));
#endif
    }
    return trace(c, &r, p->max_bounces);
}

/* GetLuminance (renderer.cpp:2237-2240), ApplyReinhardJodie (:2222-2234),
   RGBF32_to_RGB8 (template/precomp.h:372-388), lerp (tmpl8math.h:2210-2213). */
static uint32_t tonemap_pack(const float* acc)
{
    const v3 col = V3(acc[0], acc[1], acc[2]);
    const float lum = vdot(col, V3(0.2126f, 0.7152f, 0.0722f));
    const v3 rh = vdiv(col, V3(1.0f + col.x, 1.0f + col.y, 1.0f + col.z));
    const v3 la = vdivs(col, 1.0f + lum);
    const float o[3] = {la.x + rh.x * (rh.x - la.x), la.y + rh.y * (rh.y - la.y), la.z + rh.z * (rh.z - la.z)};
    const uint32_t r = (uint32_t)(int64_t)(255.0f * smin(1.0f, o[0]));
    const uint32_t g = (uint32_t)(int64_t)(255.0f * smin(1.0f, o[1]));
    const uint32_t b = (uint32_t)(int64_t)(255.0f * smin(1.0f, o[2]));
    return (r << 16) + (g << 8) + b;
}

/* Accumulator blend of the AVX path: acc = fma(1-w, acc, px*w) (renderer.cpp:1797-1828). */
void oracle_accumulate_tonemap(const float* s4, uint32_t frame_index, float* acc4, uint32_t* rgb8)
{
    const fpstate fs = fp_enter();
    const float w = 1.0f / ((float)frame_index + 1.0f);
    const float iw = 1.0f - w;
    for (int k = 0; k < 4; k++) acc4[k] = fmaf(iw, acc4[k], s4[k] * w);
    if (rgb8) *rgb8 = tonemap_pack(acc4);
    fp_leave(fs);
}

typedef struct {
    const oracle_scene* sc;
    const vpx_frame_params* p;
    const uint32_t* ids;
    uint32_t n;
    float* out4;
    float* accum;
    uint32_t* rgb8;
    uint32_t tid, nthreads;
    uint64_t shadow, nearest, cells;
} job_t;

static void* render_worker(void* arg)
{
    job_t* j = (job_t*)arg;
    const fpstate fs = fp_enter();
    tctx c;
    tctx_init(&c, j->sc);
    c.sky[0] = j->p->sky[0], c.sky[1] = j->p->sky[1], c.sky[2] = j->p->sky[2];
    c.sky_tex = (j->p->flags & VPX_FLAG_SKY) && j->sc->sky_pixels;
    c.area_samples = j->p->area_samples;
    const uint32_t W = j->p->width;
    const float w = 1.0f / ((float)j->p->frame_index + 1.0f);
    const float iw = 1.0f - w;
    for (uint32_t i = j->tid; i < j->n; i += j->nthreads) {
        const uint32_t id = j->ids ? j->ids[i] : i;
        const v3 v = pixel_sample(&c, j->p, id % W, id / W);
        if (j->out4) {
            float* o = j->out4 + 4 * (uint64_t)i;
            o[0] = v.x, o[1] = v.y, o[2] = v.z, o[3] = 0.0f;
        }
        if (j->accum) {
            float* a = j->accum + 4 * (uint64_t)id;
            const float s[4] = {v.x, v.y, v.z, 0.0f};
            for (int k = 0; k < 4; k++) a[k] = fmaf(iw, a[k], s[k] * w);
            if (j->rgb8) j->rgb8[id] = tonemap_pack(a);
        }
    }
    j->shadow = c.shadow_rays, j->nearest = c.nearest_calls, j->cells = c.dda_cells;
    fp_leave(fs);
    return NULL;
}

static int run_jobs(const oracle_scene* sc, const vpx_frame_params* p, const uint32_t* ids,
                    uint32_t n, float* out4, float* accum, uint32_t* rgb8, vpx_stats* stats,
                    int threads)
{
    if (threads <= 0) {
        const long hc = sysconf(_SC_NPROCESSORS_ONLN);
        threads = hc > 0 ? (int)hc : 1;
    }
    if (threads > 256) threads = 256;
    job_t jobs[256];
    pthread_t th[256];
    for (int t = 0; t < threads; t++) {
        jobs[t] = (job_t){sc, p, ids, n, out4, accum, rgb8, (uint32_t)t, (uint32_t)threads, 0, 0, 0};
    }
    int started = 0;
    for (int t = 1; t < threads; t++) {
        if (pthread_create(&th[t], NULL, render_worker, &jobs[t]) != 0) break;
        started = t;
    }
    if (started < threads - 1) { /* could not start all: run the rest inline */
        for (int t = started + 1; t < threads; t++) render_worker(&jobs[t]);
    }
    render_worker(&jobs[0]);
    for (int t = 1; t <= started; t++) pthread_join(th[t], NULL);
    if (stats) {
        memset(stats, 0, sizeof(*stats));
        stats->primary_rays = n;
        for (int t = 0; t < threads; t++) {
            stats->shadow_rays += jobs[t].shadow;
            stats->bounce_rays += jobs[t].nearest;
            stats->dda_cells += jobs[t].cells;
        }
        /* Trace(ray, -1) makes no FindNearest call: no bounce rays (not a negative count) */
        stats->bounce_rays = stats->bounce_rays > n ? stats->bounce_rays - n : 0;
    }
    return VPX_OK;
}

int oracle_render_pixels(const oracle_scene* sc, const vpx_frame_params* p, const uint32_t* ids,
                         uint32_t n, float* sample4, vpx_stats* stats, int threads)
{
    if (!sc || !p || !sample4 || (!ids && n)) return VPX_E_INVALID;
    return run_jobs(sc, p, ids, n, sample4, NULL, NULL, stats, threads);
}

int oracle_render(const oracle_scene* sc, const vpx_frame_params* p, float* accum, uint32_t* rgb8,
                  vpx_stats* stats, int threads)
{
    if (!sc || !p || !accum) return VPX_E_INVALID;
    return run_jobs(sc, p, NULL, p->width * p->height, NULL, accum, rgb8, stats, threads);
}

/* ------------------------------------------------- static-camera path -- */
typedef struct { v3 albedo, illum; } aidata; /* AlbedoIlluminationData, renderer.h:10-19 */
static inline v3 ai_color(aidata a) { return vmul(a.albedo, a.illum); } /* GetColor */

/* Renderer::TraceReproject and its helpers, renderer.cpp:1330-1585 (SampleSkyReproject
   :2328-2333 with activateSky == false returns {sky, 1}). */
static aidata trace_reproject(tctx* c, ray_t* r, int depth)
{
    aidata out;
    if (depth < 0) {
        out.albedo = V3(0, 0, 0), out.illum = V3(0, 0, 0);
        return out;
    }
    const int32_t vox = renderer_find_nearest(c, r);
    if (r->mat == NONE_MAT) {
        out.albedo = sample_sky(c, r->D), out.illum = V3(1, 1, 1); /* SampleSkyReproject :2328-2346 */
        return out;
    }
    const vpx_material* mat = &c->sc->materials[r->mat];
    switch (r->mat) {
    case 5: case 6: case 7: { /* TraceMetal :1330-1340 */
        const v3 refl = reflect(r->D, r->N);
        const v3 o = offset_ray(ray_point(r), r->N);
        const v3 d = vadd(refl, vmuls(random_sphere_sample(c), mat->roughness));
        ray_t nr = make_ray(o, d);
        out.illum = ai_color(trace_reproject(c, &nr, depth - 1));
        out.albedo = albedo_of(c, r->mat);
        return out;
    }
    case 0: case 1: case 2: case 3: case 4: { /* TraceNonMetal :1342-1357 */
        const v3 rdir = vadd(r->N, random_sphere_sample(c)); /* RandomLambertianReflectionVector */
        const v3 inc = illumination(c, r);
        ray_t nr = make_ray(offset_ray(ray_point(r), r->N), rdir);
        v3 il = V3(0, 0, 0);
        il = vadd(il, inc);
        il = vadd(il, ai_color(trace_reproject(c, &nr, depth - 1)));
        out.albedo = albedo_of(c, r->mat), out.illum = il;
        return out;
    }
    case VPX_MAT_GLASS: { /* TraceDialectric :1359-1421 */
        v3 color = V3(1, 1, 1);
        int in_glass = r->inside;
        const float ior = mat->ior;
        const float ratio = in_glass ? ior : 1.0f / ior;
        int inside_volume = 1;
        if (in_glass) {
            color = albedo_of(c, r->mat);
            if (vox >= 0) inside_volume = exit_march(c, r, vox, 0);
        }
        if (!inside_volume) {
            r->O = vadd(r->O, vmuls(r->D, r->t));
            r->t = 0;
        }
        const float cos_t = smin(vdot(vneg(r->D), r->N), 1.0f);
        const float sin_t = sqrtf(1.0f - cos_t * cos_t);
        const int cannot = ratio * sin_t > 1.0f;
        v3 rdir, rn;
        if (cannot || schlick(cos_t, ratio) > rf(c)) {
            rdir = reflect(r->D, r->N);
            rn = r->N;
        } else {
            rdir = refract(r->D, r->N, ratio);
            in_glass = !in_glass;
            rn = vneg(r->N);
        }
        ray_t nr = make_ray(offset_ray(ray_point(r), rn), rdir);
        nr.inside = in_glass;
        out.albedo = color, out.illum = ai_color(trace_reproject(c, &nr, depth - 1));
        return out;
    }
    case 9: case 10: case 11: case 12: case 13: case 14: { /* TraceSmoke :1423-1494 */
        v3 color = V3(1, 1, 1);
        int in_glass = r->inside;
        int inside_volume = 1;
        float intensity = 0, dist = 0;
        if (vox == 0) (void)illumination(c, r); /* player probe: only the inLight flag uses it */
        if (in_glass) {
            intensity = mat->emissive;
            color = albedo_of(c, r->mat);
            if (vox >= 0) inside_volume = exit_march(c, r, vox, 1);
            dist = r->t;
        }
        const float threshold = rf(c) * 100 - intensity;
        if (rf(c) * dist > threshold) {
            const float lo = r->t * .45f, hi = r->t;
            const float tt = lo + rf(c) * (hi - lo);
            r->O = vadd(r->O, vmuls(r->D, tt));
            r->D = random_direction(c);
            r->t = 0;
        }
        color = absorption(color, intensity, dist);
        if (!inside_volume) {
            r->O = vadd(r->O, vmuls(r->D, r->t));
            r->t = 0;
        }
        const v3 rdir = refract(r->D, r->N, 1.0f);
        in_glass = !in_glass;
        ray_t nr = make_ray(offset_ray(ray_point(r), vneg(r->N)), rdir);
        nr.inside = in_glass;
        out.albedo = color, out.illum = ai_color(trace_reproject(c, &nr, depth - 1));
        return out;
    }
    case VPX_MAT_EMISSIVE: /* TraceEmmision :1496-1499 */
        out.albedo = vmuls(albedo_of(c, r->mat), mat->emissive), out.illum = V3(1, 1, 1);
        return out;
    default: { /* TraceModelMaterials :1501-1511 */
        const v3 rdir = diffuse_reflection(c, r->N);
        const v3 inc = illumination(c, r);
        ray_t nr = make_ray(offset_ray(ray_point(r), r->N), rdir);
        v3 il = inc;
        il = vadd(il, ai_color(trace_reproject(c, &nr, depth - 1)));
        out.albedo = albedo_of(c, r->mat), out.illum = il;
        return out;
    }
    }
}

static inline v3 ycocg(v3 c) /* RGBToYCoCg, renderer.cpp:833-839 */
{
    const float k = 0.5f * 256.0f / 255.0f;
    return V3(vdot(c, V3(1, 2, 1)) * 0.25f, vdot(c, V3(2, 0, -2)) * 0.25f + k, vdot(c, V3(-1, 2, -1)) * 0.25f + k);
}
static inline v3 ycocg_rgb(v3 c) /* YCoCgToRGB, renderer.cpp:842-851 */
{
    const float k = 0.5f * 256.0f / 255.0f;
    const float co = c.y - k, cg = c.z - k;
    return V3(c.x + co - cg, c.x + cg, c.x - co - cg);
}
static inline int on_screen(int x, int y, uint32_t W, uint32_t H) /* IsValidScreen(float2) */
{
    return (float)x >= 0.0f && (float)x < (float)W && (float)y >= 0.0f && (float)y < (float)H;
}

typedef struct {
    const oracle_scene* sc;
    const vpx_frame_params* p;
    const vpx_prev_camera* prev;
    float *alb, *ill, *rd, *hist, *temp;
    uint32_t* rgb8;
    int pass;
    uint32_t tid, nthreads;
    uint64_t shadow, nearest, cells;
} rjob_t;

static void* reproject_worker(void* arg)
{
    rjob_t* j = (rjob_t*)arg;
    const fpstate fs = fp_enter();
    tctx c;
    tctx_init(&c, j->sc);
    c.sky[0] = j->p->sky[0], c.sky[1] = j->p->sky[1], c.sky[2] = j->p->sky[2];
    c.sky_tex = (j->p->flags & VPX_FLAG_SKY) && j->sc->sky_pixels;
    c.area_samples = j->p->area_samples;
    const uint32_t W = j->p->width, H = j->p->height;
    const vpx_camera* cam = &j->sc->camera;
    for (uint32_t i = j->tid; i < W * H; i += j->nthreads) {
        const uint32_t x = i % W, y = i / W;
        if (j->pass == 0) { /* Tick static branch, first loop (renderer.cpp:2001-2022) */
            c.rng = oracle_pixel_seed(j->p->seed_base, j->p->frame_index, W, H, x, y);
            const float u = (float)x * (1.0f / (float)W), v = (float)y * (1.0f / (float)H);
            const v3 tl = v3f(cam->top_left), tr = v3f(cam->top_right), bl = v3f(cam->bottom_left);
            const v3 P = vadd(vadd(tl, vmuls(vsub(tr, tl), u)), vmuls(vsub(bl, tl), v));
            const v3 cp = v3f(cam->cam_pos);
            ray_t r = make_ray(cp, vsub(P, cp)); /* GetPrimaryRayNoDOF */
            const aidata d = trace_reproject(&c, &r, j->p->max_bounces);
            const v3 ip = ray_point(&r); /* RayDataReproject::GetRayInfo */
            float* a = j->alb + 4 * (uint64_t)i;
            float* l = j->ill + 4 * (uint64_t)i;
            float* q = j->rd + 4 * (uint64_t)i;
            a[0] = d.albedo.x, a[1] = d.albedo.y, a[2] = d.albedo.z, a[3] = 0;
            l[0] = d.illum.x, l[1] = d.illum.y, l[2] = d.illum.z, l[3] = 0;
            q[0] = ip.x, q[1] = ip.y, q[2] = ip.z, q[3] = u2f_bits(r.mat);
            continue;
        }
        /* second loop (renderer.cpp:2024-2098) */
        const float* q = j->rd + 4 * (uint64_t)i;
        const v3 P = V3(q[0], q[1], q[2]);
        const uint32_t mt = f2u_bits(q[3]);
        const v3 ns = v3f(j->ill + 4 * (uint64_t)i);
        v3 fin = ns;
        const v3 pc = v3f(j->prev->cam_pos);
        const v3 delta = vsub(P, pc); /* Camera::PointToUV, camera.h:33-49 */
        const float ld = vdot(v3f(j->prev->left_normal), delta), rdd = vdot(v3f(j->prev->right_normal), delta);
        const float td = vdot(v3f(j->prev->top_normal), delta), bd = vdot(v3f(j->prev->bottom_normal), delta);
        const float hw = 1.0f / (float)W / 2.0f, hh = 1.0f / (float)H / 2.0f; /* HALF_PIXEL_W/H */
        const float uu = ld / (ld + rdd) + hw, vv = td / (td + bd) + hh;
        int use = uu >= 0.0f && uu < 1.0f && vv >= 0.0f && vv < 1.0f; /* IsValid */
        if (use) { /* IsOccludedPrevFrame, renderer.cpp:767-774 */
            const v3 dn = vnormalize(vsub(P, pc));
            const v3 pos = offset_ray(P, vneg(dn));
            ray_t occ = make_ray(pc, dn);
            occ.t = vlength(vsub(pos, pc));
            if (shadow_occluded(&c, &occ)) use = 0;
        }
        if (use) {
            /* SampleHistory, renderer.cpp:777-830 */
            const float ux = uu - hw, uy = vv - hh;
            const float ptx = ux * (float)W, pty = uy * (float)H;
            const int tlx = f2i_trunc(ptx), tly = f2i_trunc(pty);
            const float fx = ptx - (float)tlx, fy = pty - (float)tly;
            const float gx = 1 - fx, gy = 1 - fy;
            const int v1 = on_screen(tlx, tly, W, H), v2 = on_screen(tlx + 1, tly, W, H);
            const int v3_ = on_screen(tlx, tly + 1, W, H), v4 = on_screen(tlx + 1, tly + 1, W, H);
            float w1 = v1 ? gx * gy : 0.0f, w2 = v2 ? fx * gy : 0.0f, w3 = v3_ ? gx * fy : 0.0f, w4 = v4 ? fx * fy : 0.0f;
            const float tw = w1 + w2 + w3 + w4;
            const float rtw = 1.0f / tw;
            w1 *= rtw, w2 *= rtw, w3 *= rtw, w4 *= rtw;
            v3 hs = V3(0, 0, 0);
            if (v1) hs = vadd(hs, vmuls(v3f(j->hist + 4 * ((uint64_t)tly * W + tlx)), w1));
            if (v2) hs = vadd(hs, vmuls(v3f(j->hist + 4 * ((uint64_t)tly * W + tlx + 1)), w2));
            if (v3_) hs = vadd(hs, vmuls(v3f(j->hist + 4 * ((uint64_t)(tly + 1) * W + tlx)), w3));
            if (v4) hs = vadd(hs, vmuls(v3f(j->hist + 4 * ((uint64_t)(tly + 1) * W + tlx + 1)), w4));
            /* ClampHistory, renderer.cpp:856-910 */
            const v3 nsy = ycocg(ns);
            v3 hy = ycocg(hs);
            uint32_t nvalid = 1;
            v3 avg = nsy, var = vmul(nsy, nsy);
            static const int ox[8] = {-1, 0, 1, -1, 1, -1, 0, 1}, oy[8] = {-1, -1, -1, 0, 0, 1, 1, 1};
            for (int k = 0; k < 8; k++) {
                const int qx = (int)x + ox[k], qy = (int)y + oy[k];
                if (on_screen(qx, qy, W, H)) {
                    const v3 fe = ycocg(v3f(j->ill + 4 * ((uint64_t)qx + (uint64_t)qy * W)));
                    avg = vadd(avg, fe);
                    var = vadd(var, vmul(fe, fe));
                    nvalid++;
                }
            }
            const float inv = 1.0f / (float)nvalid;
            avg = vmuls(avg, inv), var = vmuls(var, inv);
            const v3 sg = V3(sqrtf(smax(0.0f, var.x - avg.x * avg.x)), sqrtf(smax(0.0f, var.y - avg.y * avg.y)),
                             sqrtf(smax(0.0f, var.z - avg.z * avg.z)));
            const v3 lo = vsub(avg, vmuls(sg, 0.75f)), hi = vadd(avg, vmuls(sg, 0.75f));
            hy = V3(fmaxf(lo.x, fminf(hy.x, hi.x)), fmaxf(lo.y, fminf(hy.y, hi.y)), fmaxf(lo.z, fminf(hy.z, hi.z)));
            v3 hr = ycocg_rgb(hy);
            hr = V3(fmaxf(hr.x, 0.0f), fmaxf(hr.y, 0.0f), fmaxf(hr.z, 0.0f));
            float wt = 0.9f; /* material weights, renderer.cpp:2050-2088 */
            if (mt <= 4) wt = 0.8f;
            else if (mt <= 7) wt = 0.5f;
            else if (mt == VPX_MAT_GLASS) wt = 0.5f;
            else if (mt == VPX_MAT_EMISSIVE) wt = 0.0f;
            fin = vadd(ns, vmuls(vsub(hr, ns), wt)); /* lerp, tmpl8math.h:2220-2223 */
        }
        float* t = j->temp + 4 * (uint64_t)i;
        t[0] = fin.x, t[1] = fin.y, t[2] = fin.z, t[3] = 0;
        if (j->rgb8) {
            const v3 col = vmul(v3f(j->alb + 4 * (uint64_t)i), fin);
            const float px[4] = {col.x, col.y, col.z, 0.0f};
            j->rgb8[i] = tonemap_pack(px);
        }
    }
    j->shadow = c.shadow_rays, j->nearest = c.nearest_calls, j->cells = c.dda_cells;
    fp_leave(fs);
    return NULL;
}

int oracle_render_reproject(const oracle_scene* sc, const vpx_frame_params* p, const vpx_prev_camera* prev,
                            float* history, uint32_t* rgb8, vpx_stats* stats, int threads)
{
    if (!sc || !p || !prev || !history) return VPX_E_INVALID;
    const uint64_t npx = (uint64_t)p->width * p->height;
    float* buf = (float*)malloc(sizeof(float) * 4 * 4 * npx);
    if (!buf) return VPX_E_NOMEM;
    if (threads <= 0) {
        const long hc = sysconf(_SC_NPROCESSORS_ONLN);
        threads = hc > 0 ? (int)hc : 1;
    }
    if (threads > 256) threads = 256;
    rjob_t jobs[256];
    pthread_t th[256];
    if (stats) memset(stats, 0, sizeof(*stats));
    for (int pass = 0; pass < 2; pass++) {
        for (int t = 0; t < threads; t++)
            jobs[t] = (rjob_t){sc, p, prev, buf, buf + 4 * npx, buf + 8 * npx, history, buf + 12 * npx, rgb8,
                               pass, (uint32_t)t, (uint32_t)threads, 0, 0, 0};
        int started = 0;
        for (int t = 1; t < threads; t++) {
            if (pthread_create(&th[t], NULL, reproject_worker, &jobs[t]) != 0) break;
            started = t;
        }
        for (int t = started + 1; t < threads; t++) reproject_worker(&jobs[t]);
        reproject_worker(&jobs[0]);
        for (int t = 1; t <= started; t++) pthread_join(th[t], NULL);
        if (stats)
            for (int t = 0; t < threads; t++) {
                stats->shadow_rays += jobs[t].shadow;
                stats->bounce_rays += jobs[t].nearest;
                stats->dda_cells += jobs[t].cells;
            }
    }
    if (stats) {
        stats->primary_rays = npx;
        stats->bounce_rays -= p->max_bounces >= 0 ? npx : 0;
    }
    memcpy(history, buf + 12 * npx, sizeof(float) * 4 * npx); /* illuminationHistoryBuffer = temp */
    free(buf);
    return VPX_OK;
}

/* Focus ray of Renderer::Tick (renderer.cpp:1987-1991): GetPrimaryRay(W/2, H/2) with DOF
   jitter is not applied here (integer centre, circle drawn from the thread RNG in the
   reference); the ray is tested against every Scene in WORLD space (reference quirk). */
float oracle_focus_distance(const oracle_scene* sc, uint32_t width, uint32_t height)
{
    const fpstate fs = fp_enter();
    tctx c;
    tctx_init(&c, sc);
    const vpx_camera* cam = &sc->camera;
    const float u = (float)(width / 2) * (1.0f / (float)width);
    const float v = (float)(height / 2) * (1.0f / (float)height);
    const v3 tl = v3f(cam->top_left), tr = v3f(cam->top_right), bl = v3f(cam->bottom_left);
    const v3 P = vadd(vadd(tl, vmuls(vsub(tr, tl), u)), vmuls(vsub(bl, tl), v));
    const v3 cp = v3f(cam->cam_pos);
    const v3 focal = vadd(cp, vmuls(vnormalize(vsub(P, cp)), cam->focal_distance));
    ray_t r = make_ray(cp, vsub(focal, cp));
    for (uint32_t i = 0; i < sc->num_volumes; i++) scene_find_nearest(&c, &sc->volumes[i], &r);
    const float t = r.t;
    fp_leave(fs);
    return smax(-1.0f, smin(t, 1e4f)); /* clamp(t, -1, 1e4), tmpl8math.h:2105-2108 */
}

/* -------------------------------------------------------------------- worlds -- */
/* Scene::LoadModel placement, template/scene.cpp:449-529 (ResetGrid() -> NONE first;
   only downscales when size_x > gridsize; y/z swapped; out-of-range writes dropped). */
void oracle_load_model(const uint8_t* vox, uint32_t sx, uint32_t sy, uint32_t sz, uint32_t n,
                       const float scale_model[3], uint8_t* out)
{
    const uint64_t n64 = n;
    memset(out, NONE_MAT, n64 * n64 * n64);
    float scl[3] = {scale_model[0], scale_model[1], scale_model[2]};
    if (sx > n) {
        scl[0] *= (float)n / (float)sx;
        scl[1] *= (float)n / (float)sy;
        scl[2] *= (float)n / (float)sz;
    }
    for (uint32_t z = 0; z < sz; ++z)
        for (uint32_t y = 0; y < sy; ++y)
            for (uint32_t x = 0; x < sx; ++x) {
                const int gx = f2i_trunc((float)x * scl[0]);
                const int gy = f2i_trunc((float)z * scl[1]);
                const int gz = f2i_trunc((float)y * scl[2]);
                const uint8_t c = vox[x + (uint64_t)y * sx + (uint64_t)z * sx * sy];
                if (c == 0) continue;
                if (gx < 0 || gy < 0 || gz < 0 || (uint32_t)gx >= n || (uint32_t)gy >= n || (uint32_t)gz >= n)
                    continue;
                out[(uint64_t)gx + (uint64_t)gy * n64 + (uint64_t)gz * n64 * n64] = c;
            }
}

/* Scene::LoadModelPartial (template/scene.cpp:531-604): ResetGrid() to NONE, the
   LoadModel scale rule, then only voxels with x in [columns - thickness, columns +
   thickness] (uint32 arithmetic, as written: the lower bound wraps when thickness >
   columns).  Writes outside the grid are skipped (the reference's Set does not check). */
void oracle_load_model_partial(const uint8_t* vox, uint32_t sx, uint32_t sy, uint32_t sz, uint32_t n,
                               const float scale_model[3], uint32_t columns, uint32_t thickness, uint8_t* out)
{
    const uint64_t n64 = n;
    memset(out, NONE_MAT, n64 * n64 * n64);
    float scl[3] = {scale_model[0], scale_model[1], scale_model[2]};
    if (sx > n) {
        scl[0] *= (float)n / (float)sx;
        scl[1] *= (float)n / (float)sy;
        scl[2] *= (float)n / (float)sz;
    }
    const uint32_t lo = columns - thickness, hi = columns + thickness;
    for (uint32_t z = 0; z < sz; ++z)
        for (uint32_t y = 0; y < sy; ++y)
            for (uint32_t x = 0; x < sx; ++x) {
                const int gx = f2i_trunc((float)x * scl[0]);
                const int gy = f2i_trunc((float)z * scl[1]);
                const int gz = f2i_trunc((float)y * scl[2]);
                const uint8_t c = vox[x + (uint64_t)y * sx + (uint64_t)z * sx * sy];
                if (c == 0 || !(x >= lo && x <= hi)) continue;
                if (gx < 0 || gy < 0 || gz < 0 || (uint32_t)gx >= n || (uint32_t)gy >= n || (uint32_t)gz >= n)
                    continue;
                out[(uint64_t)gx + (uint64_t)gy * n64 + (uint64_t)gz * n64 * n64] = c;
            }
}

/* Scene::CreateEmmisiveSphere (template/scene.cpp:685-711), worldsize = n. */
void oracle_emissive_sphere(uint8_t* grid, uint32_t n, uint8_t mat, float radius)
{
    const uint64_t n64 = n;
    const float c = (float)n / 2.0f;
    for (uint32_t z = 0; z < n; ++z)
        for (uint32_t y = 0; y < n; ++y)
            for (uint32_t x = 0; x < n; ++x) {
                const float vx = c - (float)x, vy = c - (float)y, vz = c - (float)z;
                const float d = sqrtf(vx * vx + vy * vy + vz * vz);
                if (d < radius) grid[x + (uint64_t)y * n64 + (uint64_t)z * n64 * n64] = mat;
            }
}

void oracle_orient_model(const uint8_t* vox, uint32_t sx, uint32_t sy, uint32_t sz, uint8_t* out)
{
    /* grid-oriented dims: gx = sx, gy = sz, gz = sy */
    for (uint32_t z = 0; z < sz; ++z)
        for (uint32_t y = 0; y < sy; ++y)
            for (uint32_t x = 0; x < sx; ++x) {
                const uint8_t c = vox[x + (uint64_t)y * sx + (uint64_t)z * sx * sy];
                out[x + (uint64_t)z * sx + (uint64_t)y * sx * sz] = c ? c : (uint8_t)NONE_MAT;
            }
}

void oracle_tiled_world(const uint8_t* model, uint32_t mx, uint32_t my, uint32_t mz, uint32_t px,
                        uint32_t py, uint32_t pz, uint32_t ground, uint32_t n, uint8_t* out)
{
    const uint64_t n64 = n;
    for (uint64_t z = 0; z < n64; z++)
        for (uint64_t y = 0; y < n64; y++) {
            uint8_t* row = out + y * n64 + z * n64 * n64;
            if (y < ground) {
                memset(row, VPX_MAT_NON_METAL_WHITE, n64);
                continue;
            }
            const uint64_t ly = (y - ground) % py, lz = z % pz;
            for (uint64_t x = 0; x < n64; x++) {
                const uint64_t lx = x % px;
                row[x] = (lx < mx && ly < my && lz < mz) ? model[lx + ly * mx + lz * mx * my] : (uint8_t)NONE_MAT;
            }
        }
}

/* Order-independent checksum: sum_i (cell_i + 1) * splitmix64(i)  (mod 2^64). */
static inline uint64_t splitmix64(uint64_t x)
{
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

uint64_t oracle_grid_checksum(const uint8_t* cells, uint64_t count)
{
    uint64_t s = 0;
    for (uint64_t i = 0; i < count; i++) s += (uint64_t)(cells[i] + 1u) * splitmix64(i);
    return s;
}

/* ------------------------------------------------------------------ BasicBVH -- */
/* src/BVH/BasicBVH.{h,cpp}: the reference's triangle BVH (jacco.ompf2.com tutorial, part
   1).  A Renderer member (renderer.h:220) that Trace never calls;
   restated for the vpx_bvh_* entry points. */

/* BasicBVH::BasicBVH() (BasicBVH.cpp:4-16): 64 triangles from RandomFloat.  The three
   RandomFloat() arguments of each float3 constructor are drawn left to right (C++ leaves
   the order unspecified — the same hazard as Update's RNG). */
uint32_t oracle_bvh_random_tris(uint32_t seed, vpx_bvh_tri* out)
{
    for (int i = 0; i < 64; ++i) {
        float r[9];
        for (int k = 0; k < 9; ++k) r[k] = oracle_random_float(&seed);
        const v3 r0 = V3(r[0], r[1], r[2]), r1 = V3(r[3], r[4], r[5]), r2 = V3(r[6], r[7], r[8]);
        const v3 a = vsub(vmuls(r0, 9.0f), V3(5.0f, 5.0f, 5.0f)); /* r0 * 9 - float3(5) */
        const v3 b = vadd(a, r1), c = vadd(a, r2);
        out[i].v0[0] = a.x, out[i].v0[1] = a.y, out[i].v0[2] = a.z;
        out[i].v1[0] = b.x, out[i].v1[1] = b.y, out[i].v1[2] = b.z;
        out[i].v2[0] = c.x, out[i].v2[1] = c.y, out[i].v2[2] = c.z;
    }
    return seed;
}

typedef struct {
    const vpx_bvh_tri* tri;
    v3* centroid;
    uint32_t* idx;
    vpx_bvh_node* node;
    uint32_t used;
} bvh_build_t;

static inline float fminf_t(float a, float b) { return a < b ? a : b; } /* tmpl8math.h:401-404 */
static inline float fmaxf_t(float a, float b) { return a > b ? a : b; } /* :406-409 */

/* BasicBVH::UpdateNodeBounds, BasicBVH.cpp:87-103 */
static void bvh_update_bounds(bvh_build_t* b, uint32_t ni)
{
    vpx_bvh_node* nd = &b->node[ni];
    float mn[3] = {1e30f, 1e30f, 1e30f}, mx[3] = {-1e30f, -1e30f, -1e30f};
    for (uint32_t i = 0; i < nd->tri_count; ++i) {
        const vpx_bvh_tri* t = &b->tri[b->idx[nd->left_first + i]];
        for (int k = 0; k < 3; ++k) {
            mn[k] = fminf_t(mn[k], t->v0[k]), mn[k] = fminf_t(mn[k], t->v1[k]), mn[k] = fminf_t(mn[k], t->v2[k]);
            mx[k] = fmaxf_t(mx[k], t->v0[k]), mx[k] = fmaxf_t(mx[k], t->v1[k]), mx[k] = fmaxf_t(mx[k], t->v2[k]);
        }
    }
    for (int k = 0; k < 3; ++k) nd->aabb_min[k] = mn[k], nd->aabb_max[k] = mx[k];
}

/* BasicBVH::Subdivide, BasicBVH.cpp:105-136 */
static void bvh_subdivide(bvh_build_t* b, uint32_t ni)
{
    vpx_bvh_node* nd = &b->node[ni];
    if (nd->tri_count <= 2) return;
    const float ext[3] = {nd->aabb_max[0] - nd->aabb_min[0], nd->aabb_max[1] - nd->aabb_min[1],
                          nd->aabb_max[2] - nd->aabb_min[2]};
    int axis = 0;
    if (ext[1] > ext[0]) axis = 1;
    if (ext[2] > ext[axis]) axis = 2;
    const float split = nd->aabb_min[axis] + ext[axis] * 0.5f;
    int i = (int)nd->left_first;
    int j = i + (int)nd->tri_count - 1;
    while (i <= j) {
        const v3 c = b->centroid[b->idx[i]];
        const float ca = axis == 0 ? c.x : (axis == 1 ? c.y : c.z);
        if (ca < split) {
            i++;
        } else {
            const uint32_t tmp = b->idx[i];
            b->idx[i] = b->idx[j];
            b->idx[j--] = tmp;
        }
    }
    const int left = i - (int)nd->left_first;
    if (left == 0 || (uint32_t)left == nd->tri_count) return;
    const uint32_t li = b->used++, ri = b->used++;
    b->node[li].left_first = nd->left_first;
    b->node[li].tri_count = (uint32_t)left;
    b->node[ri].left_first = (uint32_t)i;
    b->node[ri].tri_count = nd->tri_count - (uint32_t)left;
    nd->left_first = li;
    nd->tri_count = 0;
    bvh_update_bounds(b, li);
    bvh_update_bounds(b, ri);
    bvh_subdivide(b, li);
    bvh_subdivide(b, ri);
}

/* BasicBVH::BuildBVH, BasicBVH.cpp:72-85 (centroid = (v0 + v1 + v2) * 0.3333f). */
uint32_t oracle_bvh_build(const vpx_bvh_tri* tris, uint32_t n, vpx_bvh_node* nodes, uint32_t* tri_idx)
{
    if (!n) return 0;
    bvh_build_t b;
    b.tri = tris;
    b.idx = tri_idx;
    b.node = nodes;
    b.used = 1;
    b.centroid = (v3*)malloc(sizeof(v3) * n);
    for (uint32_t i = 0; i < n; ++i) tri_idx[i] = i;
    for (uint32_t i = 0; i < n; ++i)
        b.centroid[i] = vmuls(vadd(vadd(v3f(tris[i].v0), v3f(tris[i].v1)), v3f(tris[i].v2)), 0.3333f);
    memset(nodes, 0, sizeof(vpx_bvh_node) * (2 * (size_t)n - 1));
    nodes[0].left_first = 0, nodes[0].tri_count = n;
    bvh_update_bounds(&b, 0);
    bvh_subdivide(&b, 0);
    free(b.centroid);
    return b.used;
}

/* BasicBVH::IntersectTri, BasicBVH.cpp:19-36 */
static void bvh_tri(ray_t* r, const vpx_bvh_tri* t)
{
    const v3 v0 = v3f(t->v0);
    const v3 e1 = vsub(v3f(t->v1), v0), e2 = vsub(v3f(t->v2), v0);
    const v3 h = vcross(r->D, e2);
    const float a = vdot(e1, h);
    if (a > -0.0001f && a < 0.0001f) return;
    const float f = 1 / a;
    const v3 s = vsub(r->O, v0);
    const float u = f * vdot(s, h);
    if (u < 0 || u > 1) return;
    const v3 q = vcross(s, e1);
    const float v = f * vdot(r->D, q);
    if (v < 0 || u + v > 1) return;
    const float tt = f * vdot(e2, q);
    if (tt > 0.0001f) r->t = smin(r->t, tt);
}

/* BasicBVH::IntersectAABB, BasicBVH.cpp:38-48 */
static int bvh_aabb(const ray_t* r, const float* bmin, const float* bmax)
{
    const float tx1 = (bmin[0] - r->O.x) / r->D.x, tx2 = (bmax[0] - r->O.x) / r->D.x;
    float tmin = smin(tx1, tx2), tmax = smax(tx1, tx2);
    const float ty1 = (bmin[1] - r->O.y) / r->D.y, ty2 = (bmax[1] - r->O.y) / r->D.y;
    tmin = smax(tmin, smin(ty1, ty2)), tmax = smin(tmax, smax(ty1, ty2));
    const float tz1 = (bmin[2] - r->O.z) / r->D.z, tz2 = (bmax[2] - r->O.z) / r->D.z;
    tmin = smax(tmin, smin(tz1, tz2)), tmax = smin(tmax, smax(tz1, tz2));
    return tmax >= tmin && tmin < r->t && tmax > 0;
}

/* BasicBVH::IntersectBVH, BasicBVH.cpp:50-70 (recursive: left subtree, then right). */
static void bvh_node_visit(ray_t* r, const vpx_bvh_node* nodes, const vpx_bvh_tri* tris, const uint32_t* idx,
                           uint32_t ni)
{
    const vpx_bvh_node* nd = &nodes[ni];
    if (!bvh_aabb(r, nd->aabb_min, nd->aabb_max)) return;
    if (nd->tri_count > 0) {
        for (uint32_t i = 0; i < nd->tri_count; ++i) bvh_tri(r, &tris[idx[nd->left_first + i]]);
    } else {
        bvh_node_visit(r, nodes, tris, idx, nd->left_first);
        bvh_node_visit(r, nodes, tris, idx, nd->left_first + 1);
    }
}

int oracle_bvh_intersect(const vpx_bvh_node* nodes, const vpx_bvh_tri* tris, const uint32_t* tri_idx,
                         const vpx_ray* rays, uint32_t n, float* t_out)
{
    if ((!rays || !t_out) && n) return VPX_E_INVALID;
    const fpstate fs = fp_enter();
    for (uint32_t i = 0; i < n; ++i) {
        ray_t r = ray_from_api(&rays[i]);
        if (nodes) bvh_node_visit(&r, nodes, tris, tri_idx, 0);
        t_out[i] = r.t;
    }
    fp_leave(fs);
    return VPX_OK;
}
