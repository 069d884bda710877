// vpx_trace.hpp — device-side voxel ray-trace path for gfx950 (CDNA4).
//
// One ray per lane.  The reference's recursive Renderer::Trace (renderer.cpp:1076-1328)
// is a single chain (every material makes at most one recursive call), so it runs here
// as a loop that records one (a, b, form) combine record per level and folds them
// bottom-up at the end — the same rounding order as the recursion, so results are
// bit-identical to the CPU restatement, not merely close.
//
// Float semantics match the reference as restated in oracle/vpx_oracle.c: the library is
// built with -ffp-contract=off and f32 denormal flush (template/template.cpp:130 sets
// FTZ|DAZ); division and sqrt are correctly rounded (hipcc default); std::min/std::max
// are spelled as the exact ternaries; sin/cos/pow/exp are the correctly rounded f32
// values obtained through f64.  No approximations (rcp/rsq) are used anywhere; note that
// HIP's __fsqrt_rn lowers to a 3-ulp sqrt (!fpmath 3.0), so plain sqrtf (correctly
// rounded under hipcc's default -fhip-fp32-correctly-rounded-divide-sqrt) is used.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/vpx.h"
#include "vpx_skip.hpp"
#include "vpx_x86.hpp"

namespace vpx {

constexpr uint32_t kNone = 255u;
constexpr float kPi = 3.14159265358979323846264f;  // common.h:8
constexpr float kBig = 1e34f;
constexpr int kMaxLevels = 16;                     // max_bounces <= 14 -> 15 levels

// ----------------------------------------------------------------------- device view
// A voxel grid as the device walks it: the dense MatType bytes (x + y*N + z*N^2) plus
// two levels built from them (build_masks, layout in vpx_skip.hpp GridView): l2 = one
// 64-bit brick-occupancy mask per 16^3 macro, l1 = per 4^3 brick its cell mask (occupied)
// or its directional distance-field word (empty).  They only decide WHETHER a cell must
// be read; the march still visits every cell in the reference order with the reference
// float arithmetic, so t / cells / normals are unchanged.
struct DevGrid {
    const uint8_t* cells;
    const uint64_t* l1;
    const uint64_t* l2;
    uint32_t n;
    uint32_t nb1;  // bricks per axis  = ceil(n / 4)
    uint32_t nb2;  // macros per axis  = ceil(nb1 / 4)
    uint32_t nb3;  // macro parents per axis (l2 blocking) = ceil(nb2 / 4)
    const uint8_t* dfp;  // the distance field as 8 octant planes of bytes (vpx_skip.hpp GridView)
    uint64_t plane;      // bytes per octant plane = nb2^3 * 64
};

// Instance TLAS over the world bounds of volumes 1..n-1 (built on the host by vpx_set_volumes
// for 2..kTlasMaxVolumes volumes: the world volume 0 and up to 64 instances, C4's scene).
// Nodes in depth-first order, stackless: an interior node continues at i + 1 when its box
// is hit and at `skip` (the node after its subtree) when missed; a leaf holds the bit mask
// of its volumes (bit k = volume k + 1).
constexpr uint32_t kTlasMaxVolumes = 65;
#ifndef VPX_TLAS_SLOAD
#define VPX_TLAS_SLOAD 1  // the instance pass reads the TLAS and its candidates' records with scalar loads
#endif
constexpr uint32_t kTlasMaxNodes = 128;  // 2 x 64 - 1 with one volume per leaf
struct TlasNode {
    float lo[3];
    uint32_t skip;
    float hi[3];
    uint32_t leaf;
    uint64_t mask;
};

struct SceneView {
    const DevGrid* grids;
    const vpx_volume* volumes;
    const float4* vbounds;  // per volume: its cube's inflated world AABB, [2i] lo xyz, [2i + 1] hi xyz
    const TlasNode* tlas;   // instance TLAS (global memory; the multi-volume kernels stage it in LDS)
    uint32_t tlas_on, tlas_nodes;
    uint64_t tlas_always;   // instances outside the tree (no finite bounds): always candidates
    const vpx_material* materials;
    const vpx_point_light* points;
    const vpx_spot_light* spots;
    const vpx_area_light* areas;
    const vpx_sphere* spheres;
    const vpx_triangle* triangles;
    uint32_t num_volumes, num_points, num_spots, num_areas, num_spheres, num_triangles;
    vpx_dir_light dir;
    float sky[3];
    int32_t area_samples;
    // activateSky: an equirectangular HDR (stbi_loadf RGB floats, renderer.cpp:691) with
    // HDRLightContribution (renderer.h:224-226); sky_tex == 0 -> the constant `sky`.
    const float* sky_px;
    uint32_t sky_w, sky_h;
    float sky_hdr;
    uint32_t sky_tex;
    // the grid every volume after the world (1 .. n-1) uses, or -1: then a wave's lanes can walk
    // different instances in one walk (lane_volumes), the grid data being the same
    int32_t inst_grid;
    // reference arithmetic (vpx_set_arithmetic): the host's rcpss / rsqrtss tables, or a null
    // tab for the exact 1/x and 1/sqrtf of the default mode
    X86Arith x86;
};

// Read-only scene tables through the constant address space (VPX_CONST_AS): a load at a
// wave-uniform index becomes a scalar load through the scalar cache.  Through a generic
// pointer the compiler cannot prove the table unclobbered by the kernel's own global stores,
// so a uniform read was a vector load (L2 latency) into VGPRs.  Used where a wave walks a
// chain of uniform loads (the instance TLAS and the candidates' records); applied everywhere
// it moved the walkers' matrices into SGPRs and spilled them (round 4).  The tables are
// written only by the host between renders.
#define VPX_CONST_AS __attribute__((address_space(4)))

// p[i] for a wave-uniform i: a scalar load (VPX_TLAS_SLOAD) or the plain vector load.
template <class T>
__device__ __forceinline__ T ldu(const T* p, uint32_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (VPX_TLAS_SLOAD) {
        static_assert(sizeof(T) % 4 == 0, "ldu: dword-sized records");
        T v;
        const VPX_CONST_AS uint32_t* src = (const VPX_CONST_AS uint32_t*)(p + i);
        uint32_t* dst = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
        for (uint32_t k = 0; k < sizeof(T) / 4u; ++k) dst[k] = src[k];
        return v;
    }
#endif
    return p[i];
}

struct f3 {
    float x, y, z;
};

__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 ld3(const float* p) { return f3{p[0], p[1], p[2]}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 operator*(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ f3 operator/(f3 a, f3 b) { return mk(a.x / b.x, a.y / b.y, a.z / b.z); }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ f3 operator/(f3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
__device__ __forceinline__ f3 operator-(f3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float length(f3 a) { return sqrtf(dot(a, a)); }
__device__ __forceinline__ f3 normalize(f3 v) {
    const float inv = __fdiv_rn(1.0f, sqrtf(dot(v, v)));
    return v * inv;
}
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
// std::min / std::max exactly (first operand returned on ties / NaN).
__device__ __forceinline__ float smin(float a, float b) { return (b < a) ? b : a; }
__device__ __forceinline__ float smax(float a, float b) { return (a < b) ? b : a; }

// static_cast<int>(float) as the x86 reference evaluates it (cvttss2si: INT_MIN when
// out of range or NaN); v_cvt_i32_f32 would saturate instead.
__device__ __forceinline__ int trunc_i32(float f) {
    return (f > -2147483904.0f && f < 2147483648.0f) ? (int)f : (int)0x80000000u;
}
__device__ __forceinline__ float sign_of(float d) { return (float)(__float_as_uint(d) >> 31); }
__device__ __forceinline__ f3 dsign(f3 d) { return mk(sign_of(d.x), sign_of(d.y), sign_of(d.z)); }

// sinf / cosf / expf / powf(x, 5) of the reference (tmpl8math.h:2506-2508, renderer.cpp:
// 1593, 1607, 1615) as float results of one fixed double-precision evaluation that the
// oracle repeats operation for operation (vpx_oracle.c dm_*): Cody-Waite reduction and the
// fdlibm kernel polynomials, within 1 ulp (double) of the true value, so the float result
// is the correctly rounded one except at double-rounding midpoints (none in 4M samples per
// function, tests/test_cpu_oracle.py).  ocml's sin/cos/exp/pow carry a large-argument
// reduction path whose registers spilled the fused level-0 shade; the callers' arguments
// are bounded (sin/cos: [0, 2pi), exp: <= 0, pow5: [0, 2]).
namespace dm {
constexpr double kS1 = -1.66666666666666324348e-01, kS2 = 8.33333333332248946124e-03,
                 kS3 = -1.98412698298579493134e-04, kS4 = 2.75573137070700676789e-06,
                 kS5 = -2.50507602534068634195e-08, kS6 = 1.58969099521155010221e-10;
constexpr double kC1 = 4.16666666666666019037e-02, kC2 = -1.38888888888741095749e-03,
                 kC3 = 2.48015872894767294178e-05, kC4 = -2.75573143513906633035e-07,
                 kC5 = 2.08757232129817482790e-09, kC6 = -1.13596475577881948265e-11;
constexpr double kInvPio2 = 6.36619772367581382433e-01, kPio2_1 = 1.57079632673412561417e+00,
                 kPio2_1t = 6.07710050650619224932e-11;
constexpr double kLn2Hi = 6.93147180369123816490e-01, kLn2Lo = 1.90821492927058770002e-10,
                 kInvLn2 = 1.44269504088896338700e+00;
constexpr double kP1 = 1.66666666666666019037e-01, kP2 = -2.77777777770155933842e-03,
                 kP3 = 6.61375632143793436117e-05, kP4 = -1.65339022054652515390e-06,
                 kP5 = 4.13813679705723846039e-08;
__device__ __forceinline__ double ksin(double x) {  // |x| <= pi/4
    const double z = x * x, v = z * x;
    const double r = kS2 + z * (kS3 + z * (kS4 + z * (kS5 + z * kS6)));
    return x + v * (kS1 + z * r);
}
__device__ __forceinline__ double kcos(double x) {  // |x| <= pi/4
    const double z = x * x;
    const double r = z * (kC1 + z * (kC2 + z * (kC3 + z * (kC4 + z * (kC5 + z * kC6)))));
    const double hz = 0.5 * z, w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + z * r);
}
// sin and cos of one argument, |x| < 2^20 (k * kPio2_1 exact: kPio2_1 has 33 bits)
__device__ __forceinline__ void sincos(float xf, float& sf, float& cf) {
    const double x = (double)xf;
    const double k = __builtin_rint(x * kInvPio2);
    const double r = (x - k * kPio2_1) - k * kPio2_1t;
    const int n = (int)k & 3;
    const double s = ksin(r), c = kcos(r);
    sf = (float)(n == 0 ? s : n == 1 ? c : n == 2 ? -s : -c);
    cf = (float)(n == 0 ? c : n == 1 ? -s : n == 2 ? -c : s);
}
__device__ __forceinline__ float exp(float xf) {
    if (xf != xf) return xf;
    double x = (double)xf;
    x = x < -800.0 ? -800.0 : (x > 800.0 ? 800.0 : x);
    const double k = __builtin_rint(x * kInvLn2);
    const double hi = x - k * kLn2Hi, lo = k * kLn2Lo;
    const double r = hi - lo, t = r * r;
    const double c = r - t * (kP1 + t * (kP2 + t * (kP3 + t * (kP4 + t * kP5))));
    const double y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);
    return (float)__builtin_ldexp(y, (int)k);
}
__device__ __forceinline__ float pow5(float xf) {
    const double x = (double)xf, x2 = x * x, x4 = x2 * x2;
    return (float)(x4 * x);
}
}  // namespace dm
__device__ __forceinline__ float cr_sin(float x) { float s, c; dm::sincos(x, s, c); return s; }
__device__ __forceinline__ float cr_cos(float x) { float s, c; dm::sincos(x, s, c); return c; }
__device__ __forceinline__ float cr_exp(float x) { return dm::exp(x); }
__device__ __forceinline__ float cr_pow5(float x) { return dm::pow5(x); }

// ---------------------------------------------------------------------------- RNG
// WangHash / xorshift32 / RandomFloat: template/tmpl8math.cpp:20-27, 119-133.
__host__ __device__ __forceinline__ uint32_t wang_hash(uint32_t s) {
    s = (s ^ 61u) ^ (s >> 16);
    s *= 9u;
    s = s ^ (s >> 4);
    s *= 0x27d4eb2du;
    s = s ^ (s >> 15);
    return s;
}
__host__ __device__ __forceinline__ uint32_t pixel_seed(uint32_t base, uint32_t frame, uint32_t w,
                                                        uint32_t h, uint32_t x, uint32_t y) {
    const uint32_t k = base + frame * (w * h) + y * w + x;
    return 0x12345678u + wang_hash((k + 1u) * 17u);
}

struct Rng {
    uint32_t s;
    __device__ __forceinline__ float next() {
        s ^= s << 13;
        s ^= s >> 17;
        s ^= s << 5;
        return (float)s * 2.3283064365387e-10f;
    }
};

// --------------------------------------------------------------------- transforms
// TransformPosition_SSEM / TransformVector_SSEM (tmpl8math.cpp:369-402): pairwise sums.
__device__ __forceinline__ f3 xform_pos_ssem(f3 a, const float* m) {
    return mk((a.x * m[0] + a.y * m[1]) + (a.z * m[2] + m[3]),
              (a.x * m[4] + a.y * m[5]) + (a.z * m[6] + m[7]),
              (a.x * m[8] + a.y * m[9]) + (a.z * m[10] + m[11]));
}
__device__ __forceinline__ f3 xform_vec_ssem(f3 a, const float* m) {
    return mk((a.x * m[0] + a.y * m[1]) + a.z * m[2], (a.x * m[4] + a.y * m[5]) + a.z * m[6],
              (a.x * m[8] + a.y * m[9]) + a.z * m[10]);
}
// TransformPosition / TransformVector (tmpl8math.cpp:345-353): left-to-right sums.
__device__ __forceinline__ f3 xform_pos(f3 a, const float* m) {
    return mk(m[0] * a.x + m[1] * a.y + m[2] * a.z + m[3] * 1.0f,
              m[4] * a.x + m[5] * a.y + m[6] * a.z + m[7] * 1.0f,
              m[8] * a.x + m[9] * a.y + m[10] * a.z + m[11] * 1.0f);
}
__device__ __forceinline__ f3 xform_vec(f3 a, const float* m) {
    return mk(m[0] * a.x + m[1] * a.y + m[2] * a.z + m[3] * 0.0f,
              m[4] * a.x + m[5] * a.y + m[6] * a.z + m[7] * 0.0f,
              m[8] * a.x + m[9] * a.y + m[10] * a.z + m[11] * 0.0f);
}

// OffsetRay (tmpl8math.cpp:473-487): integer ULP nudge, float nudge near the origin.
__device__ __forceinline__ float offset1(float p, float n) {
    const int o = trunc_i32(256.0f * n);
    const float pi = __uint_as_float(__float_as_uint(p) + (uint32_t)((p < 0) ? -o : o));
    return fabsf(p) < (1.0f / 32.0f) ? p + (1.0f / 65536.0f) * n : pi;
}
__device__ __forceinline__ f3 offset_ray(f3 p, f3 n) {
    return mk(offset1(p.x, n.x), offset1(p.y, n.y), offset1(p.z, n.z));
}

// --------------------------------------------------------------------------- rays
// World-space ray.  Dsign and rD are always derivable from D where the reference
// reads them (they are recomputed per volume in object space), so only O/D are kept.
struct Ray {
    f3 O, D, N;
    float t;
    uint32_t mat;
    bool inside;
};

// Ray::Ray(origin, direction), template/scene.cpp:83-93.
__device__ __forceinline__ Ray make_ray(f3 o, f3 dir) {
    Ray r;
    r.O = o;
    r.D = normalize(dir);
    r.N = mk(0.f, 0.f, 0.f);
    r.t = kBig;
    r.mat = kNone;
    r.inside = false;
    return r;
}
__device__ __forceinline__ f3 ray_point(const Ray& r) { return r.O + r.D * r.t; }

// Object-space ray inside one volume visit (Ray fields after the per-volume transform).
struct ORay {
    f3 O, D, rD;
};

// rD of a Renderer::FindNearest volume visit.  Default: exact 1/D.  Reference arithmetic
// (xa.tab set, wave-uniform): FastReciprocal = rcpps + one Newton step, (r + r) - D * (r * r)
// (renderer.cpp:929-934, :969), rcpps from the host's captured table (vpx_x86.hpp) — a zero
// component gives inf * 0 = NaN there, as on the host.
__device__ __forceinline__ float fast_reciprocal1(float x, uint32_t t) {  // t: x's table entry
    const float r = __uint_as_float(x86_rcp_from(__float_as_uint(x), t));
    const float muls = x * (r * r);
    return (r + r) - muls;
}
// The multi-volume walkers look the rcp table up once per component of every volume visit
// (C4: up to 64 instance visits per wave), and from global memory each lookup is an L2 round
// trip ahead of Setup3DDDA (C4 47.3 vs 42.4 ms per step).  These kernels stage the rcp part of
// the table (2^(23 - rcp_shift) words: 16 KiB for the 12-bit key of the AMD EPYC host, 8 KiB for
// the 11-bit Intel key; vpx_set_arithmetic refuses keys wider than kX86LdsBits) into their
// dynamic LDS once per workgroup and read it there.  Call before any early return (barrier).
constexpr uint32_t kX86LdsBits = 13;
__device__ __forceinline__ X86Arith x86_stage_lds(const X86Arith& xa, uint32_t* lds) {
    X86Arith o = xa;
#ifndef VPX_NO_X86
    if (xa.tab) {
        for (uint32_t i = threadIdx.x; i < xa.rsq_off; i += blockDim.x) lds[i] = xa.tab[i];
        __syncthreads();
        o.tab = lds;
    }
#endif
    return o;
}
__device__ __forceinline__ f3 nearest_rd(f3 d, const X86Arith& xa) {
#if !defined(VPX_NO_X86) && !defined(VPX_DEBUG_X86_NO_RCP)  // (the debug hook: a timing probe, wrong results)
    if (xa.tab) {  // the three entries' loads issued together, then the branch-free results
        const uint32_t tx = xa.tab[x86_rcp_key(__float_as_uint(d.x), xa.rcp_shift)];
        const uint32_t ty = xa.tab[x86_rcp_key(__float_as_uint(d.y), xa.rcp_shift)];
        const uint32_t tz = xa.tab[x86_rcp_key(__float_as_uint(d.z), xa.rcp_shift)];
#ifdef VPX_DEBUG_X86_WORK_EXACT  // timing probe: the table work done, the exact values used
        const f3 fr = mk(fast_reciprocal1(d.x, tx), fast_reciprocal1(d.y, ty), fast_reciprocal1(d.z, tz));
        return mk(__fdiv_rn(1.0f, d.x) + 0.0f * fr.x, __fdiv_rn(1.0f, d.y) + 0.0f * fr.y,
                  __fdiv_rn(1.0f, d.z) + 0.0f * fr.z);
#endif
        return mk(fast_reciprocal1(d.x, tx), fast_reciprocal1(d.y, ty), fast_reciprocal1(d.z, tz));
    }
#endif
    return mk(__fdiv_rn(1.0f, d.x), __fdiv_rn(1.0f, d.y), __fdiv_rn(1.0f, d.z));
}

// ------------------------------------------------------------------------ the DDA
struct Dda {
    uint32_t X, Y, Z;
    int sx, sy, sz;
    float t;
    f3 tdelta, tmax;
};

// Cube::Intersect, template/scene.cpp:166-202.
__device__ __forceinline__ float cube_intersect(f3 b0, f3 b1, const ORay& r) {
    const bool sgx = r.D.x < 0, sgy = r.D.y < 0, sgz = r.D.z < 0;
    float tmin_x = ((sgx ? b1.x : b0.x) - r.O.x) * r.rD.x;
    float tmax_x = ((sgx ? b0.x : b1.x) - r.O.x) * r.rD.x;
    const float tmin_y = ((sgy ? b1.y : b0.y) - r.O.y) * r.rD.y;
    const float tmax_y = ((sgy ? b0.y : b1.y) - r.O.y) * r.rD.y;
    if (tmin_x > tmax_y || tmin_y > tmax_x) return kBig;
    tmin_x = smax(tmin_x, tmin_y);
    tmax_x = smin(tmax_x, tmax_y);
    const float tmin_z = ((sgz ? b1.z : b0.z) - r.O.z) * r.rD.z;
    const float tmax_z = ((sgz ? b0.z : b1.z) - r.O.z) * r.rD.z;
    if (tmin_x > tmax_z || tmin_z > tmax_x) return kBig;
    tmin_x = smax(tmin_x, tmin_z);
    return tmin_x > 0 ? tmin_x : kBig;
}

// Scene::Setup3DDDA, template/scene.cpp:719-749.
__device__ __forceinline__ bool dda_setup(const vpx_volume& vol, uint32_t n, const ORay& r, Dda& s) {
    const f3 b0 = ld3(vol.b0), b1 = ld3(vol.b1);
    s.t = 0;
    const bool contains = r.O.x >= b0.x && r.O.y >= b0.y && r.O.z >= b0.z && r.O.x <= b1.x &&
                          r.O.y <= b1.y && r.O.z <= b1.z;
    if (!contains) {
        s.t = cube_intersect(b0, b1, r);
        if (s.t > 1e33f) return false;
    }
    const f3 vmax = b1 - b0;
    const float g = (float)n;
    const float cell = __fdiv_rn(1.0f, g);
    const f3 ds = dsign(r.D);
    s.sx = trunc_i32(1.0f - ds.x * 2.0f);
    s.sy = trunc_i32(1.0f - ds.y * 2.0f);
    s.sz = trunc_i32(1.0f - ds.z * 2.0f);
    const f3 pos = (((r.O - b0) + r.D * (s.t + 0.00005f)) * g) / vmax;
    const f3 planes = (mk(ceilf(pos.x), ceilf(pos.y), ceilf(pos.z)) - ds) * cell;
    const int hi = (int)(n - 1);
    int px = trunc_i32(pos.x), py = trunc_i32(pos.y), pz = trunc_i32(pos.z);
    px = px < 0 ? 0 : (px > hi ? hi : px);
    py = py < 0 ? 0 : (py > hi ? hi : py);
    pz = pz < 0 ? 0 : (pz > hi ? hi : pz);
    s.X = (uint32_t)px;
    s.Y = (uint32_t)py;
    s.Z = (uint32_t)pz;
    s.tdelta = mk(cell * (float)s.sx, cell * (float)s.sy, cell * (float)s.sz) * r.rD;
    s.tmax = ((planes * vmax) - (r.O - b0)) * r.rD;
    return true;
}

// Ray::GetNormalVoxel, template/scene.cpp:121-148 (object-space O/D/t, Dsign of D).
__device__ __forceinline__ f3 normal_voxel(const ORay& r, float t, uint32_t n, const float* matrix) {
    const f3 i1 = (r.O + r.D * t) * (float)n;
    const f3 fg = mk(i1.x - floorf(i1.x), i1.y - floorf(i1.y), i1.z - floorf(i1.z));
    const f3 d = mk(smin(fg.x, 1.0f - fg.x), smin(fg.y, 1.0f - fg.y), smin(fg.z, 1.0f - fg.z));
    const float mind = smin(smin(d.x, d.y), d.z);
    const f3 sg = dsign(r.D) * 2.0f - mk(1.f, 1.f, 1.f);
    const f3 nn = mk(mind == d.x ? sg.x : 0.0f, mind == d.y ? sg.y : 0.0f, mind == d.z ? sg.z : 0.0f);
    return normalize(xform_vec(nn, matrix));
}

// Wave-uniform copy of a grid view (callers walk the same volume in every active lane),
// kept in scalar registers.
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
template <class T>
__device__ __forceinline__ T* uni_ptr(T* p) {
    const uint64_t v = (uint64_t)p;
    return (T*)(((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v));
}
__device__ __forceinline__ skip::GridView grid_view(const DevGrid& g) {
    return skip::GridView{uni_ptr(g.cells), uni_ptr(g.l1), uni_ptr(g.l2), uni(g.n), uni(g.nb1), uni(g.nb2),
                          uni(g.nb3),       uni_ptr(g.dfp), g.plane};
}
__device__ __forceinline__ skip::Walk to_walk(const Dda& s) {
    skip::Walk w;
    w.X = s.X, w.Y = s.Y, w.Z = s.Z;
    w.t = s.t;
    w.tx = s.tmax.x, w.ty = s.tmax.y, w.tz = s.tmax.z;
    w.dx = s.tdelta.x, w.dy = s.tdelta.y, w.dz = s.tdelta.z;
    w.sx = s.sx, w.sy = s.sy, w.sz = s.sz;
    skip::walk_begin(w);
    return w;
}

// skip::walk_skip with wave-aware scheduling: each lane runs exactly the same sequence of
// classify / skip_box / step1 as skip::walk_skip (so results are identical), but the long
// skip_box is executed in batches — only when few lanes of the wave still want to take
// plain cell steps — instead of inside every step iteration of the wave.
// Skip-phase weights SKIPW per walk kind: keep stepping while steppers x SKIPW >= waiting
// skippers (measured on C1 / C3 / C2: FindNearest 2, IsOccluded 4, bounces 2; with the
// two-compare step FindNearest 1: C1 0.666 vs 0.671 ms over two three-run A/Bs).
constexpr uint32_t kSkipwNearest = 1, kSkipwBounce = 2, kSkipwShadow = 4;
// Smallest distance-field cube worth a skip per walk kind (C1, ms: FindNearest 0.430 with
// 2 / 0.435 with 1; IsOccluded 0.383 with 2 / 0.354 with 1).
#ifndef VPX_MINC_NEAREST
#define VPX_MINC_NEAREST 2
#endif
constexpr uint32_t kMincNearest = VPX_MINC_NEAREST, kMincBounce = 2, kMincShadow = 1;
// Brick runs per walk kind, the RUN word: cap | passes << 8 | seg2 << 17 | min2 << 18.
// After its octant-plane byte (and, in an occupied brick, its cell mask) loads, a lane
// steps up to `cap` cells inside its 4^3 brick on the register copy; `passes` brick loads
// per step-phase iteration.  Measured (ms, one box): primary C1 0.432 -> 0.402 with 3|2<<8;
// shadow C3 4.01 -> 3.82 with 3|1<<8; bounce C2 0.654 -> 0.569 with 4|1<<8.  Caps above 4
// spill (the runs are unrolled); caps 6 / 10 for runs through all-empty bricks: C1 0.751 /
// 0.765 vs 0.703 ms.
// seg2 (bit 17): the skip's second closed-form segment only when a lane of the wave needs it
// (skip_box_lean<true>).  Measured (ms, one box): C1 0.713 -> 0.693, C3 5.57 -> 5.34, rank
// 0's C1 share at 8 ranks 0.234 -> 0.222; bounce walks (rays leaving surfaces, whose boxes
// cross binades in most waves) C2 4.27 -> 4.34 with it, so off there.
// min2 (bit 18): step1's two-compare axis choice (vpx_skip.hpp).  Measured (ms, three
// interleaved runs, vs the three-compare form): C1 0.678 vs 0.687; the shadow walkers (72
// VGPRs, 7 waves/SIMD) spilled two more VGPRs with it and C3 went 5.26 -> 5.53, so they keep
// the three-compare form.
// Rejected walk variants (DESIGN.md §4 keeps the measurements): classifying from the l1 + l2
// words instead of the octant plane, a branch-free select-committed step, loading two
// cells' words per round trip, prefetching the exit brick's byte, speculative cell-mask
// loads after an occupied brick, walk continuations with a step budget.
#ifndef VPX_RUN_NEAREST
#define VPX_RUN_NEAREST (3u | 3u << 8 | 1u << 17 | 1u << 18)
#endif
constexpr uint32_t kRunNearest = VPX_RUN_NEAREST;
constexpr uint32_t kRunBounce = 4u | 1u << 8 | 0u << 17 | 1u << 18;
#ifndef VPX_RUN_SHADOW
#define VPX_RUN_SHADOW (3u | 1u << 8 | 1u << 17 | 0u << 18)
#endif
constexpr uint32_t kRunShadow = VPX_RUN_SHADOW;
// Round 5 (ms per step, three interleaved runs, tools/gpu_ab.sh): FindNearest runs of 3 cells in
// three passes instead of two, C1 0.5419-0.5446 vs 0.5491-0.5496, C3 3.57 either way (four
// passes 0.5424-0.5459; runs of 4 in three passes 0.5462-0.5497); k_frame0's shadow walks in two
// passes on top, C1 0.5413-0.5431 (its own word: the other shadow walkers with two passes, C2
// 2.466-2.480 vs 2.427-2.452).
// k_frame0's FindNearest (7 waves/SIMD, round 5): runs of 3 cells in four passes, C1
// 0.5433-0.5444 vs 0.5456-0.5482 ms in three, then 0.5427-0.5457 vs 0.5447-0.5484 (two boxes,
// three interleaved runs each); five passes 0.5464-0.5474, runs of 2 in four 0.5428-0.5472.
#ifndef VPX_RUN_FRAME_NEAREST
#define VPX_RUN_FRAME_NEAREST (3u | 4u << 8 | 1u << 17 | 1u << 18)
#endif
constexpr uint32_t kRunFrameNearest = VPX_RUN_FRAME_NEAREST;
// At 7 waves/SIMD the frame's shadow walks take the two-compare step too: C1 0.5418-0.5489 vs
// 0.5456-0.5539 ms (seven interleaved runs, all won; three passes 0.5479-0.5591).
#ifndef VPX_RUN_FRAME_SHADOW
#define VPX_RUN_FRAME_SHADOW (3u | 2u << 8 | 1u << 17 | 1u << 18)
#endif
constexpr uint32_t kRunFrameShadow = VPX_RUN_FRAME_SHADOW;
// The pools' walks (k_nearest_pool, k_shadow_pool: 96 VGPRs at 5 waves/SIMD) have their own
// words (A/B overrides: VPX_*_POOL).  With the pool's registers the shadow walks take the
// two-compare step without spilling: C3 3.684-3.719 vs 3.724-3.756 ms (three interleaved runs,
// round 3; skip weight 2 / 8 or skip minimum 2 on top: 3.70-3.73 / 3.70-3.72 / 3.77-3.78).
// The bounce pool takes the bounce words (kRunBounce, kSkipwBounce, kMincBounce): seg2, skip
// weight 1 / 4, runs of 3 cells in two passes measured C2 2.63-2.66 / 2.60-2.64 / 2.66-2.75 /
// 2.65-2.71 vs 2.59-2.65 ms, and re-checked at three lanes in round 5 (within noise).
#ifndef VPX_RUN_SHADOW_POOL
#define VPX_RUN_SHADOW_POOL (3u | 1u << 8 | 1u << 17 | 1u << 18)
#endif
#ifndef VPX_SKIPW_SHADOW_POOL
#define VPX_SKIPW_SHADOW_POOL 4u
#endif
#ifndef VPX_MINC_SHADOW_POOL
#define VPX_MINC_SHADOW_POOL 1u
#endif
constexpr uint32_t kRunShadowPool = VPX_RUN_SHADOW_POOL, kSkipwShadowPool = VPX_SKIPW_SHADOW_POOL,
                   kMincShadowPool = VPX_MINC_SHADOW_POOL;
#ifdef VPX_ASM_MARKS  // analysis builds only: label the walk phases in the ISA listing
#define VPX_MARK(s) asm volatile("; MARK " s)
#else
#define VPX_MARK(s)
#endif

#ifdef VPX_PHASE_PROF
// Debug build only (-DVPX_PHASE_PROF): per-wave cycles / iterations / active lanes of the
// step and skip phases of walk_wave, read back with vpx_debug_phase().
__device__ unsigned long long g_phase[32];
#define VPX_PH(...) __VA_ARGS__
#else
#define VPX_PH(...)
#endif

// Lane modes: kStep wants a cell step, kSkip an empty-box skip (the distance-field cube
// of its brick, skip::df_box, through skip::skip_box_lean), kMiss / kHit are done.
// Phases are wave-uniform: cell steps while enough lanes want one (see SKIPW), then the
// waiting lanes skip together.  Each lane runs exactly skip::walk_skip's sequence (the
// reference's cells with the reference's floats).
// POOL (the bounce pool, k_nearest_pool): the lanes' modes come in and go out through *pmode
// (lanes without a ray are kWalkMiss), and the walk also returns, with its lanes' state intact,
// once `leave` or more lanes of the wave have finished, so that their rays can be replaced.
constexpr int kWalkStep = 0, kWalkSkip = 1, kWalkMiss = 2, kWalkHit = 3;
template <int PHK, uint32_t SKIPW, uint32_t MINC, uint32_t RUN, bool POOL = false>
__device__ __forceinline__ bool walk_wave(const skip::GridView& g, skip::Walk& w, float bound, uint32_t& cells,
                                          int* pmode = nullptr, uint32_t leave = 65u) {
    enum : int { kStep = kWalkStep, kSkip = kWalkSkip, kMiss = kWalkMiss, kHit = kWalkHit };
    constexpr int kRun = (int)(RUN & 255u);
    constexpr int kPasses = (int)((RUN >> 8) & 255u);
    constexpr bool kSeg2Branch = (RUN >> 17) & 1u;
    constexpr bool kMin2 = (RUN >> 18) & 1u;  // step1's two-compare axis choice (vpx_skip.hpp)
    static_assert(SKIPW > 0 && kRun > 0 && kPasses > 0, "walk_wave: skip weight, run cap and passes");
    const uint32_t opar = skip::plane_parent(g, w.osh >> 3);  // the ray's octant plane
    int mode = POOL ? *pmode : kStep;
    VPX_PH(uint64_t cs = 0, ck = 0, ns = 0, nk = 0, ls = 0, lk = 0, fb = 0, cf = 0;)
    for (;;) {
        VPX_PH(uint64_t t0 = __builtin_amdgcn_s_memtime();)
        for (;;) {
            const uint64_t stepping = __ballot(mode == kStep);
            if (!stepping) break;
            // cost-weighted: a skip phase costs several step phases, so keep stepping while
            // steppers x SKIPW >= waiting skippers
            const uint32_t nskip = (uint32_t)__popcll(__ballot(mode == kSkip));
            if ((uint32_t)__popcll(stepping) * SKIPW < nskip) break;
            if (POOL && 64u - (uint32_t)__popcll(stepping) - nskip >= leave) goto pool_out;
            VPX_PH(++ns; ls += __popcll(stepping); cf += __popcll(__ballot(mode >= kMiss));)  // cf: finished lanes per step iteration
            VPX_MARK("step body");
            // Brick runs: the class of a cell is a function of its brick's plane byte and cell
            // mask only, so once they are loaded a lane keeps stepping on the register copy
            // while it stays in that brick — the cell mask (class 1) or "all empty" (class 3)
            // decides each cell exactly as classify would — and reloads only when it crosses
            // into another brick (or after kRun cells): fewer dependent memory round trips.
#pragma unroll
            for (int u = 0; u < kPasses; ++u) {
                if (mode == kStep) {
                    if (!(w.t < bound)) {
                        mode = kMiss;
                    } else {
                        const int cls = skip::classify_dfp_o<MINC>(w, g, opar);
                        // the class's outcome by selects: 0 = the solid cell (visited, hit), 2 =
                        // skip; 1 / 3 visit the cell and run on in the brick
                        cells += cls != 2 ? 1u : 0u;
                        mode = cls == 0 ? kHit : (cls == 2 ? kSkip : mode);
                        if (cls & 1) {
                            const uint64_t solid = cls == 1 ? w.m1 : 0ull;
#pragma unroll
                            for (int r = 0; r < kRun; ++r) {
                                const uint32_t ox = w.X, oy = w.Y, oz = w.Z;
                                // the same outcomes with one exit per cell (fewer exec-mask
                                // merges): left the grid -> miss; left the brick (or the run's
                                // cap) -> the next pass loads; bound reached -> miss; else the
                                // cell is visited, a solid one ends the walk
                                const bool ing = skip::step1<kMin2>(w, g.n);
                                const bool inb = r + 1 < kRun && ((w.X ^ ox) | (w.Y ^ oy) | (w.Z ^ oz)) <= 3u;
                                const bool inbound = w.t < bound;
                                const bool sol =
                                    (solid >> ((w.X & 3u) | ((w.Y & 3u) << 2) | ((w.Z & 3u) << 4))) & 1ull;
                                const bool visit = ing && inb && inbound;
                                cells += visit ? 1u : 0u;
                                mode = !ing || (inb && !inbound) ? kMiss : (visit && sol ? kHit : mode);
                                if (!visit || sol) break;
                            }
                        }
                    }
                }
            }
        }
        VPX_MARK("step phase end");
        VPX_PH(uint64_t t1 = __builtin_amdgcn_s_memtime(); cs += t1 - t0;)
        const uint64_t skipping = __ballot(mode == kSkip);
        if (!skipping) {
            if (!__ballot(mode == kStep)) break;
            continue;
        }
        VPX_PH(++nk; lk += __popcll(skipping);)
        VPX_MARK("skip phase");
        if (mode == kSkip) {
            uint32_t lo[3], hi[3];
            skip::df_box(w, g.n, skip::cube_dfp(w), lo, hi);
            const int sr = skip::skip_box_lean<kSeg2Branch>(w, lo, hi, bound, cells);  // 2 (refused): a plain step
            VPX_MARK("skip end");
            VPX_PH(fb += __popcll(__ballot(sr == 2));)
            if (sr == 1) {
                mode = kMiss;
            } else {
                ++cells;  // visit the landing cell, then take the leaving event
                mode = skip::step1<kMin2>(w, g.n) ? kStep : kMiss;
            }
        }
        VPX_PH(ck += __builtin_amdgcn_s_memtime() - t1;)
    }
    if (POOL) {
    pool_out:
        *pmode = mode;
    }
#ifdef VPX_PHASE_PROF
    if ((threadIdx.x & 63) == __builtin_amdgcn_readfirstlane(threadIdx.x & 63)) {
        atomicAdd(&g_phase[PHK + 0], cs);
        atomicAdd(&g_phase[PHK + 1], ck);
        atomicAdd(&g_phase[PHK + 2], ns);
        atomicAdd(&g_phase[PHK + 3], nk);
        atomicAdd(&g_phase[PHK + 4], ls);
        atomicAdd(&g_phase[PHK + 5], lk);
        atomicAdd(&g_phase[PHK + 6], 1ull);
        atomicAdd(&g_phase[PHK + 7], fb);
        atomicAdd(&g_phase[PHK + 8], cf);
    }
#endif
    return mode == kHit;
}

// Walk modes (all share the stepping of scene.cpp:773-802).
enum WalkMode { kNearest = 0, kGlassExit = 1, kSmokeExit = 2, kOcclusion = 3 };

struct WalkResult {
    bool hit;     // nearest: found a cell with t < bound; exits: left the material; occl: occluded
    float t;      // hit t (nearest / exits) or last s.t (exits leaving the grid)
    uint32_t cell;
};

// The Amanatides-Woo march.  `bound` is Ray::t on entry.  Loads one byte per visited
// cell (x + y*N + z*N^2, 64-bit index) and counts it in `cells`.
template <int MODE>
__device__ __forceinline__ WalkResult dda_walk(const DevGrid& g, Dda s, float bound, uint32_t& cells) {
    WalkResult res{false, s.t, kNone};
    const uint64_t n = g.n;
    const uint64_t nn = n * n;
    const uint8_t* __restrict__ grid = g.cells;
    for (;;) {
        if (MODE == kNearest || MODE == kOcclusion) {
            if (!(s.t < bound)) break;
        }
        const uint32_t cell = grid[(uint64_t)s.X + (uint64_t)s.Y * n + (uint64_t)s.Z * nn];
        ++cells;
        if (MODE == kNearest) {
            if (cell != kNone && s.t < bound) {
                res.hit = true, res.t = s.t, res.cell = cell;
                return res;
            }
        } else if (MODE == kOcclusion) {
            if (cell != kNone) {
                res.hit = s.t < bound;
                return res;
            }
        } else {
            const bool leave = (MODE == kGlassExit) ? (cell != VPX_MAT_GLASS)
                                                    : (cell > VPX_MAT_SMOKE_PLAYER || cell < VPX_MAT_SMOKE_LOW_DENSITY);
            if (leave) {
                res.hit = true, res.t = s.t, res.cell = cell;
                return res;
            }
        }
        // Axis choice: x<y ? (x<z ? x : z) : (y<z ? y : z), strict compares (scene.cpp:773-802).
        const bool xy = s.tmax.x < s.tmax.y, xz = s.tmax.x < s.tmax.z, yz = s.tmax.y < s.tmax.z;
        const int axis = xy ? (xz ? 0 : 2) : (yz ? 1 : 2);
        if (axis == 0) {
            if (MODE != kOcclusion) s.t = s.tmax.x;
            s.X += (uint32_t)s.sx;
            if (s.X >= g.n) break;
            if (MODE == kOcclusion) s.t = s.tmax.x;
            s.tmax.x += s.tdelta.x;
        } else if (axis == 1) {
            if (MODE != kOcclusion) s.t = s.tmax.y;
            s.Y += (uint32_t)s.sy;
            if (s.Y >= g.n) break;
            if (MODE == kOcclusion) s.t = s.tmax.y;
            s.tmax.y += s.tdelta.y;
        } else {
            if (MODE != kOcclusion) s.t = s.tmax.z;
            s.Z += (uint32_t)s.sz;
            if (s.Z >= g.n) break;
            if (MODE == kOcclusion) s.t = s.tmax.z;
            s.tmax.z += s.tdelta.z;
        }
    }
    res.t = s.t;  // exits: Scene::FindMaterialExit/FindSmokeExit set ray.t = s.t on leaving
    return res;
}

// ------------------------------------------------------------------------ shapes
// Sphere::Hit / IsHit, Triangle::Hit / IsHit — src/BVH/Shapes.h:12-139.
__device__ __forceinline__ void sphere_hit(const vpx_sphere& sp, Ray& r) {
    const f3 c = ld3(sp.center);
    const f3 to = r.O - c;
    const float b = dot(to, r.D);
    const float cc = dot(to, to) - (sp.radius * sp.radius);
    const float disc = b * b - cc;
    if (cc > 0.0f && b > 0.0f) return;
    if (disc < 0) return;
    const float len = -b - sqrtf(disc);
    if (len > r.t) return;
    if (len < 0) return;
    const f3 ip = r.O + r.D * len;
    const f3 outn = (ip - c) / sp.radius;
    const bool outside = dot(r.D, outn) < 0;
    r.N = outside ? outn : -outn;
    r.inside = !outside;
    r.t = len;
    r.mat = sp.material;
}
__device__ __forceinline__ bool sphere_is_hit(const vpx_sphere& sp, const Ray& r) {
    const f3 c = ld3(sp.center);
    const f3 to = r.O - c;
    const float b = dot(to, r.D);
    const float cc = dot(to, to) - (sp.radius * sp.radius);
    const float disc = b * b - cc;
    if (cc > 0.0f && b > 0.0f) return false;
    if (disc < 0) return false;
    const float len = -b - sqrtf(disc);
    if (len < 0) return false;
    if (len > r.t) return false;
    return true;
}
__device__ __forceinline__ bool tri_core(const vpx_triangle& tr, const Ray& r, float& t, f3& e1o, f3& e2o) {
    const f3 pos = ld3(tr.position);
    const f3 p1 = pos + ld3(tr.v0), p2 = pos + ld3(tr.v1), p3 = pos + ld3(tr.v2);
    const f3 e1 = p2 - p1, e2 = p3 - p1;
    const f3 h = cross(r.D, e2);
    const float a = dot(e1, h);
    if (a > -0.0001f && a < 0.0001f) return false;
    const float f = __fdiv_rn(1.0f, a);
    const f3 s = r.O - p1;
    const float u = f * dot(s, h);
    if (u < 0 || u > 1) return false;
    const f3 q = cross(s, e1);
    const float v = f * dot(r.D, q);
    if (v < 0 || u + v > 1) return false;
    t = f * dot(e2, q);
    e1o = e1;
    e2o = e2;
    return true;
}
__device__ __forceinline__ void tri_hit(const vpx_triangle& tr, Ray& r) {
    float t;
    f3 e1, e2;
    if (!tri_core(tr, r, t, e1, e2)) return;
    if (t > 0.0001f && r.t > t) {
        r.t = t;
        r.mat = tr.material;
        const f3 nrm = normalize(cross(e1, e2));
        r.N = dot(r.D, nrm) < 0 ? nrm : -nrm;
    }
}
__device__ __forceinline__ bool tri_is_hit(const vpx_triangle& tr, const Ray& r) {
    float t;
    f3 e1, e2;
    if (!tri_core(tr, r, t, e1, e2)) return false;
    if (t < 0.0001f) return false;
    if (t > r.t) return false;
    return true;
}

// ---------------------------------------------------------------- renderer level
struct Counters {
    uint32_t cells;
    uint32_t shadow;
    uint32_t nearest;
};

// Conservative slab test of a box against the segment o + t d, 0 <= t <= bound (inv = 1 / d
// per component, exact): false only when the segment misses the box.  A box that starts
// beyond `bound` is missed: a cube inside it (with a margin far above float rounding) is
// entered beyond the bound too, so the reference's walk of that volume ends before its first
// cell (`while (s.t < ray.t)`, scene.cpp:761, 1015).
__device__ __forceinline__ bool seg_box(float lx, float ly, float lz, float hx, float hy, float hz, f3 o, f3 inv,
                                        float bound) {
    float t0 = 0.0f, t1 = bound;
    const float ta[3] = {(lx - o.x) * inv.x, (ly - o.y) * inv.y, (lz - o.z) * inv.z};
    const float tb[3] = {(hx - o.x) * inv.x, (hy - o.y) * inv.y, (hz - o.z) * inv.z};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        t0 = fmaxf(t0, fminf(ta[k], tb[k]));
        t1 = fminf(t1, fmaxf(ta[k], tb[k]));
    }
    return !(t1 < t0);
}
__device__ __forceinline__ f3 world_inv(f3 d) { return mk(__fdiv_rn(1.0f, d.x), __fdiv_rn(1.0f, d.y), __fdiv_rn(1.0f, d.z)); }

// Volume cull: true when the ray's segment [0, bound] misses the inflated world AABB of the
// volume's cube (vpx_kernels.hip volume_bounds: the 8 corners through the affine map the
// walks use, padded and rounded outward) — then Setup3DDDA (Cube::Contains / Cube::Intersect,
// scene.cpp:166-210) fails, or enters the cube beyond ray.t, and the reference reads no cell of
// that volume, so skipping it changes nothing.  bound = the ray's t as it stands, which the
// reference's loop bounds each volume's walk with.  (Until round 6 a bounding sphere and the
// ray's line: the zone scene's long thin volumes passed ~7 spheres per ray, but ~2 cubes.)
__device__ __forceinline__ bool misses_volume(const float4* vb, uint32_t i, f3 o, f3 inv, float bound) {
    const float4 lo = vb[2u * i], hi = vb[2u * i + 1u];
    return !seg_box(lo.x, lo.y, lo.z, hi.x, hi.y, hi.z, o, inv, bound);
}
__device__ __forceinline__ bool misses_volume_u(const float4* vb, uint32_t i, f3 o, f3 inv, float bound) {
    const float4 lo = ldu(vb, 2u * i), hi = ldu(vb, 2u * i + 1u);  // i wave-uniform: scalar loads
    return !seg_box(lo.x, lo.y, lo.z, hi.x, hi.y, hi.z, o, inv, bound);
}

// A TLAS node's box (seg_box): a NaN slab (0 * inf on an axis the ray runs along a box face)
// yields NaN bounds that fminf / fmaxf drop.
__device__ __forceinline__ bool tlas_box(const TlasNode& nd, f3 o, f3 inv, float bound) {
    return seg_box(nd.lo[0], nd.lo[1], nd.lo[2], nd.hi[0], nd.hi[1], nd.hi[2], o, inv, bound);
}

// The volume loop of Renderer::FindNearest / IsOccluded over the TLAS.  Volume 0 (the world,
// first in the reference's order) is walked by every lane first; then the wave traverses the
// tree once, wave-uniform (a node is entered when any lane's segment reaches its box: the
// ray packet of an 8x8 pixel block), each lane collecting the leaves IT reaches before its
// bound as it stands after volume 0.  Every volume whose walk the reference would start and
// read a cell of is among them (boxes hold the inflated cube boxes of misses_volume,
// and a box starting beyond the bound holds a cube whose walk ends before its first cell,
// `while (s.t < ray.t)`, scene.cpp:761, 1015).  The wave then walks the union of the lanes'
// candidates in increasing index order, each lane only its own — the linear loop restricted
// to volumes some lane can reach, one call site of the walk.  body(i) returns false to end
// the lane's loop (IsOccluded's first occluder).
// SKIP0: volume 0 was walked already (the instance pass, k_instances, after the world pass):
// start from the tree with the bound as it stands.
template <bool SKIP0 = false, class Body>
__device__ __forceinline__ void for_volumes(const SceneView& sv, f3 o, f3 inv, const float& bound, Body body) {
    bool live = true, first = true;
    uint64_t mine = 0, any = 0;  // this lane's / the wave's candidates, bit k = volume k + 1
    for (;;) {
        uint32_t i = 0;
        if (!first) {
            if (!any) break;
            i = (uint32_t)__ffsll((unsigned long long)any);
            any &= any - 1;
        }
        if (live && (first ? !SKIP0 : ((mine >> (i - 1u)) & 1u))) live = body(i);
        if (first) {
            first = false;
            mine = sv.tlas_always;
            any = sv.tlas_always;
            for (uint32_t n = 0; n < sv.tlas_nodes;) {
                const TlasNode nd = ldu(sv.tlas, n);
                const bool h = live && tlas_box(nd, o, inv, bound);
                const bool wave_h = __ballot(h) != 0;
                if (nd.leaf) {
                    if (h) mine |= nd.mask;
                    if (wave_h) any |= nd.mask;
                    ++n;
                } else {
                    n = wave_h ? n + 1 : nd.skip;
                }
            }
        }
    }
}

// A lane's TLAS candidates (bit k = volume k + 1): the leaves its segment [0, bound] reaches
// (wave-uniform traversal, as for_volumes), plus the always-set.
__device__ __forceinline__ uint64_t tlas_candidates(const SceneView& sv, f3 o, f3 inv, float bound) {
    uint64_t mine = sv.tlas_always;
    for (uint32_t n = 0; n < sv.tlas_nodes;) {
        const TlasNode nd = ldu(sv.tlas, n);
        const bool h = tlas_box(nd, o, inv, bound);
        if (nd.leaf) {
            if (h) mine |= nd.mask;
            ++n;
        } else {
            n = __ballot(h) ? n + 1 : nd.skip;
        }
    }
    return mine;
}

// Lane volumes: when every volume after the world uses one grid (SceneView::inst_grid, C4's 64
// instances of one model), a wave walks each lane's own next candidate in one walk — the grid
// data is shared, only the object-space rays differ — so a wave costs the most candidates any
// one lane visits instead of the union of its lanes' candidates (walked one volume at a time,
// for_volumes).  Each lane visits its candidates in increasing index order with its bound as it
// stands: the reference's loop for that ray (renderer.cpp:209-243, 946-1018), the same cells,
// hits and counts.  next(): the lane's next volume whose walk can read a cell (Setup3DDDA
// succeeds) and its walk state; false when it has none.
template <class Next, class Done>
__device__ __forceinline__ void lane_volumes(const skip::GridView& gv, Next next, Done done) {
    for (;;) {
        skip::Walk w;
        uint32_t vi = 0;
        const bool have = next(w, vi);
        if (!__ballot(have)) break;
        if (have) done(w, vi);
    }
}

// Renderer::FindNearest, renderer.cpp:946-1018.  Linear loop over the volumes with the
// SSE transforms; a later volume wins only with a strictly smaller t (ties -> lowest index).
// The winner's normal and material are formed once after the loop (the reference forms
// them at every improving hit; the last one is the winner's, from the same object-space
// ray and t), so only t and the hit cell are carried through the walks.
#ifdef VPX_PHASE_PROF  // FindNearest volume visits: waves, lanes, lanes past the sphere cull / Setup3DDDA
__device__ __forceinline__ void prof_visit(int what, bool pass) {
    const uint64_t act = __ballot(true), ok = __ballot(pass);
    if ((threadIdx.x & 63u) != (uint32_t)__ffsll((unsigned long long)act) - 1u) return;
    if (what == 0) atomicAdd(&g_phase[10], 1ull), atomicAdd(&g_phase[11], (unsigned long long)__popcll(act));
    if (what == 1) atomicAdd(&g_phase[12], (unsigned long long)__popcll(ok));
    if (what == 2) atomicAdd(&g_phase[13], (unsigned long long)__popcll(ok)), atomicAdd(&g_phase[14], ok ? 1ull : 0ull);
}
#define VPX_PROF_VISIT(what, pass) prof_visit(what, pass)
#else
#define VPX_PROF_VISIT(what, pass)
#endif
template <uint32_t SKIPW = kSkipwNearest, uint32_t MINC = kMincNearest, uint32_t RUN = kRunNearest>
__device__ __forceinline__ int32_t find_nearest(const SceneView& sv, Ray& r, Counters& k) {
    int32_t vox = -2;
    ++k.nearest;
    uint32_t hx = 0, hy = 0, hz = 0;  // hit cell in volume `vox`
    const f3 inv = world_inv(r.D);     // the volume culls' slabs (misses_volume)
    auto visit = [&](uint32_t i) {
        VPX_PROF_VISIT(0, true);
        const bool mv = misses_volume(sv.vbounds, i, r.O, inv, r.t);
        VPX_PROF_VISIT(1, !mv);
        if (mv) return true;  // Setup3DDDA would fail
        const vpx_volume& vol = sv.volumes[i];
        const DevGrid g = sv.grids[vol.grid_id];
        skip::Walk w;
        {
            ORay o;
            o.O = xform_pos_ssem(r.O, vol.inv_matrix);
            o.D = xform_vec_ssem(r.D, vol.inv_matrix);
            o.rD = nearest_rd(o.D, sv.x86);
            Dda s;
            const bool ok = dda_setup(vol, g.n, o, s);
            VPX_PROF_VISIT(2, ok);
            if (!ok) return true;
            w = to_walk(s);
        }
        if (walk_wave<0, SKIPW, MINC, RUN>(grid_view(g), w, r.t, k.cells)) {
            r.t = w.t;
            hx = w.X, hy = w.Y, hz = w.Z;
            vox = (int32_t)i;
        }
        return true;
    };
    // with the TLAS, volume 0 (the world, first in the reference's order) is walked before
    // the tree is asked, so the instances' candidates are bounded by its hit
    if (sv.tlas_on)
        for_volumes(sv, r.O, inv, r.t, visit);
    else
        for (uint32_t i = 0; i < sv.num_volumes; ++i) visit(i);
    if (vox >= 0) {
        const vpx_volume& vol = sv.volumes[vox];
        const DevGrid g = sv.grids[vol.grid_id];
        ORay o;
        o.O = xform_pos_ssem(r.O, vol.inv_matrix);
        o.D = xform_vec_ssem(r.D, vol.inv_matrix);
        r.N = normal_voxel(o, r.t, g.n, vol.matrix);
        r.mat = g.cells[(uint64_t)hx + (uint64_t)hy * g.n + (uint64_t)hz * ((uint64_t)g.n * g.n)];
    }
    if (sv.num_spheres | sv.num_triangles) {
        Ray sh = make_ray(r.O, r.D);
        for (uint32_t i = 0; i < sv.num_spheres; ++i) sphere_hit(sv.spheres[i], sh);
        for (uint32_t i = 0; i < sv.num_triangles; ++i) tri_hit(sv.triangles[i], sh);
        if (r.t > sh.t) {
            r.t = sh.t;
            r.mat = sh.mat;
            r.N = sh.N;
            r.inside = sh.inside;
            vox = -1;
        }
    }
    return vox;
}

#ifndef VPX_LANE_VOLUMES
#define VPX_LANE_VOLUMES 1
#endif
// Renderer::FindNearest from volume 1 on (renderer.cpp:946-1018), for a ray whose walk of
// volume 0 already left r.t / the hit record (*vox = 0 on a hit there, else -2): the
// instance pass of multi-volume primary rays (k_instances), whose world walk ran in the lean
// single-volume kernel (k_primary<true, false>).  The same loop from the same state — the
// later volumes through the TLAS (or linearly), then the shapes — so the same winner, t and
// counts as find_nearest; the FindNearest call itself was counted by the world pass.
// Returns whether the record changed (a later volume or a shape won: r.t, r.N, r.mat, *vox).
template <uint32_t SKIPW = kSkipwNearest, uint32_t MINC = kMincNearest, uint32_t RUN = kRunNearest>
__device__ __forceinline__ bool find_nearest_rest(const SceneView& sv, Ray& r, Counters& k, int32_t* vox_io) {
    int32_t vox = *vox_io;
    const int32_t vox0 = vox;
    uint32_t hx = 0, hy = 0, hz = 0;
    const f3 inv = world_inv(r.D);
    auto visit = [&](uint32_t i) {  // i is wave-uniform (for_volumes / the linear loop)
        VPX_PROF_VISIT(0, true);
        const bool mv = misses_volume_u(sv.vbounds, i, r.O, inv, r.t);
        VPX_PROF_VISIT(1, !mv);
        if (mv) return true;
        const vpx_volume vol = ldu(sv.volumes, i);
        const DevGrid g = ldu(sv.grids, vol.grid_id);
        skip::Walk w;
        {
            ORay o;
            o.O = xform_pos_ssem(r.O, vol.inv_matrix);
            o.D = xform_vec_ssem(r.D, vol.inv_matrix);
            o.rD = nearest_rd(o.D, sv.x86);
            Dda s;
            const bool ok = dda_setup(vol, g.n, o, s);
            VPX_PROF_VISIT(2, ok);
            if (!ok) return true;
            w = to_walk(s);
        }
        if (walk_wave<0, SKIPW, MINC, RUN>(grid_view(g), w, r.t, k.cells)) {
            r.t = w.t;
            hx = w.X, hy = w.Y, hz = w.Z;
            vox = (int32_t)i;
        }
        return true;
    };
    if (sv.tlas_on && sv.inst_grid >= 0 && VPX_LANE_VOLUMES) {
        uint64_t rest = tlas_candidates(sv, r.O, inv, r.t);
        const DevGrid g = ldu(sv.grids, (uint32_t)sv.inst_grid);
        auto next = [&](skip::Walk& w, uint32_t& vi) {
            while (rest) {
                const uint32_t i = (uint32_t)__ffsll((unsigned long long)rest);  // bit i - 1 = volume i
                rest &= rest - 1ull;
                if (misses_volume(sv.vbounds, i, r.O, inv, r.t)) continue;
                const vpx_volume& vol = sv.volumes[i];  // this lane's own volume
                ORay o;
                o.O = xform_pos_ssem(r.O, vol.inv_matrix);
                o.D = xform_vec_ssem(r.D, vol.inv_matrix);
                o.rD = nearest_rd(o.D, sv.x86);
                Dda s;
                if (!dda_setup(vol, g.n, o, s)) continue;
                w = to_walk(s);
                vi = i;
                return true;
            }
            return false;
        };
        auto done = [&](skip::Walk& w, uint32_t vi) {
            if (walk_wave<0, SKIPW, MINC, RUN>(grid_view(g), w, r.t, k.cells)) {
                r.t = w.t;
                hx = w.X, hy = w.Y, hz = w.Z;
                vox = (int32_t)vi;
            }
        };
        lane_volumes(grid_view(g), next, done);
    } else if (sv.tlas_on) {
        for_volumes<true>(sv, r.O, inv, r.t, visit);
    } else {
        for (uint32_t i = 1; i < sv.num_volumes; ++i) visit(i);
    }
    bool changed = vox != vox0;
    if (changed) {
        const vpx_volume& vol = sv.volumes[vox];
        const DevGrid g = sv.grids[vol.grid_id];
        ORay o;
        o.O = xform_pos_ssem(r.O, vol.inv_matrix);
        o.D = xform_vec_ssem(r.D, vol.inv_matrix);
        r.N = normal_voxel(o, r.t, g.n, vol.matrix);
        r.mat = g.cells[(uint64_t)hx + (uint64_t)hy * g.n + (uint64_t)hz * ((uint64_t)g.n * g.n)];
    }
    if (sv.num_spheres | sv.num_triangles) {
        Ray sh = make_ray(r.O, r.D);
        for (uint32_t i = 0; i < sv.num_spheres; ++i) sphere_hit(sv.spheres[i], sh);
        for (uint32_t i = 0; i < sv.num_triangles; ++i) tri_hit(sv.triangles[i], sh);
        if (r.t > sh.t) {
            r.t = sh.t;
            r.mat = sh.mat;
            r.N = sh.N;
            r.inside = sh.inside;
            vox = -1;
            changed = true;
        }
    }
    *vox_io = vox;
    return changed;
}

// Renderer::IsOccluded, renderer.cpp:209-243 (scalar transforms, exact 1/D).  The linear
// volume loop: through the instance TLAS it measured slower (C4 IsOccluded 2.67 vs 2.57 ms:
// most shadow rays end in the world volume, the rest cross the instance lattice).
// first: the volume the loop starts at (k_shadow_slots: 1, after the shadow pool walked the
// world, volume 0).  The instances alone through the TLAS (the world's walk left to the pool)
// were slower too: C4 48.6-48.9 vs 47.2-47.4 ms per step at 5 waves/SIMD (8 spilled VGPRs),
// 50.4-50.6 at 4 (round 3, three interleaved runs).
__device__ __forceinline__ bool is_occluded(const SceneView& sv, const Ray& r, Counters& k, uint32_t first = 0) {
    bool occ = false;
    const f3 inv = world_inv(r.D);
    auto visit = [&](uint32_t i) {
        if (misses_volume(sv.vbounds, i, r.O, inv, r.t)) return true;  // no cell read
        const vpx_volume& vol = sv.volumes[i];
        ORay o;
        o.O = xform_pos(r.O, vol.inv_matrix);
        o.D = xform_vec(r.D, vol.inv_matrix);
        o.rD = mk(__fdiv_rn(1.0f, o.D.x), __fdiv_rn(1.0f, o.D.y), __fdiv_rn(1.0f, o.D.z));
        const DevGrid g = sv.grids[vol.grid_id];
        Dda s;
        if (!dda_setup(vol, g.n, o, s)) return true;
        skip::Walk w = to_walk(s);
        // first solid cell with t < bound: occluded, the reference returns (no later volume)
        occ = walk_wave<16, kSkipwShadow, kMincShadow, kRunShadow>(grid_view(g), w, r.t, k.cells);
        return !occ;
    };
    for (uint32_t i = first; i < sv.num_volumes && !occ; ++i) visit(i);
    if (occ) return true;
    for (uint32_t i = 0; i < sv.num_spheres; ++i)
        if (sphere_is_hit(sv.spheres[i], r)) return true;
    for (uint32_t i = 0; i < sv.num_triangles; ++i)
        if (tri_is_hit(sv.triangles[i], r)) return true;
    return false;
}

__device__ __forceinline__ bool shadow(const SceneView& sv, const Ray& r, Counters& k) {
    ++k.shadow;
    return is_occluded(sv, r, k);
}

__device__ __forceinline__ f3 albedo(const SceneView& sv, uint32_t m) { return ld3(sv.materials[m].albedo); }

// atan2_approximation2, template/tmpl8math.cpp:405-426.  ONEQTR_PI / THRQTR_PI are the
// float PI (common.h:8) divided in double and stored as float.
__device__ __forceinline__ float atan2_approx(float y, float x) {
    const float q1 = (float)((double)kPi / 4.0), q3 = (float)(3.0 * (double)kPi / 4.0);
    const float ay = fabsf(y) + 1e-10f;
    float r, angle;
    if (x < 0.0f) {
        r = __fdiv_rn(x + ay, ay - x);
        angle = q3;
    } else {
        r = __fdiv_rn(x - ay, x + ay);
        angle = q1;
    }
    angle += (0.1963f * r * r - 0.9817f) * r;
    return y < 0.0f ? -angle : angle;
}

// FastAcos, template/tmpl8math.cpp:429-443 (float arithmetic; the first constant is a
// double literal rounded to float).
__device__ __forceinline__ float fast_acos(float x) {
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
    ret = ret - 2.0f * negate * ret;
    return negate * 3.14159265358979f + ret;
}

// Renderer::SampleSky, renderer.cpp:2308-2326 (and SampleSkyReproject :2328-2346, whose
// albedo is the same value).  INV2PI / INVPI: common.h:13-14.  The index arithmetic wraps
// like the x86 reference; the only out-of-range index (a NaN direction, cvttss2si ->
// INT_MIN) is clamped to the image instead of reading outside it.
__device__ __forceinline__ f3 sample_sky(const SceneView& sv, f3 d) {
    if (!sv.sky_tex) return ld3(sv.sky);
    const float uf = (float)sv.sky_w * atan2_approx(d.z, d.x) * 0.15915494309189533576888f - 0.5f;
    const int u = trunc_i32(uf);
    const float vf = (float)sv.sky_h * fast_acos(d.y) * 0.31830988618379067153777f - 0.5f;
    const int v = trunc_i32(vf);
    const int32_t lin = (int32_t)((uint32_t)u + (uint32_t)v * sv.sky_w);
    uint32_t idx = lin > 0 ? (uint32_t)lin : 0u;
    const uint32_t last = sv.sky_w * sv.sky_h - 1u;
    idx = idx < last ? idx : last;
    const float* px = sv.sky_px + 3u * (uint64_t)idx;
    return mk(sv.sky_hdr * px[0], sv.sky_hdr * px[1], sv.sky_hdr * px[2]);
}

// RandomDirection (tmpl8math.cpp:76-93), RandomSphereSample (tmpl8math.h:2502-2511),
// DiffuseReflection (tmpl8math.h:2518-2528; argument order left to right).
__device__ __forceinline__ f3 random_direction(Rng& g) {
    for (;;) {
        const float a = g.next(), b = g.next(), c = g.next();
        const f3 p = mk(a, b, c);
        if (dot(p, p) < 1) return normalize(p);
    }
}
__device__ __forceinline__ f3 random_sphere_sample(Rng& g) {
    const float theta = g.next() * 2.0f * kPi;
    const float phi = g.next() * kPi;
    const float r = g.next();
    float sp, cp, st, ct;
    dm::sincos(phi, sp, cp);
    dm::sincos(theta, st, ct);
    return mk(r * sp * ct, r * sp * st, r * cp);
}
__device__ __forceinline__ f3 diffuse_reflection(Rng& g, f3 n) {
    f3 r;
    do {
        const float a = g.next() * 2.0f - 1.0f;
        const float b = g.next() * 2.0f - 1.0f;
        const float c = g.next() * 2.0f - 1.0f;
        r = mk(a, b, c);
    } while (dot(r, r) > 1);
    if (dot(r, n) < 0) r = r * -1.0f;
    return normalize(r);
}

// Reflect / Refract (renderer.cpp:913-925), Schlick (:1588-1594, :1611-1616).
__device__ __forceinline__ f3 reflect(f3 d, f3 n) { return d - (n * 2.0f) * dot(n, d); }
__device__ __forceinline__ f3 refract(f3 d, f3 n, float ratio) {
    const float c = smin(dot(-d, n), 1.0f);
    const f3 rper = (d + n * c) * ratio;
    const f3 rpar = n * (-sqrtf(fabsf(1.0f - dot(rper, rper))));
    return rper + rpar;
}
__device__ __forceinline__ float schlick(float cosine, float ior) {
    float r0 = __fdiv_rn(1 - ior, 1 + ior);
    r0 = r0 * r0;
    return r0 + (1 - r0) * cr_pow5(1 - cosine);
}
__device__ __forceinline__ float schlick_nonmetal(float cosine) {
    const float r0 = 0.04f;
    return r0 + (1 - r0) * cr_pow5(1 - cosine);
}

// Light evaluation: PointLightEvaluate (renderer.cpp:102-131), AreaLightEvaluation
// (:161-207), SpotLightEvaluate (:133-159), DirectionalLightEvaluate (:315-338),
// Illumination (:738-764).
__device__ __noinline__ f3 illumination(const SceneView& sv, const Ray& r, Rng& g, Counters& k) {
    const uint64_t pc = sv.num_points, scn = sv.num_spots, ac = sv.num_areas;
    const uint64_t lc = pc + scn + ac + 1;
    const uint64_t idx = (uint64_t)(g.next() * (float)lc);
    const f3 ip = ray_point(r);
    const f3 n = r.N;
    const f3 kd = albedo(sv, r.mat);
    f3 inc = mk(0.f, 0.f, 0.f);
    if (idx < pc) {
        const vpx_point_light& l = sv.points[idx];
        const f3 dir = ld3(l.position) - ip;
        const float dst = length(dir);
        const f3 dn = dir * __fdiv_rn(1.0f, dst);
        const float c = dot(dn, n);
        if (!(c <= 0.0f)) {  // `if (cosTheta <= 0) return 0` (NaN continues)
            const f3 li = (ld3(l.color) * smax(0.0f, c)) * __fdiv_rn(1.0f, dst * dst);
            Ray sh = make_ray(offset_ray(ip, n), dn);
            sh.t = dst;
            if (!shadow(sv, sh, k)) inc = li * kd;
        }
    } else if (idx < ac + pc) {
        const vpx_area_light& l = sv.areas[idx - pc];
        const f3 center = ld3(l.position);
        const float radius = l.radius;
        const f3 point = offset_ray(ip, n);
        f3 acc = mk(0.f, 0.f, 0.f);
        for (int i = 0; i < sv.area_samples; ++i) {
            f3 rp = random_direction(g);
            rp = rp * radius;
            rp = rp + center;
            const f3 dir = rp - ip;
            const float dst = length(dir);
            const f3 dn = dir * __fdiv_rn(1.0f, dst);
            const float c = dot(dn, n);
            if (c <= 0) continue;
            Ray sh = make_ray(point, dn);
            sh.t = dst;
            if (shadow(sv, sh, k)) continue;
            f3 li = ld3(l.color) * c;
            li = li * l.color_multiplier;
            li = li * (radius * radius);
            li = li * kPi;
            li = li * 4.0f;
            li = li / (dst * dst);
            acc = acc + li;
        }
        acc = acc / (float)sv.area_samples;
        inc = acc * kd;
    } else if (idx < ac + scn + pc) {
        const vpx_spot_light& l = sv.spots[idx - ac - pc];
        const f3 dir = ld3(l.position) - ip;
        const float dst = length(dir);
        const f3 dn = dir / dst;
        const float c = dot(dn, ld3(l.direction));
        if (!(c <= l.angle)) {
            const float alpha = 1.0f - __fdiv_rn((1.0f - c) * 1.0f, 1.0f - l.angle);
            const f3 li = (ld3(l.color) * smax(0.0f, c)) / (dst * dst);
            Ray sh = make_ray(offset_ray(ip, n), dn);
            sh.t = dst;
            if (!shadow(sv, sh, k)) inc = (li * kd) * alpha;
        }
    } else {
        const f3 dir = -ld3(sv.dir.direction);
        const float c = dot(dir, n);
        if (!(c <= 0)) {
            const f3 li = ld3(sv.dir.color) * smax(0.0f, c);
            Ray sh = make_ray(offset_ray(ip, n), dir);
            if (!shadow(sv, sh, k)) inc = li * kd;
        }
    }
    return inc * (float)lc;
}

// Glass/smoke interior march in object space (renderer.cpp:1160-1173, 1266-1279).
template <int MODE>
__device__ __forceinline__ bool exit_march(const SceneView& sv, Ray& r, int32_t vox, Counters& k) {
    const vpx_volume& vol = sv.volumes[vox];
    ORay o;
    o.O = xform_pos(r.O, vol.inv_matrix);
    o.D = xform_vec(r.D, vol.inv_matrix);
    o.rD = mk(__fdiv_rn(1.0f, o.D.x), __fdiv_rn(1.0f, o.D.y), __fdiv_rn(1.0f, o.D.z));
    const DevGrid g = sv.grids[vol.grid_id];
    Dda s;
    if (!dda_setup(vol, g.n, o, s)) return false;
    const WalkResult w = dda_walk<MODE>(g, s, 0.0f, k.cells);
    r.t = w.t;
    if (w.hit) {
        r.N = normal_voxel(o, w.t, g.n, vol.matrix);
        r.mat = w.cell;
    }
    return w.hit;
}

// One combine record per Trace level, folded bottom-up in trace_path():
//   kFormMulAdd:  v*a + b   (non-metal diffuse: incLight + Trace*albedo)
//   kFormAddMul:  (v + b)*a (model materials: (Trace + incLight)*albedo)
//   kFormMul:     v*a       (metal, glass, smoke)
//   kFormPass:    v         (non-metal specular)
enum { kFormMulAdd = 0, kFormAddMul = 1, kFormMul = 2, kFormPass = 3 };

struct Level {
    f3 a, b;
};

// Renderer::Trace(ray, depth) — renderer.cpp:1076-1328, recursion unrolled to a loop.
template <int LEVELS>
__device__ __forceinline__ f3 trace_path(const SceneView& sv, Ray ray, int depth, Rng& g, Counters& k) {
    Level lv[LEVELS];
    uint32_t forms = 0;
    int nl = 0;
    f3 leaf = mk(0.f, 0.f, 0.f);
    for (;;) {
        if (depth < 0) break;  // Trace(depth < 0) returns 0
        const int32_t vox = find_nearest(sv, ray, k);
        if (ray.mat == kNone) {
            leaf = sample_sky(sv, ray.D);
            break;
        }
        const uint32_t m = ray.mat;
        const vpx_material& mat = sv.materials[m];
        f3 a = mk(1.f, 1.f, 1.f), b = mk(0.f, 0.f, 0.f);
        uint32_t form;
        Ray next;
        if (m >= VPX_MAT_METAL_HIGH && m <= VPX_MAT_METAL_LOW) {  // :1103-1114
            const f3 refl = reflect(ray.D, ray.N);
            const f3 o = offset_ray(ray_point(ray), ray.N);
            next = make_ray(o, refl + random_sphere_sample(g) * mat.roughness);
            a = albedo(sv, m);
            form = kFormMul;
        } else if (m <= VPX_MAT_NON_METAL_PINK) {  // :1117-1144
            if (g.next() > schlick_nonmetal(dot(-ray.D, ray.N))) {
                const f3 rdir = ray.N + random_sphere_sample(g);
                b = illumination(sv, ray, g, k);
                next = make_ray(offset_ray(ray_point(ray), ray.N), rdir);
                a = albedo(sv, m);
                form = kFormMulAdd;
            } else {
                const f3 refl = reflect(ray.D, ray.N);
                const f3 o = offset_ray(ray_point(ray), ray.N);
                next = make_ray(o, refl + random_sphere_sample(g) * mat.roughness);
                form = kFormPass;
            }
        } else if (m == VPX_MAT_GLASS) {  // :1146-1209
            bool in_glass = ray.inside;
            const float ior = mat.ior;
            const float ratio = in_glass ? ior : __fdiv_rn(1.0f, ior);
            bool inside_volume = true;
            if (in_glass) {
                a = albedo(sv, m);
                if (vox >= 0) inside_volume = exit_march<kGlassExit>(sv, ray, vox, k);
            }
            if (!inside_volume) {
                ray.O = ray.O + ray.D * ray.t;
                ray.t = 0;
            }
            const float c = smin(dot(-ray.D, ray.N), 1.0f);
            const float s = sqrtf(1.0f - c * c);
            const bool cannot = ratio * s > 1.0f;
            f3 rdir, rn;
            if (cannot || schlick(c, ratio) > g.next()) {
                rdir = reflect(ray.D, ray.N);
                rn = ray.N;
            } else {
                rdir = refract(ray.D, ray.N, ratio);
                in_glass = !in_glass;
                rn = -ray.N;
            }
            next = make_ray(offset_ray(ray_point(ray), rn), rdir);
            next.inside = in_glass;
            form = kFormMul;
        } else if (m <= VPX_MAT_SMOKE_PLAYER) {  // smoke :1210-1314
            f3 color = mk(1.f, 1.f, 1.f);
            bool in_glass = ray.inside;
            bool inside_volume = true;
            float intensity = 0.f, dist = 0.f;
            if (vox == 0) (void)illumination(sv, ray, g, k);  // player light probe :1228-1240
            if (in_glass) {
                intensity = mat.emissive;
                color = albedo(sv, m);
                if (vox >= 0) inside_volume = exit_march<kSmokeExit>(sv, ray, vox, k);
                dist = ray.t;
            }
            const float threshold = g.next() * 100.0f - intensity;
            if (g.next() * dist > threshold) {
                const float lo = ray.t * .45f, hi = ray.t;
                const float tt = lo + g.next() * (hi - lo);
                ray.O = ray.O + ray.D * tt;
                ray.D = random_direction(g);
                ray.t = 0;
            }
            const f3 flipped = mk(1.f, 1.f, 1.f) - color;
            const f3 e = flipped * ((-dist) * intensity);
            a = mk(cr_exp(e.x), cr_exp(e.y), cr_exp(e.z));
            if (!inside_volume) {
                ray.O = ray.O + ray.D * ray.t;
                ray.t = 0;
            }
            const f3 rdir = refract(ray.D, ray.N, 1.0f);
            next = make_ray(offset_ray(ray_point(ray), -ray.N), rdir);
            next.inside = !in_glass;
            form = kFormMul;
        } else if (m == VPX_MAT_EMISSIVE) {  // :1315-1316
            leaf = albedo(sv, m) * mat.emissive;
            break;
        } else {  // model materials :1319-1326
            const f3 rdir = diffuse_reflection(g, ray.N);
            b = illumination(sv, ray, g, k);
            next = make_ray(offset_ray(ray_point(ray), ray.N), rdir);
            a = albedo(sv, m);
            form = kFormAddMul;
        }
        if (nl < LEVELS) {
            lv[nl].a = a;
            lv[nl].b = b;
            forms |= form << (2 * nl);
            ++nl;
        }
        ray = next;
        --depth;
    }
    f3 v = leaf;
    for (int i = nl - 1; i >= 0; --i) {
        const uint32_t form = (forms >> (2 * i)) & 3u;
        const f3 a = lv[i].a, b = lv[i].b;
        if (form == kFormMulAdd)
            v = b + v * a;
        else if (form == kFormAddMul)
            v = (v + b) * a;
        else if (form == kFormMul)
            v = v * a;
    }
    return v;
}

}  // namespace vpx
