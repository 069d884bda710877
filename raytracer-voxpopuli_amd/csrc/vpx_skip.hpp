// vpx_skip.hpp — exact empty-space skipping for the reference DDA (host + device).
//
// The reference march (Scene::FindNearest / IsOccluded, template/scene.cpp:751-811,
// 1009-1047) advances three float accumulators tmax.{x,y,z} += tdelta one cell at a time
// and always steps the axis with the smallest head (ties: z, then y, then x —
// `x<y ? (x<z ? x : z) : (y<z ? y : z)`).  The visited cells, the t of the first solid
// cell and the number of cells visited are therefore a pure function of the three
// sequences A(i+1) = fl(A(i) + d) and of their merge in (value, z>y>x) order.
//
// Inside one binade [2^E, 2^(E+1)) every A(i) is a multiple of u = 2^(E-23), and as long
// as the exact sum stays below 2^(E+1), fl(A + d) = A + c*u with c = d/u rounded to the
// nearest integer (no tie).  So A(k) and "how many A(i) lie below T" are O(1) per binade
// instead of O(k) — exactly, bit for bit.  Ties, stagnation, non-positive or non-finite
// values fall back to single IEEE additions (or to the cell-by-cell march).
//
// walk_skip() uses that to cross boxes of empty cells in one jump: it finds the merged
// event that leaves the box, counts the events before it per axis, and lands on the
// reference state just before that event, adding the skipped cells to the count.  The
// boxes come from a directional distance field over 4^3 bricks (an empty brick stores,
// per ray octant, the side of the largest empty cube of bricks that starts at it and
// grows in that octant's direction).  Cells in non-empty bricks are marched one by one.
// Results equal the cell-by-cell march exactly.
#pragma once

#include <stdint.h>

#ifndef __HIP_DEVICE_COMPILE__
#include <cstring>
#endif

#if defined(__HIPCC__)
#define VPX_HD __host__ __device__ __forceinline__
#else
#define VPX_HD inline
#endif

namespace vpx {
namespace skip {

VPX_HD uint32_t fbits(float f) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __float_as_uint(f);
#else
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
#endif
}
VPX_HD float bitsf(uint32_t u) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __uint_as_float(u);
#else
    float f;
    std::memcpy(&f, &u, 4);
    return f;
#endif
}

// Exact a / b for a, b < 2^26, b >= 1, given rb ~ 1/b within 2^-20 relative.  The device
// has no integer divider: two reciprocal-multiply estimates plus one integer correction.
VPX_HD uint32_t udiv_rcp(uint32_t a, uint32_t b, float rb) {
    int32_t q = (int32_t)((float)a * rb);
    int32_t r = (int32_t)a - q * (int32_t)b;  // |r| < 16 b
    q += (int32_t)((float)r * rb);
    r = (int32_t)a - q * (int32_t)b;  // |r| < 2 b
    if (r < 0) q -= 1, r += (int32_t)b;
    if (r < 0) q -= 1, r += (int32_t)b;
    if (r >= (int32_t)b) q += 1, r -= (int32_t)b;
    if (r >= (int32_t)b) q += 1;
    return (uint32_t)q;
}

VPX_HD uint32_t udiv(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return udiv_rcp(a, b, __builtin_amdgcn_rcpf((float)b));
#else
    return a / b;
#endif
}

// Closed-form segment of A(i+1) = fl(A(i) + d) starting at A > 0 (normal, finite):
// A = b*2^(E-23) with b in [2^23, 2^24).  ok=false: this step must be a plain addition.
struct Seg {
    uint32_t b;      // integer significand of A
    uint32_t c;      // increment in ulps
    uint32_t m;      // closed-form steps available in this binade (>= 1 when ok)
    uint32_t ebits;  // biased exponent of A
    bool ok;
    bool stuck;      // fl(A + d) == A forever
};

VPX_HD Seg segment(float a, float d) {
    Seg s{0u, 0u, 0u, 0u, false, false};
    const uint32_t ab = fbits(a), db = fbits(d);
    const uint32_t ea = ab >> 23, ed = db >> 23;  // sign bits are 0 (callers ensure a,d > 0)
    if (ea == 0 || ea >= 255 || ed == 0 || ed >= 255) return s;  // zero/denormal/inf/nan: single step
    s.ebits = ea;
    s.b = (ab & 0x7fffffu) | 0x800000u;
    const uint32_t md = (db & 0x7fffffu) | 0x800000u;
    if (ed >= ea) return s;  // d >= 2^E: at most a few steps per binade, do them one by one
    const uint32_t sh = ea - ed;  // >= 1
    if (sh > 25) {                // d < u/2: A + d rounds back to A (md < 2^24 <= 2^(sh-1))
        s.ok = true;
        s.stuck = true;
        return s;
    }
    uint32_t c = md >> sh;
    const uint32_t rem = md & ((1u << sh) - 1u), half = 1u << (sh - 1);
    if (rem == half) return s;  // exact tie: rounding alternates with parity -> single step
    if (rem > half) ++c;
    if (c == 0) {
        s.ok = true;
        s.stuck = true;
        return s;
    }
    // step i -> i+1 is closed-form while b + (i+1)*c <= 2^24 - 1 (exact sum < 2^(E+1))
    const uint32_t room = 0xffffffu - s.b;
    s.m = udiv(room, c);
    if (s.m == 0) return s;
    s.c = c;
    s.ok = true;
    return s;
}

VPX_HD float seg_value(uint32_t b, uint32_t ebits) {
    // b may have reached 2^24 only through an exact closed-form landing below 2^24 - 1,
    // so it is still a valid significand of this binade.
    return bitsf((ebits << 23) | (b & 0x7fffffu));
}

// A(k): k accumulations of d onto a (a, d > 0).  Exact.  With a cap, returns early with
// some A(j) > cap (j <= k) once the sequence exceeds it (then A(k) > cap too).
VPX_HD float jump(float a, float d, uint32_t k, float cap = 3.4e38f) {
    float A = a;
    while (k > 0) {
        if (!(A < 3.0e38f) || A > cap) return A;  // inf stays inf; beyond the cap
        const Seg s = segment(A, d);
        if (!s.ok) {
            A = A + d;
            --k;
            continue;
        }
        if (s.stuck) return A;
        const uint32_t st = k < s.m ? k : s.m;
        A = seg_value(s.b + st * s.c, s.ebits);
        k -= st;
    }
    return A;
}

// #{ i in [0, kmax) : A(i) < T }  (strict)  or  A(i) <= T  (!strict).  Exact.
VPX_HD uint32_t count_below(float a, float d, float T, bool strict, uint32_t kmax) {
    float A = a;
    uint32_t i = 0;
    while (i < kmax) {
        const bool below = strict ? (A < T) : (A <= T);
        if (!below) return i;
        if (!(A < 3.0e38f)) return kmax;  // A = inf <= T = inf: every later term equal
        const Seg s = segment(A, d);
        if (!s.ok) {
            A = A + d;
            ++i;
            continue;
        }
        if (s.stuck) return kmax;  // constant and below T forever
        // A(i+j) = (b + j c) u for j = 0..m.  Smallest j >= 1 with A(i+j) not below T.
        const uint32_t left = kmax - i;
        const uint32_t lim = left < s.m ? left : s.m;
        const uint32_t tb = fbits(T);
        uint32_t jj = 0xffffffffu;
        if ((tb >> 23) == s.ebits) {  // T in the same binade: T = t*u with integer t
            const uint32_t t = (tb & 0x7fffffu) | 0x800000u;  // t > b (A < T) or t >= b
            // strict: b + j c >= t ; non-strict: b + j c > t
            const uint32_t need = strict ? udiv(t - s.b + s.c - 1u, s.c) : udiv(t - s.b, s.c) + 1u;
            jj = need;
        } else if ((tb >> 23) < s.ebits || (tb >> 31)) {
            jj = 1;  // cannot happen (A below T), kept for safety
        }
        if (jj <= lim) return i + jj;
        A = seg_value(s.b + lim * s.c, s.ebits);
        i += lim;
    }
    return kmax;
}

// count_below plus the sequence values around the stop: returns n, sets Aend = A(n) and
// Aprev = A(n-1) (Aprev unspecified when n == 0).
VPX_HD uint32_t count_below2(float a, float d, float T, bool strict, uint32_t kmax, float& Aend, float& Aprev) {
    float A = a, P = a;
    uint32_t i = 0;
    while (i < kmax) {
        const bool below = strict ? (A < T) : (A <= T);
        if (!below) break;
        if (!(A < 3.0e38f)) {  // inf: constant from here on
            P = A;
            i = kmax;
            break;
        }
        const Seg s = segment(A, d);
        if (!s.ok) {
            P = A;
            A = A + d;
            ++i;
            continue;
        }
        if (s.stuck) {
            P = A;
            i = kmax;
            break;
        }
        const uint32_t left = kmax - i;
        const uint32_t lim = left < s.m ? left : s.m;
        const uint32_t tb = fbits(T);
        uint32_t jj = 0xffffffffu;
        if ((tb >> 23) == s.ebits) {
            const uint32_t t = (tb & 0x7fffffu) | 0x800000u;
            jj = strict ? udiv(t - s.b + s.c - 1u, s.c) : udiv(t - s.b, s.c) + 1u;
        }
        const uint32_t st = jj <= lim ? jj : lim;  // st >= 1
        P = seg_value(s.b + (st - 1u) * s.c, s.ebits);
        A = seg_value(s.b + st * s.c, s.ebits);
        i += st;
        if (jj <= lim) break;
    }
    Aend = A;
    Aprev = P;
    return i;
}

}  // namespace skip
}  // namespace vpx

namespace vpx {
namespace skip {

// A grid as the skipping walker sees it: the MatType bytes and two occupancy levels.
// l2 (16^3 macros): bit per child brick, set <=> the brick holds a solid cell.
// l1 (4^3 bricks): for an occupied brick, bit lx + 4ly + 16lz per solid cell; for an
// empty brick, its distance-field word: byte o (octant o = [sx<0] | [sy<0]<<1 | [sz<0]<<2)
// = k >= 1 such that the k^3 bricks from this one toward the octant are all empty (bricks
// outside the grid count as empty), capped at 255.
// dfp (optional): the distance field again as 8 octant planes of one byte per brick (plane
// o at dfp + o * plane, brick at blk_index), 0 for an occupied brick — a walk reads only
// its own octant's plane, 1 byte per brick instead of an 8-byte word (classify_dfp).
struct GridView {
    const uint8_t* cells;
    const uint64_t* l1;
    const uint64_t* l2;
    uint32_t n, nb1, nb2, nb3;
    const uint8_t* dfp;
    uint64_t plane;
};

struct Walk {
    uint32_t X, Y, Z;
    float t, tx, ty, tz;
    float dx, dy, dz;
    int32_t sx, sy, sz;
    uint32_t osh;  // 8 x the ray's octant: the shift of its byte in a distance-field word
    uint64_t m1, m2;  // the level words of the current cell's brick / macro (set by classify)
};

// Reset the level words and set the octant (after X..sz are set).
VPX_HD void walk_begin(Walk& w) {
    w.m1 = w.m2 = 0ull;
    w.osh = ((w.sx < 0 ? 1u : 0u) | (w.sy < 0 ? 2u : 0u) | (w.sz < 0 ? 4u : 0u)) * 8u;
}


// Occupancy-level layout.  l1 (bricks) and l2 (macros) are stored BLOCKED: the 64 words
// of one parent (a 4x4x4 group of blocks) are contiguous, parents in linear order.  A
// wave's rays then share 128-byte lines across y/z neighbours too, and a parent's bits
// come from 64 consecutive child words.  `np` = parents per axis.  np <= 256 (grids up to 4096^3): every product fits the 24-bit multiplier.
VPX_HD uint32_t blk_index(uint32_t bx, uint32_t by, uint32_t bz, uint32_t np) {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t parent = __umul24(bz >> 2, __umul24(np, np)) + __umul24(by >> 2, np) + (bx >> 2);
#else
    const uint32_t parent = (bz >> 2) * np * np + (by >> 2) * np + (bx >> 2);
#endif
    return (parent << 6) | (bx & 3u) | ((by & 3u) << 2) | ((bz & 3u) << 4);
}

VPX_HD uint64_t load_mask(const uint64_t* p, uint32_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
    return ((const __attribute__((address_space(1))) uint64_t*)p)[i];
#else
    return p[i];
#endif
}

VPX_HD uint32_t lin_index(uint32_t x, uint32_t y, uint32_t z, uint32_t nb) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul24(z, __umul24(nb, nb)) + __umul24(y, nb) + x;
#else
    return z * nb * nb + y * nb + x;
#endif
}

// Smallest distance-field cube (in bricks) worth a skip; smaller ones are stepped through.
constexpr uint32_t kMinCube = 2;
// 0: solid cell, 1: empty cell of an occupied brick (step), 2: empty brick with a
// distance-field cube of at least kMinCube bricks (skip it: df_box), 3: empty brick with a
// smaller cube (step; every cell of the brick is empty).  Both level words are loaded at
// every call and the class is formed with selects: the loads hit the cache while the
// brick does not change, and a per-brick key cache with load branches measured 3.5 %
// slower on C1 (the divergent branches cost more than the loads they avoid).
template <uint32_t MINC = kMinCube>
VPX_HD int classify(Walk& w, const GridView& g) {
    const uint32_t X = w.X, Y = w.Y, Z = w.Z;
    w.m2 = load_mask(g.l2, blk_index(X >> 4, Y >> 4, Z >> 4, g.nb3));
    w.m1 = load_mask(g.l1, blk_index(X >> 2, Y >> 2, Z >> 2, g.nb2));
    const uint32_t bb = ((X >> 2) & 3u) | (((Y >> 2) & 3u) << 2) | (((Z >> 2) & 3u) << 4);
    const uint32_t cb = (X & 3u) | ((Y & 3u) << 2) | ((Z & 3u) << 4);
    const int cell = ((w.m1 >> cb) & 1ull) ? 0 : 1;
    const int brick = ((uint32_t)(w.m1 >> w.osh) & 255u) >= MINC ? 2 : 3;
    return ((w.m2 >> bb) & 1ull) ? cell : brick;
}

// The same class from the octant plane `pl` (g.dfp + octant * g.plane): one byte per step
// from a plane an eighth the size of l1, and the brick's cell mask only when the byte says
// occupied (0) — a dependent second load, but walks step mostly through empty bricks.
// For an empty brick m1 gets the byte itself (the cube, unshifted: cube_dfp reads it back
// without the octant shift, so the walk loop keeps no shift live).
VPX_HD uint32_t load_u8(const uint8_t* p, uint32_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
    return ((const __attribute__((address_space(1))) uint8_t*)p)[i];
#else
    return p[i];
#endif
}
// (k: the brick's plane byte, already loaded)
template <uint32_t MINC = kMinCube>
VPX_HD int classify_dfp_byte(Walk& w, const GridView& g, uint32_t k) {
    const uint32_t X = w.X, Y = w.Y, Z = w.Z;
    if (k == 0u) {
        const uint32_t bi = blk_index(X >> 2, Y >> 2, Z >> 2, g.nb2);
        w.m1 = load_mask(g.l1, bi);
        const uint32_t cb = (X & 3u) | ((Y & 3u) << 2) | ((Z & 3u) << 4);
        return ((w.m1 >> cb) & 1ull) ? 0 : 1;
    }
    w.m1 = k;
    return k >= MINC ? 2 : 3;
}
template <uint32_t MINC = kMinCube>
VPX_HD int classify_dfp(Walk& w, const GridView& g, const uint8_t* pl) {
    return classify_dfp_byte<MINC>(w, g, load_u8(pl, blk_index(w.X >> 2, w.Y >> 2, w.Z >> 2, g.nb2)));
}
// classify_dfp with the plane named by its first parent, opar = octant * nb2^3: the planes
// are consecutive and parent-major, so octant and parent fold into one 32-bit parent index
// (< 2^27 up to 4096^3 grids) and only the byte offset is formed in 64 bits — a walk keeps
// one 32-bit value live for its plane instead of a 64-bit pointer.
template <uint32_t MINC = kMinCube>
VPX_HD int classify_dfp_o(Walk& w, const GridView& g, uint32_t opar) {
    const uint32_t bx = w.X >> 2, by = w.Y >> 2, bz = w.Z >> 2, np = g.nb2;
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t parent = opar + __umul24(bz >> 2, __umul24(np, np)) + __umul24(by >> 2, np) + (bx >> 2);
#else
    const uint32_t parent = opar + (bz >> 2) * np * np + (by >> 2) * np + (bx >> 2);
#endif
    const uint64_t i = (uint64_t)parent << 6 | ((bx & 3u) | ((by & 3u) << 2) | ((bz & 3u) << 4));
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t k = ((const __attribute__((address_space(1))) uint8_t*)g.dfp)[i];
#else
    const uint32_t k = g.dfp[i];
#endif
    return classify_dfp_byte<MINC>(w, g, k);
}
// The first parent of octant o's plane (classify_dfp_o).
VPX_HD uint32_t plane_parent(const GridView& g, uint32_t o) { return o * (g.nb2 * g.nb2 * g.nb2); }
// The distance-field cube (in bricks) of an empty brick from m1: after classify (the l1
// word, byte at the octant's shift) / after classify_dfp (the plane byte itself).
VPX_HD uint32_t cube_l1(const Walk& w) { return (uint32_t)(w.m1 >> w.osh) & 255u; }
VPX_HD uint32_t cube_dfp(const Walk& w) { return (uint32_t)w.m1 & 255u; }
// The empty box of a class-2 cell: its brick's distance-field cube `k` toward the ray's
// octant, clipped to the grid.  Only the faces ahead of the ray matter to skip_box, so the
// faces behind are put at the current cell.
VPX_HD void df_box(const Walk& w, uint32_t n, uint32_t k, uint32_t lo[3], uint32_t hi[3]) {
    const uint32_t k4 = k * 4u;
    const uint32_t c[3] = {w.X, w.Y, w.Z};
    const int32_t sg[3] = {w.sx, w.sy, w.sz};
    for (int k = 0; k < 3; ++k) {
        const uint32_t b = c[k] & ~3u;
        const uint32_t up = b + k4 - 1u, dn = b + 4u > k4 ? b + 4u - k4 : 0u;
        lo[k] = sg[k] > 0 ? c[k] : dn;
        hi[k] = sg[k] > 0 ? (up < n - 1u ? up : n - 1u) : c[k];
    }
}

// The chosen axis' cell and head advance (shared by both forms of step1).
VPX_HD bool step1_commit(Walk& w, uint32_t n, bool ax, bool ay, bool az) {
    w.X += ax ? (uint32_t)w.sx : 0u;
    w.Y += ay ? (uint32_t)w.sy : 0u;
    w.Z += az ? (uint32_t)w.sz : 0u;
    w.tx = ax ? w.tx + w.dx : w.tx;
    w.ty = ay ? w.ty + w.dy : w.ty;
    w.tz = az ? w.tz + w.dz : w.tz;
    const uint32_t m = w.X > w.Y ? w.X : w.Y;
    return (m > w.Z ? m : w.Z) < n;
}

// One reference step (scene.cpp:773-802), branch-free; false = left the grid.
// MIN2: the reference's axis choice `x<y ? (x<z ? x : z) : (y<z ? y : z)` read as
// "a = x<y ? x : y; a<z ? (the axis of a) : z" — the same axis for every input, NaN and ties
// included (x<y false -> a = y, then y<z; x<y true -> x<z), with two compares and one select
// instead of three compares and a select chain.
// The walkers choose per walk kind (bit 18 of their RUN word, vpx_trace.hpp): with the
// shadow walkers' 72-VGPR budget this form spilled more and measured slower on C3.
template <bool MIN2 = true>
VPX_HD bool step1(Walk& w, uint32_t n) {
  if (MIN2) {
    const bool xy = w.tx < w.ty;
    const float a = xy ? w.tx : w.ty;
    const bool nz = a < w.tz;
    const bool ax = xy && nz;
    const bool ay = !xy && nz;
    const bool az = !nz;
    w.t = nz ? a : w.tz;
    return step1_commit(w, n, ax, ay, az);
  }
    const bool xy = w.tx < w.ty, xz = w.tx < w.tz, yz = w.ty < w.tz;
    const bool ax = xy && xz;
    const bool ay = !xy && yz;
    const bool az = !(ax || ay);
    w.t = ax ? w.tx : (ay ? w.ty : w.tz);
    return step1_commit(w, n, ax, ay, az);
}

// Cross the empty box [lo, hi] (per axis, inclusive) around the current cell.
// 0: landed just before the event that leaves the box (cells += skipped visits);
// 1: the walk ends inside the box (bound reached; cells += visits); 2: not applicable.
VPX_HD int skip_box(Walk& w, const uint32_t lo[3], const uint32_t hi[3], float bound, uint32_t& cells) {
    const float h[3] = {w.tx, w.ty, w.tz};
    const float d[3] = {w.dx, w.dy, w.dz};
    const int32_t s[3] = {w.sx, w.sy, w.sz};
    const uint32_t c[3] = {w.X, w.Y, w.Z};
    uint32_t e[3];
    float approx[3];
    for (int k = 0; k < 3; ++k) {
        if (!(h[k] > 0.0f) || !(d[k] > 0.0f)) return 2;  // NaN, zero or negative: march instead
        e[k] = s[k] > 0 ? hi[k] - c[k] + 1u : c[k] - lo[k] + 1u;
        // A(e-1) ~ h + (e-1) d, relative error < (e+1) 2^-24 (< 6.2e-5 for e <= 1024)
        approx[k] = e[k] > 1u ? h[k] + (float)(e[k] - 1u) * d[k] : h[k];
    }
    // leaving event = smallest A_k(e_k - 1), ties -> z, then y, then x.  Decide on the
    // approximations when they are apart by more than their error; otherwise exactly.
    float V[3], Vp[3];
    bool exact[3] = {false, false, false};
    int a = (approx[2] <= approx[0] && approx[2] <= approx[1]) ? 2 : (approx[1] <= approx[0] ? 1 : 0);
    const float amin = approx[a];
    bool close = false;
    for (int k = 0; k < 3; ++k)
        if (k != a && !(approx[k] > amin * 1.0003f)) close = true;
    if (close) {
        for (int k = 0; k < 3; ++k) {
            count_below2(h[k], d[k], 3.4e38f, true, e[k] - 1u, V[k], Vp[k]);
            exact[k] = true;
        }
        a = (V[2] <= V[0] && V[2] <= V[1]) ? 2 : (V[1] <= V[0] ? 1 : 0);
    } else {
        count_below2(h[a], d[a], 3.4e38f, true, e[a] - 1u, V[a], Vp[a]);
        exact[a] = true;
    }
    const float vs = V[a];
    uint32_t nk[3];
    float head[3], prev[3];
    for (int k = 0; k < 3; ++k) {
        if (k == a) {
            nk[k] = e[k] - 1u;
            head[k] = V[k];
            prev[k] = Vp[k];
        } else {
            // axis k precedes axis a on ties iff k > a (priority z=2 > y=1 > x=0)
            nk[k] = count_below2(h[k], d[k], vs, k < a, e[k] - 1u, head[k], prev[k]);
        }
    }
    if (vs < bound) {
        float tl = w.t;
        bool moved = false;
        for (int k = 0; k < 3; ++k) {
            if (nk[k] == 0) continue;
            tl = moved ? (tl < prev[k] ? prev[k] : tl) : prev[k];
            moved = true;
        }
        if (moved) w.t = tl;
        w.tx = head[0], w.ty = head[1], w.tz = head[2];
        w.X += nk[0] * (uint32_t)w.sx;
        w.Y += nk[1] * (uint32_t)w.sy;
        w.Z += nk[2] * (uint32_t)w.sz;
        cells += nk[0] + nk[1] + nk[2];
        return 0;
    }
    uint32_t v = 1u;
    for (int k = 0; k < 3; ++k) v += count_below(h[k], d[k], bound, true, nk[k]);
    cells += v;
    return 1;
}

// ------------------------------------------------------- lean tier
// skip_box in straight-line integer code.  Each axis's sequence is put in closed form as
// up to two segments (its own binade, then the next one after one plain IEEE step), and
// the box is first clipped, per axis, to the events those two segments reach.  So every
// box is taken: where a sequence crosses more binades (rays that start near t = 0) the
// lane skips the clipped part now and the rest in later iterations.  Only a non-positive
// or NaN head is refused (2: the caller takes a plain step instead).  Boxes span at most
// 1024 cells per axis; every product formed is below 2^32 with both factors below 2^24,
// so it uses the full-rate 24-bit multiplier.

VPX_HD uint32_t mul24(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul24(a, b);
#else
    return a * b;
#endif
}

// a * b + c with a, b < 2^24 (full-rate v_mad_u32_u24; left to itself the compiler picks
// the quarter-rate 64-bit multiply-add for these).
VPX_HD uint32_t mad24(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
#else
    return a * b + c;
#endif
}

// The lean tier below names every operand before selecting between them: a conditional
// whose arm holds arithmetic becomes a divergent branch on the device, a select does not.

VPX_HD float rcp_approx(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcpf(x);
#else
    return 1.0f / x;
#endif
}

// Closed form of A -> fl(A + d) in A's binade, without branches, valid for i >= 1:
// A(i) = (b + i c) u.  Without a tie, c = round(d / u) and b is A's significand.  With a
// tie (d / u = c0 + 1/2 exactly) round-half-even makes every significand from A(1) on
// even, so from there the increment is c0 rounded up to even; b is then the base that
// reproduces A(1) = A + c0 + ((A + c0) & 1) (A(0) itself is read from the float).
VPX_HD bool seg_params_nb(float a, float d, uint32_t& b, uint32_t& c, uint32_t& e) {
    const uint32_t ab = fbits(a), db = fbits(d);
    const uint32_t ea = ab >> 23, ed = db >> 23;
    const uint32_t sh = ea - ed;  // meaningful when ok
    const uint32_t shc = sh > 24u ? 24u : (sh < 1u ? 1u : sh);
    const uint32_t md = (db & 0x7fffffu) | 0x800000u;
    const uint32_t rem = md & ((1u << shc) - 1u), half = 1u << (shc - 1u);
    const uint32_t c0 = md >> shc;
    const uint32_t b0 = (ab & 0x7fffffu) | 0x800000u;
    const bool tie = rem == half;
    c = tie ? c0 + (c0 & 1u) : c0 + (rem > half ? 1u : 0u);
    b = tie ? b0 + ((b0 + c0) & 1u) - (c0 & 1u) : b0;
    e = ea;
    return (ea - 1u < 254u) & (ed - 1u < 254u) & (ed < ea) & (sh <= 24u) & (c != 0u);
}

// ceil(p / c) clamped to 1025 (p <= 2^24 + 1, 1 <= c < 2^24).  q's error is far below 1
// (relative 2^-22, q <= 1024.5), so one correction each way makes it exact; the products
// stay below 2^25 (j ~ p / c, or c < 2^14 when clamped).
VPX_HD uint32_t ceil_div_cap_r(uint32_t p, uint32_t c, float rc) {  // rc ~ 1/c (2^-22 relative)
    const float q = (float)p * rc;
    uint32_t j = (uint32_t)(q < 1024.5f ? q : 1024.5f) + 1u;  // ceil(p/c) or one off, <= 1025
    j -= mul24(j - 1u, c) >= p ? 1u : 0u;
    j += mul24(j, c) < p ? 1u : 0u;
    return j < 1025u ? j : 1025u;
}
VPX_HD uint32_t ceil_div_cap(uint32_t p, uint32_t c) { return ceil_div_cap_r(p, c, rcp_approx((float)c)); }

// floor(r / c) clamped to 1024 (r < 2^24, 1 <= c < 2^24).
VPX_HD uint32_t floor_div_cap_r(uint32_t r, uint32_t c, float rc) {
    const float q = (float)r * rc;
    uint32_t m = (uint32_t)(q < 1024.5f ? q : 1024.5f);
    m -= ((m != 0u) & (mul24(m, c) > r)) ? 1u : 0u;
    m += mul24(m + 1u, c) <= r ? 1u : 0u;
    return m < 1024u ? m : 1024u;
}
VPX_HD uint32_t floor_div_cap(uint32_t r, uint32_t c) { return floor_div_cap_r(r, c, rcp_approx((float)c)); }

// First j >= 0 with (b + j c) u not below T (strict: >= T, else > T), clamped to 1025.
VPX_HD uint32_t seg_first_cap(uint32_t b, uint32_t c, uint32_t e, float T, bool strict) {
    const uint32_t tb = fbits(T), te = tb >> 23;
    const uint32_t need = ((tb & 0x7fffffu) | 0x800000u) + (strict ? 0u : 1u);
    const uint32_t q = ceil_div_cap(need - b, c);
    const uint32_t f = need <= b ? 0u : q;
    return te == e ? f : (te < e ? 0u : 1025u);
}

// One axis over the box: A(0..l) as one or two closed-form segments: A(i) = (b1 + i c1) u1
// for i <= m1, then (b2 + (i - m1 - 1) c2) u2 after the plain IEEE step m1 -> m1 + 1.
struct Axis {
    uint32_t b1, c1, e1, m1, b2, c2, e2, l;
};

// l = the events wanted inside the box, clipped to what the two segments reach (0 when
// not even the first applies: then only A(0) = h is read).  In three parts: the first
// segment (axis_seg1, sets fit1 = the events it reaches), the second (axis_seg2, returns
// the events both reach; skipped when no lane of the wave wants more than fit1 on any
// axis — its parameters are then never read: every index used is <= m1), the clip.
VPX_HD bool axis_seg1(float h, float d, Axis& a, uint32_t& fit1) {
    const bool ok1 = seg_params_nb(h, d, a.b1, a.c1, a.e1);
    // A(i), 1 <= i <= fit1, stay below 2^24 u (a tie base may be 2^24 itself: fit1 = 0)
    const uint32_t room = a.b1 <= 0xffffffu ? 0xffffffu - a.b1 : 0u;
    fit1 = floor_div_cap(room, a.c1 ? a.c1 : 1u);  // (c1 == 0: not ok1)
    a.b2 = 0u, a.c2 = 1u, a.e2 = 0u;
    return ok1;
}
VPX_HD uint32_t axis_seg2(float h, float d, Axis& a, uint32_t fit1) {
    const uint32_t amc = (a.e1 << 23) | (mad24(fit1, a.c1, a.b1) & 0x7fffffu);
    const uint32_t am = fit1 ? amc : fbits(h);
    const float A = bitsf(am) + d;  // the plain IEEE step into the next binade
    uint32_t b2;
    const bool ok2 = seg_params_nb(A, d, b2, a.c2, a.e2);
    const bool exact2 = b2 == ((fbits(A) & 0x7fffffu) | 0x800000u);  // closed form from j = 0
    a.b2 = b2;
    const uint32_t room2 = b2 <= 0xffffffu ? 0xffffffu - b2 : 0u;
    const uint32_t fit2 = floor_div_cap(room2, a.c2 ? a.c2 : 1u);
    return (ok2 & exact2) ? fit1 + 1u + fit2 : fit1;
}
VPX_HD void axis_clip(Axis& a, uint32_t l, bool ok1, uint32_t reach, uint32_t fit1) {
    const uint32_t lim = ok1 ? reach : 0u;
    a.l = l < lim ? l : lim;
    a.m1 = a.l < fit1 ? a.l : fit1;
}
// True when any lane of the wave (calling it together) passes true; the host: this call's.
VPX_HD bool any_lane(bool b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __ballot(b) != 0ull;
#else
    return b;
#endif
}

VPX_HD void axis_setup(float h, float d, uint32_t l, Axis& a) {
    const bool ok1 = seg_params_nb(h, d, a.b1, a.c1, a.e1);
    // A(i), 1 <= i <= fit1, stay below 2^24 u (a tie base may be 2^24 itself: fit1 = 0)
    const uint32_t room = a.b1 <= 0xffffffu ? 0xffffffu - a.b1 : 0u;
    const uint32_t fit1 = floor_div_cap(room, a.c1 ? a.c1 : 1u);  // (c1 == 0: not ok1)
    const uint32_t amc = (a.e1 << 23) | (mad24(fit1, a.c1, a.b1) & 0x7fffffu);
    const uint32_t am = fit1 ? amc : fbits(h);
    const float A = bitsf(am) + d;  // the plain IEEE step into the next binade
    uint32_t b2;
    const bool ok2 = seg_params_nb(A, d, b2, a.c2, a.e2);
    const bool exact2 = b2 == ((fbits(A) & 0x7fffffu) | 0x800000u);  // closed form from j = 0
    a.b2 = b2;
    const uint32_t room2 = b2 <= 0xffffffu ? 0xffffffu - b2 : 0u;
    const uint32_t fit2 = floor_div_cap(room2, a.c2 ? a.c2 : 1u);
    const uint32_t lim = ok1 ? ((ok2 & exact2) ? fit1 + 1u + fit2 : fit1) : 0u;
    a.l = l < lim ? l : lim;
    a.m1 = a.l < fit1 ? a.l : fit1;
}

VPX_HD float axis_at(const Axis& a, float h, uint32_t i) {
    const bool one = i <= a.m1;
    const uint32_t b1 = mad24(i, a.c1, a.b1), b2 = mad24(i - a.m1 - 1u, a.c2, a.b2);
    const uint32_t v = ((one ? a.e1 : a.e2) << 23) | ((one ? b1 : b2) & 0x7fffffu);
    return bitsf(i ? v : fbits(h));
}

// #{ i < cap : A(i) below T } (A increasing), cap <= a.l.  T's binade picks the segment.
VPX_HD uint32_t axis_count(const Axis& a, float h, float T, bool strict, uint32_t cap) {
    const bool h_below = strict ? h < T : h <= T;
    const bool s2 = (fbits(T) >> 23) > a.e1;  // every A(1..m1) is below T
    uint32_t f = seg_first_cap(s2 ? a.b2 : a.b1, s2 ? a.c2 : a.c1, s2 ? a.e2 : a.e1, T, strict);
    f = s2 ? a.m1 + 1u + f : (f < a.m1 + 1u ? f : a.m1 + 1u);
    f = h_below ? (f > 1u ? f : 1u) : 0u;  // index 0 is h itself
    return f < cap ? f : cap;
}

// Cross the empty box [lo, hi] around the current cell, clipped per axis as above (lo / hi
// receive the clipped box).  0: landed just before the event that leaves the clipped box
// (cells += skipped visits); 1: the walk ends inside it (cells += visits); 2: refused.
// SEG2_BRANCH: the second closed-form segment only when a lane of the wave needs it.
template <bool SEG2_BRANCH = true>
VPX_HD int skip_box_lean(Walk& w, uint32_t lo[3], uint32_t hi[3], float bound, uint32_t& cells) {
    if (!((w.tx > 0.0f) & (w.ty > 0.0f) & (w.tz > 0.0f))) return 2;
    Axis ax, ay, az;
    if (SEG2_BRANCH) {
    const uint32_t wx = w.sx > 0 ? hi[0] - w.X : w.X - lo[0], wy = w.sy > 0 ? hi[1] - w.Y : w.Y - lo[1],
                   wz = w.sz > 0 ? hi[2] - w.Z : w.Z - lo[2];
    uint32_t fx, fy, fz;
    const bool okx = axis_seg1(w.tx, w.dx, ax, fx), oky = axis_seg1(w.ty, w.dy, ay, fy),
               okz = axis_seg1(w.tz, w.dz, az, fz);
    uint32_t rx = fx, ry = fy, rz = fz;
    if (any_lane((okx & (wx > fx)) | (oky & (wy > fy)) | (okz & (wz > fz)))) {  // a box crosses a binade
        rx = axis_seg2(w.tx, w.dx, ax, fx);
        ry = axis_seg2(w.ty, w.dy, ay, fy);
        rz = axis_seg2(w.tz, w.dz, az, fz);
    }
    axis_clip(ax, wx, okx, rx, fx);
    axis_clip(ay, wy, oky, ry, fy);
    axis_clip(az, wz, okz, rz, fz);
    } else {
    axis_setup(w.tx, w.dx, w.sx > 0 ? hi[0] - w.X : w.X - lo[0], ax);
    axis_setup(w.ty, w.dy, w.sy > 0 ? hi[1] - w.Y : w.Y - lo[1], ay);
    axis_setup(w.tz, w.dz, w.sz > 0 ? hi[2] - w.Z : w.Z - lo[2], az);
    }
    const uint32_t lx = ax.l, ly = ay.l, lz = az.l;
    if (w.sx > 0) hi[0] = w.X + lx; else lo[0] = w.X - lx;
    if (w.sy > 0) hi[1] = w.Y + ly; else lo[1] = w.Y - ly;
    if (w.sz > 0) hi[2] = w.Z + lz; else lo[2] = w.Z - lz;
    const float Vx = axis_at(ax, w.tx, lx), Vy = axis_at(ay, w.ty, ly), Vz = axis_at(az, w.tz, lz);
    const int a = (Vz <= Vx && Vz <= Vy) ? 2 : (Vy <= Vx ? 1 : 0);
    const float vs = a == 2 ? Vz : (a == 1 ? Vy : Vx);
    const bool inside = vs < bound;
    const float T = inside ? vs : bound;
    // events of the other axes before the leaving event (axis k precedes a on ties iff
    // k > a), or, when the walk ends inside the box, before the bound (strict)
    uint32_t nx = axis_count(ax, w.tx, T, true, lx);
    uint32_t ny = axis_count(ay, w.ty, T, inside ? a == 2 : true, ly);
    uint32_t nz = axis_count(az, w.tz, T, inside ? false : true, lz);
    if (inside) {
        nx = a == 0 ? lx : nx;
        ny = a == 1 ? ly : ny;
        nz = a == 2 ? lz : nz;
        // t = the last event before the landing: the largest A_k(n_k - 1) over moved axes
        const float px = axis_at(ax, w.tx, nx - 1u), py = axis_at(ay, w.ty, ny - 1u), pz = axis_at(az, w.tz, nz - 1u);
        float tl = nx ? px : w.t;
        tl = ny ? ((nx && !(tl < py)) ? tl : py) : tl;
        tl = nz ? (((nx | ny) && !(tl < pz)) ? tl : pz) : tl;
        w.t = tl;
        w.tx = axis_at(ax, w.tx, nx), w.ty = axis_at(ay, w.ty, ny), w.tz = axis_at(az, w.tz, nz);
        w.X += nx * (uint32_t)w.sx;
        w.Y += ny * (uint32_t)w.sy;
        w.Z += nz * (uint32_t)w.sz;
        cells += nx + ny + nz;
        return 0;
    }
    // the counts relative to the leaving event bound the counts below `bound`
    const uint32_t cx = a == 0 ? lx : axis_count(ax, w.tx, vs, true, lx);
    const uint32_t cy = a == 1 ? ly : axis_count(ay, w.ty, vs, a == 2, ly);
    const uint32_t cz = a == 2 ? lz : axis_count(az, w.tz, vs, false, lz);
    cells += 1u + (nx < cx ? nx : cx) + (ny < cy ? ny : cy) + (nz < cz ? nz : cz);
    return 1;
}

// Scene::FindNearest (MODE nearest) / Scene::IsOccluded walk from an initialised state.
// Returns true at the first solid cell (w.t / w.X,Y,Z describe it).  Exact.  The device
// walker (walk_wave, vpx_trace.hpp) runs the same per-lane sequence.
VPX_HD bool walk_skip(const GridView& g, Walk& w, float bound, uint32_t& cells) {
    for (;;) {
        if (!(w.t < bound)) return false;
        const int cls = classify(w, g);
        if (cls == 0) {
            ++cells;
            return true;
        }
        if (cls == 2) {
            uint32_t lo[3], hi[3];
            df_box(w, g.n, cube_l1(w), lo, hi);
            if (skip_box_lean(w, lo, hi, bound, cells) == 1) return false;
        }
        ++cells;  // visit the (empty) current cell
        if (!step1(w, g.n)) return false;
    }
}

// Distance-field byte of an empty brick (x, y, z) for octant o from its 7 neighbours
// ahead (the recurrence both builders use): 1 + the minimum over the neighbours (0 for an
// occupied one, 255 outside [0, nb1)), capped at 255.  The k^3 cube at a brick is empty
// iff the brick and the (k-1)^3 cubes at its 7 neighbours ahead are.
template <class Occ, class Get>
VPX_HD uint8_t df_value(uint32_t x, uint32_t y, uint32_t z, uint32_t o, uint32_t nb1, Occ occ, Get get) {
    const int32_t s[3] = {(o & 1u) ? -1 : 1, (o & 2u) ? -1 : 1, (o & 4u) ? -1 : 1};
    uint32_t mn = 255;
    for (uint32_t j = 1; j < 8; ++j) {
        const uint32_t a = x + ((j & 1u) ? (uint32_t)s[0] : 0u), b = y + ((j & 2u) ? (uint32_t)s[1] : 0u),
                       c = z + ((j & 4u) ? (uint32_t)s[2] : 0u);
        const uint32_t v = (a < nb1 && b < nb1 && c < nb1) ? (occ(a, b, c) ? 0u : get(a, b, c, o)) : 255u;
        mn = v < mn ? v : mn;
    }
    return (uint8_t)(mn < 255u ? mn + 1u : 255u);
}

#if !defined(__HIP_DEVICE_COMPILE__)
// Host builder of the same levels (tests and tools).  Sizes: l1 nb2^3*64 words, l2
// nb3^3*64 words (nb1 = ceil(n/4), nb2 = ceil(nb1/4), nb3 = ceil(nb2/4)).
inline void build_masks_host(const uint8_t* cells, uint32_t n, uint64_t* l1, uint64_t* l2) {
    const uint32_t nb1 = (n + 3) / 4, nb2 = (nb1 + 3) / 4, nb3 = (nb2 + 3) / 4;
    std::memset(l1, 0, 8ull * nb2 * nb2 * nb2 * 64);
    std::memset(l2, 0, 8ull * nb3 * nb3 * nb3 * 64);
    for (uint64_t z = 0; z < n; ++z)
        for (uint64_t y = 0; y < n; ++y)
            for (uint64_t x = 0; x < n; ++x)
                if (cells[x + y * n + z * (uint64_t)n * n] != 255)
                    l1[blk_index((uint32_t)x >> 2, (uint32_t)y >> 2, (uint32_t)z >> 2, nb2)] |=
                        1ull << ((x & 3) + 4 * (y & 3) + 16 * (z & 3));
    for (uint32_t z = 0; z < nb1; ++z)
        for (uint32_t y = 0; y < nb1; ++y)
            for (uint32_t x = 0; x < nb1; ++x)
                if (l1[blk_index(x, y, z, nb2)])
                    l2[blk_index(x >> 2, y >> 2, z >> 2, nb3)] |= 1ull << ((x & 3) + 4 * (y & 3) + 16 * (z & 3));
    auto occ = [&](uint32_t x, uint32_t y, uint32_t z) {
        return (l2[blk_index(x >> 2, y >> 2, z >> 2, nb3)] >> ((x & 3) + 4 * (y & 3) + 16 * (z & 3))) & 1ull;
    };
    uint8_t* bytes = reinterpret_cast<uint8_t*>(l1);
    auto get = [&](uint32_t x, uint32_t y, uint32_t z, uint32_t o) -> uint32_t {
        return bytes[(size_t)blk_index(x, y, z, nb2) * 8 + o];
    };
    for (uint32_t o = 0; o < 8; ++o)  // sweep each octant from its far corner
        for (uint32_t fz = nb1; fz-- > 0;)
            for (uint32_t fy = nb1; fy-- > 0;)
                for (uint32_t fx = nb1; fx-- > 0;) {
                    const uint32_t x = (o & 1u) ? nb1 - 1 - fx : fx, y = (o & 2u) ? nb1 - 1 - fy : fy,
                                   z = (o & 4u) ? nb1 - 1 - fz : fz;
                    if (!occ(x, y, z)) bytes[(size_t)blk_index(x, y, z, nb2) * 8 + o] = df_value(x, y, z, o, nb1, occ, get);
                }
}

// The octant planes from built levels (as build_planes_k): dfp holds 8 * nb2^3 * 64 bytes.
inline void build_planes_host(const uint64_t* l1, const uint64_t* l2, uint32_t n, uint8_t* dfp) {
    const uint32_t nb1 = (n + 3) / 4, nb2 = (nb1 + 3) / 4, nb3 = (nb2 + 3) / 4;
    const uint64_t plane = 64ull * nb2 * nb2 * nb2;
    std::memset(dfp, 0, 8 * plane);
    for (uint32_t z = 0; z < nb1; ++z)
        for (uint32_t y = 0; y < nb1; ++y)
            for (uint32_t x = 0; x < nb1; ++x) {
                if ((l2[blk_index(x >> 2, y >> 2, z >> 2, nb3)] >> ((x & 3) + 4 * (y & 3) + 16 * (z & 3))) & 1ull) continue;
                const uint32_t b = blk_index(x, y, z, nb2);
                for (uint32_t o = 0; o < 8; ++o) dfp[o * plane + b] = (uint8_t)(l1[b] >> (8 * o));
            }
}
#endif

}  // namespace skip
}  // namespace vpx
