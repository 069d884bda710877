// vpx_x86.hpp — the reference's x86 approximations, reproduced bit for bit from tables
// captured on the host CPU (VPX_ARITH_X86_HOST, vpx_set_arithmetic).
//
// The reference computes the object-space rD of every Renderer::FindNearest volume visit with
// FastReciprocal — rcpps plus one Newton step (renderer.cpp:929-934, called at :969) — and
// normalises the primary direction of Renderer::Update with normalize(__m128) = v *
// rsqrtps(dpps(v, v, 0x7F)) (template/tmpl8math.h:2356-2360; renderer.cpp:1735-1765, rD from
// the unnormalised direction).  rcpps / rsqrtps are table approximations whose bits differ
// between CPU vendors, so the library reproduces the host's own: vpx_x86_host.cpp evaluates
// the host's rcpss / rsqrtss over every mantissa of one binade (rcp: [1, 2); rsqrt: [1, 4),
// the exponent parity selects the half), keeps the shortest key (the top mantissa bits the
// result depends on), and the functions below scale the table value by the input's exponent
// and handle zeros, denormals (DAZ: as zeros), infinities and NaNs as x86 does.  The model is
// checked against the intrinsic for all 2^32 inputs (vpx_x86_arith_verify, tests/test_x86_arith.py)
// and spot-checked at every vpx_set_arithmetic.  Host (verification) and device (the walkers)
// run this same code.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define VPX_HDX __host__ __device__ inline __attribute__((always_inline))
#else
#define VPX_HDX inline
#endif

namespace vpx {

// The captured tables as a kernel sees them (SceneView::x86).  tab == nullptr: exact mode.
struct X86Arith {
    const uint32_t* tab;  // rcp entries [0, 2^(23 - rcp_shift)), then rsqrt entries at rsq_off
    uint32_t rcp_shift;   // rcp key = mantissa >> rcp_shift
    uint32_t rsq_shift;   // rsqrt key = (parity << 23 | mantissa) >> rsq_shift
    uint32_t rsq_off;     // first rsqrt entry
    uint32_t pad;
};

// rcpss(x) as bits: the table holds rcp(1.m) for the key's mantissas; the exponent moves the
// result by 2^-(e - 127).  Zero / denormal -> signed infinity, infinity -> signed zero, NaN ->
// the quieted NaN, results below the normal range -> signed zero (flush).
// Split in two so that a caller can issue the table loads of several inputs before using any
// (the key is a valid index for every input, specials included): x86_rcp_key gives the index,
// x86_rcp_from the result from the input and its entry t, branch-free.
VPX_HDX uint32_t x86_rcp_key(uint32_t u, uint32_t shift) { return (u & 0x7fffffu) >> shift; }
VPX_HDX uint32_t x86_rcp_from(uint32_t u, uint32_t t) {
    const uint32_t s = u & 0x80000000u, e = (u >> 23) & 0xffu, m = u & 0x7fffffu;
    const int32_t ne = (int32_t)((t >> 23) & 0xffu) + 127 - (int32_t)e;
    uint32_t r = ne <= 0 ? s : (s | ((uint32_t)ne << 23) | (t & 0x7fffffu));
    r = e == 0u ? (s | 0x7f800000u) : r;
    r = e == 255u ? (m ? (u | 0x400000u) : s) : r;
    return r;
}
VPX_HDX uint32_t x86_rcp_bits(uint32_t u, const uint32_t* tab, uint32_t shift) {
    return x86_rcp_from(u, tab[x86_rcp_key(u, shift)]);
}

// rsqrtss(x) as bits: the table holds rsqrt of [1, 4) (parity 1 = [2, 4)); an even exponent
// step 2q moves the result by 2^-q.  +-0 / denormals -> signed infinity, negative -> the
// default NaN, +inf -> +0, NaN -> the quieted NaN.  (Key and result split as for rcp.)
VPX_HDX uint32_t x86_rsq_key(uint32_t u, uint32_t shift) {
    const uint32_t par = ((u >> 23) & 1u) ^ 1u;  // (e - 127) odd: the [2, 4) half
    return ((par << 23) | (u & 0x7fffffu)) >> shift;
}
VPX_HDX uint32_t x86_rsq_from(uint32_t u, uint32_t t) {
    const uint32_t e = (u >> 23) & 0xffu, m = u & 0x7fffffu;
    const uint32_t par = (e & 1u) ^ 1u;
    const int32_t q = ((int32_t)e - 127 - (int32_t)par) / 2;  // exact: the difference is even
    uint32_t r = ((uint32_t)((int32_t)((t >> 23) & 0xffu) - q) << 23) | (t & 0x7fffffu);
    r = (u & 0x80000000u) ? 0xffc00000u : r;
    r = e == 255u ? (m ? (u | 0x400000u) : ((u & 0x80000000u) ? 0xffc00000u : 0u)) : r;
    r = e == 0u ? ((u & 0x80000000u) | 0x7f800000u) : r;
    return r;
}
VPX_HDX uint32_t x86_rsq_bits(uint32_t u, const uint32_t* tab, uint32_t shift) {
    return x86_rsq_from(u, tab[x86_rsq_key(u, shift)]);
}

}  // namespace vpx
