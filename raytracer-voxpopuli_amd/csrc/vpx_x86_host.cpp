// vpx_x86_host.cpp — capture and verification of the host CPU's rcpss / rsqrtss tables for
// the reference-arithmetic mode (VPX_ARITH_X86_HOST; the model is vpx_x86.hpp).  Host code
// only, no device work.  The reference runs with FTZ | DAZ (template/template.cpp:130), so
// every evaluation here does too.
#include <atomic>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/vpx.h"
#include "vpx_x86.hpp"

#if defined(__x86_64__) || defined(__i386__)
#include <xmmintrin.h>
#define VPX_HOST_X86 1
#endif

namespace {

#ifdef VPX_HOST_X86
struct MxcsrScope {  // FTZ | DAZ for this thread while in scope
    unsigned int saved;
    MxcsrScope() : saved(_mm_getcsr()) { _mm_setcsr(saved | 0x8040u); }
    ~MxcsrScope() { _mm_setcsr(saved); }
};
inline __m128 bits4(uint32_t a) {  // a, a+1, a+2, a+3 as floats
    return _mm_castsi128_ps(_mm_add_epi32(_mm_set1_epi32((int)a), _mm_set_epi32(3, 2, 1, 0)));
}
inline uint32_t rcp_host(uint32_t u) {
    float f;
    std::memcpy(&f, &u, 4);
    const float r = _mm_cvtss_f32(_mm_rcp_ss(_mm_set_ss(f)));
    uint32_t o;
    std::memcpy(&o, &r, 4);
    return o;
}
inline uint32_t rsq_host(uint32_t u) {
    float f;
    std::memcpy(&f, &u, 4);
    const float r = _mm_cvtss_f32(_mm_rsqrt_ss(_mm_set_ss(f)));
    uint32_t o;
    std::memcpy(&o, &r, 4);
    return o;
}

// The smallest shift s such that full[i] == full[i with its low s bits cleared] for every i.
uint32_t key_shift(const std::vector<uint32_t>& full, uint32_t max_shift) {
    uint32_t s = max_shift;
    for (;; --s) {
        const uint32_t mask = ~((1u << s) - 1u);
        bool ok = true;
        for (size_t i = 0; i < full.size() && ok; ++i) ok = full[i] == full[i & mask];
        if (ok || s == 0) return s;
    }
}

// Captured model: the rcp entries, then the rsqrt entries.
struct Model {
    std::vector<uint32_t> tab;
    uint32_t rcp_shift = 0, rsq_shift = 0, rsq_off = 0;
};

void capture(Model& md) {
    MxcsrScope fz;
    std::vector<uint32_t> rcp(1u << 23), rsq(1u << 24);
    for (uint32_t m = 0; m < (1u << 23); ++m) rcp[m] = rcp_host(0x3f800000u | m);
    for (uint32_t i = 0; i < (1u << 24); ++i) rsq[i] = rsq_host(((127u + (i >> 23)) << 23) | (i & 0x7fffffu));
    md.rcp_shift = key_shift(rcp, 23);
    md.rsq_shift = key_shift(rsq, 24);
    const uint32_t nr = 1u << (23 - md.rcp_shift), ns = 1u << (24 - md.rsq_shift);
    md.tab.resize((size_t)nr + ns);
    for (uint32_t j = 0; j < nr; ++j) md.tab[j] = rcp[(size_t)j << md.rcp_shift];
    for (uint32_t j = 0; j < ns; ++j) md.tab[nr + j] = rsq[(size_t)j << md.rsq_shift];
    md.rsq_off = nr;
}

// Model vs intrinsic over [lo, hi] (inclusive), 4 inputs per step; counts per op.
void verify_range(const Model& md, uint64_t lo, uint64_t hi, uint64_t mis[2], uint32_t bad[2]) {
    MxcsrScope fz;
    const uint32_t* rt = md.tab.data();
    const uint32_t* st = md.tab.data() + md.rsq_off;
    uint64_t u = lo;
    for (; u + 3 <= hi; u += 4) {
        const __m128 x = bits4((uint32_t)u);
        alignas(16) uint32_t r[4], s[4];
        _mm_store_ps(reinterpret_cast<float*>(r), _mm_rcp_ps(x));
        _mm_store_ps(reinterpret_cast<float*>(s), _mm_rsqrt_ps(x));
        for (uint32_t k = 0; k < 4; ++k) {
            const uint32_t v = (uint32_t)u + k;
            if (vpx::x86_rcp_bits(v, rt, md.rcp_shift) != r[k] && mis[0]++ == 0) bad[0] = v;
            if (vpx::x86_rsq_bits(v, st, md.rsq_shift) != s[k] && mis[1]++ == 0) bad[1] = v;
        }
    }
    for (; u <= hi; ++u) {
        const uint32_t v = (uint32_t)u;
        if (vpx::x86_rcp_bits(v, rt, md.rcp_shift) != rcp_host(v) && mis[0]++ == 0) bad[0] = v;
        if (vpx::x86_rsq_bits(v, st, md.rsq_shift) != rsq_host(v) && mis[1]++ == 0) bad[1] = v;
    }
}

// The check vpx_x86_arith_tables runs on every capture: both signs of every exponent, each
// with its binade's first, last and 2046 pseudo-random mantissas, plus the specials.
bool spot_check(const Model& md, uint32_t bad[2]) {
    uint64_t mis[2] = {0, 0};
    uint32_t seed = 0x2545f491u;
    for (uint32_t sgn = 0; sgn < 2; ++sgn)
        for (uint32_t e = 0; e < 256; ++e)
            for (uint32_t i = 0; i < 2048; ++i) {
                seed ^= seed << 13, seed ^= seed >> 17, seed ^= seed << 5;
                const uint32_t m = i == 0 ? 0u : (i == 1 ? 0x7fffffu : (seed & 0x7fffffu));
                const uint32_t v = (sgn << 31) | (e << 23) | m;
                verify_range(md, v, v, mis, bad);
            }
    return mis[0] == 0 && mis[1] == 0;
}

// The host's tables do not change while the process runs: capture and spot-check once, and
// serve every vpx_set_arithmetic (size query, data copy, each member of a device set) and
// every verify from that copy.
struct Cached {
    Model md;
    bool ok = false;
};
const Cached& cached_model() {
    static Cached c;
    static std::once_flag once;
    std::call_once(once, [] {
        capture(c.md);
        uint32_t bad[2] = {0, 0};
        c.ok = spot_check(c.md, bad);
    });
    return c;
}
#endif

}  // namespace

extern "C" {

int vpx_x86_arith_tables(uint32_t* out, uint64_t cap, uint32_t info[4]) {
#ifdef VPX_HOST_X86
    if (!info) return VPX_E_INVALID;
    const Cached& cm = cached_model();
    if (!cm.ok) return VPX_E_STATE;
    const Model& md = cm.md;
    info[0] = md.rcp_shift;
    info[1] = md.rsq_shift;
    info[2] = md.rsq_off;
    info[3] = (uint32_t)md.tab.size();
    if (out) {
        if (cap < md.tab.size()) return VPX_E_INVALID;
        std::memcpy(out, md.tab.data(), md.tab.size() * 4);
    }
    return VPX_OK;
#else
    (void)out, (void)cap, (void)info;
    return VPX_E_STATE;
#endif
}

int vpx_x86_arith_verify(uint32_t lo, uint32_t hi, uint32_t threads, uint64_t mismatches[2], uint32_t first_bad[2]) {
#ifdef VPX_HOST_X86
    if (!mismatches || !first_bad || hi < lo) return VPX_E_INVALID;
    const Model& md = cached_model().md;
    const uint32_t nt = threads ? (threads > 256 ? 256 : threads) : 1u;
    const uint64_t n = (uint64_t)hi - lo + 1;
    std::vector<uint64_t> mis(2 * nt, 0);
    std::vector<uint32_t> bad(2 * nt, 0);
    std::vector<std::thread> pool;
    for (uint32_t t = 0; t < nt; ++t) {
        const uint64_t a = lo + n * t / nt, b = lo + n * (t + 1) / nt;  // [a, b)
        if (a == b) continue;
        pool.emplace_back([&, t, a, b] { verify_range(md, a, b - 1, &mis[2 * t], &bad[2 * t]); });
    }
    for (auto& th : pool) th.join();
    mismatches[0] = mismatches[1] = 0;
    first_bad[0] = first_bad[1] = 0;
    for (uint32_t t = 0; t < nt; ++t)  // threads in range order: the first bad input overall
        for (uint32_t k = 0; k < 2; ++k) {
            if (mis[2 * t + k] && !mismatches[k]) first_bad[k] = bad[2 * t + k];
            mismatches[k] += mis[2 * t + k];
        }
    return VPX_OK;
#else
    (void)lo, (void)hi, (void)threads, (void)mismatches, (void)first_bad;
    return VPX_E_STATE;
#endif
}

}  // extern "C"
