// CPU model of the skipping walker for tuning: per-ray counts of classify iterations,
// plain steps and skip_box calls (by level) on a real world.  Build: see tools/walkstats.py
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#include "vpx_skip.hpp"
using namespace vpx::skip;

extern "C" void build_masks(const uint8_t* cells, uint32_t n, uint64_t* l1, uint64_t* l2, uint64_t* l3) {
    const uint32_t nb1 = (n + 3) / 4, nb2 = (nb1 + 3) / 4, nb3 = (nb2 + 3) / 4;
    memset(l1, 0, 8ull * nb1 * nb1 * nb1); memset(l2, 0, 8ull * nb2 * nb2 * nb2); memset(l3, 0, 8ull * nb3 * nb3 * nb3);
    for (uint64_t z = 0; z < n; ++z) for (uint64_t y = 0; y < n; ++y) for (uint64_t x = 0; x < n; ++x)
        if (cells[x + y * n + z * n * n] != 255) l1[(x >> 2) + (y >> 2) * nb1 + (z >> 2) * nb1 * nb1] |= 1ull << ((x & 3) + 4 * (y & 3) + 16 * (z & 3));
    for (uint64_t z = 0; z < nb1; ++z) for (uint64_t y = 0; y < nb1; ++y) for (uint64_t x = 0; x < nb1; ++x)
        if (l1[x + y * nb1 + z * nb1 * nb1]) l2[(x >> 2) + (y >> 2) * nb2 + (z >> 2) * nb2 * nb2] |= 1ull << ((x & 3) + 4 * (y & 3) + 16 * (z & 3));
    for (uint64_t z = 0; z < nb2; ++z) for (uint64_t y = 0; y < nb2; ++y) for (uint64_t x = 0; x < nb2; ++x)
        if (l2[x + y * nb2 + z * nb2 * nb2]) l3[(x >> 2) + (y >> 2) * nb3 + (z >> 2) * nb3 * nb3] |= 1ull << ((x & 3) + 4 * (y & 3) + 16 * (z & 3));
}

static bool fast_ok(const Walk& w, const uint32_t lo[3], const uint32_t hi[3]) {
    const float h[3] = {w.tx, w.ty, w.tz}, d[3] = {w.dx, w.dy, w.dz};
    const int32_t s[3] = {w.sx, w.sy, w.sz};
    const uint32_t c[3] = {w.X, w.Y, w.Z};
    for (int k = 0; k < 3; ++k) {
        if (!(h[k] > 0.0f) || !(d[k] > 0.0f)) return false;
        const uint32_t e = s[k] > 0 ? hi[k] - c[k] + 1u : c[k] - lo[k] + 1u;
        const Seg g = segment(h[k], d[k]);
        if (!g.ok || g.stuck) return false;
        if ((uint64_t)(e - 1u) * g.c > 0xffffffu - g.b) return false;
    }
    return true;
}

static uint64_t g_why[8];
static void why(const Walk& w, const uint32_t lo[3], const uint32_t hi[3]) {
    const float h[3] = {w.tx, w.ty, w.tz}, d[3] = {w.dx, w.dy, w.dz};
    const int32_t s[3] = {w.sx, w.sy, w.sz};
    const uint32_t c[3] = {w.X, w.Y, w.Z};
    for (int k = 0; k < 3; ++k) {
        const uint32_t e = s[k] > 0 ? hi[k] - c[k] + 1u : c[k] - lo[k] + 1u;
        const uint32_t ab = fbits(h[k]), db = fbits(d[k]), ea = ab >> 23, ed = db >> 23;
        if (ea - 1u >= 254u || ed - 1u >= 254u) { g_why[0]++; continue; }
        if (ed >= ea) { g_why[1]++; continue; }
        uint32_t b, cc, ee;
        if (!seg_params(h[k], d[k], b, cc, ee)) { g_why[2]++; continue; }
        Seq2 q;
        if (!seq2_init(h[k], d[k], e - 1, q)) { g_why[3]++; continue; }
    }
}
extern "C" void why_out(uint64_t* o) { for (int i = 0; i < 8; ++i) o[i] = g_why[i]; }

// walks: setup state per ray given as (X,Y,Z,t,tx,ty,tz,dx,dy,dz,sx,sy,sz) float/int arrays
extern "C" void walk_stats(const uint8_t* cells, const uint64_t* l1, const uint64_t* l2, const uint64_t* l3, uint32_t n,
                           const float* st, const int32_t* si, uint32_t nrays, float bound, uint64_t* out /*8*/) {
    const uint32_t nb1 = (n + 3) / 4, nb2 = (nb1 + 3) / 4, nb3 = (nb2 + 3) / 4;
    GridView g{cells, l1, l2, l3, n, nb1, nb2, nb3};
    for (uint32_t r = 0; r < nrays; ++r) {
        Walk w{};
        w.X = si[6 * r], w.Y = si[6 * r + 1], w.Z = si[6 * r + 2];
        w.sx = si[6 * r + 3], w.sy = si[6 * r + 4], w.sz = si[6 * r + 5];
        w.t = st[7 * r], w.tx = st[7 * r + 1], w.ty = st[7 * r + 2], w.tz = st[7 * r + 3];
        w.dx = st[7 * r + 4], w.dy = st[7 * r + 5], w.dz = st[7 * r + 6];
        w.k1 = w.k2 = w.k3 = 0xffffffffu;
        uint32_t c = 0;
        uint64_t iters = 0, steps = 0, sk16 = 0, sk64 = 0, land0 = 0;
        for (;;) {
            if (!(w.t < bound)) break;
            ++iters;
            const int cls = classify(w, g);
            if (cls == 0) { ++c; break; }
            if (cls >= 2) {
                const uint32_t m = cls == 3 ? 63u : 15u;
                (cls == 3 ? sk64 : sk16)++;
                const uint32_t lo[3] = {w.X & ~m, w.Y & ~m, w.Z & ~m};
                uint32_t hi[3] = {lo[0] + m, lo[1] + m, lo[2] + m};
                for (int k = 0; k < 3; ++k) hi[k] = hi[k] < n - 1u ? hi[k] : n - 1u;
                const uint32_t before = c;
                { Walk t = w; uint32_t cc = 0; const bool okf = skip_box_fast(t, lo, hi, bound, cc) != 2; out[7] += okf; if (!okf) why(w, lo, hi); }
                const int rr = skip_box(w, lo, hi, bound, c);
                if (rr == 1) break;
                if (c == before) ++land0;
            } else ++steps;
            ++c;
            if (!step1(w, n)) break;
        }
        out[0] += c; out[1] += iters; out[2] += steps; out[3] += sk16; out[4] += sk64; out[5] += land0;
        out[6] = out[6] > iters ? out[6] : iters;
    }
}
