// CPU model of the skipping walker for tuning: per-ray counts of classify iterations,
// plain steps and skip_box calls (by level) on a real world.  Build: see tools/walkstats.py
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#include "vpx_skip.hpp"
using namespace vpx::skip;

extern "C" void build_masks(const uint8_t* cells, uint32_t n, uint64_t* l1, uint64_t* l2, uint64_t* l3) {
    build_masks_host(cells, n, l1, l2, l3);
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
static uint64_t g_cross[16];
extern "C" void cross_out(uint64_t* o) { for (int i = 0; i < 16; ++i) { o[i] = g_cross[i]; g_cross[i] = 0; } }
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
                { Walk t = w; uint32_t cc = 0; const bool okf = skip_box_fast1(t, lo, hi, bound, cc) != 2; out[7] += okf; if (!okf) why(w, lo, hi); }
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

// ---- box-choice simulation: how many steps / skips per ray for alternative empty boxes
// opt bit 0: 32^3 groups of empty macros (from the l3 word); bit 1: 128^3 / 256^3 groups of
// empty supers (l4 = bit per super); bit 2: 8^3 / 4^3 empty bricks inside non-empty macros.
static uint64_t l3word(const GridView& g, uint32_t sx, uint32_t sy, uint32_t sz) {
    if (sx >= g.nb3 || sy >= g.nb3 || sz >= g.nb3) return ~0ull;
    return g.l3[lin_index(sx, sy, sz, g.nb3)];
}
extern "C" void walk_sim(const uint8_t* cells, const uint64_t* l1, const uint64_t* l2, const uint64_t* l3, uint32_t n,
                         const float* st, const int32_t* si, const float* bounds, uint32_t nrays, int opt, uint64_t* out, float* tout) {
    const uint32_t nb1 = (n + 3) / 4, nb2 = (nb1 + 3) / 4, nb3 = (nb2 + 3) / 4;
    GridView g{cells, l1, l2, l3, n, nb1, nb2, nb3};
    for (uint32_t r = 0; r < nrays; ++r) {
        Walk w{};
        w.X = si[6 * r], w.Y = si[6 * r + 1], w.Z = si[6 * r + 2];
        w.sx = si[6 * r + 3], w.sy = si[6 * r + 4], w.sz = si[6 * r + 5];
        w.t = st[7 * r], w.tx = st[7 * r + 1], w.ty = st[7 * r + 2], w.tz = st[7 * r + 3];
        w.dx = st[7 * r + 4], w.dy = st[7 * r + 5], w.dz = st[7 * r + 6];
        w.k1 = w.k2 = w.k3 = 0xffffffffu;
        const float bound = bounds[r];
        uint32_t c = 0;
        uint64_t steps = 0, skips = 0;
        bool hit = false;
        for (;;) {
            if (!(w.t < bound)) break;
            const int cls = classify(w, g);
            if (cls == 0) { ++c; hit = true; break; }
            uint32_t m = 0, lo[3], hi[3];
            bool box = false;
            if (cls == 3) {
                box = true, m = 63;
                if (opt & 2) {  // 4x4x4 / 2x2x2 groups of empty supers
                    const uint32_t sx = w.X >> 6, sy = w.Y >> 6, sz = w.Z >> 6;
                    bool e4 = true, e2 = true;
                    for (uint32_t z = 0; z < 4; ++z) for (uint32_t y = 0; y < 4; ++y) for (uint32_t x = 0; x < 4; ++x) {
                        const uint64_t v = l3word(g, (sx & ~3u) + x, (sy & ~3u) + y, (sz & ~3u) + z);
                        if (v) { e4 = false; if (((x >> 1) == ((sx >> 1) & 1)) && ((y >> 1) == ((sy >> 1) & 1)) && ((z >> 1) == ((sz >> 1) & 1))) e2 = false; }
                    }
                    m = e4 ? 255 : (e2 ? 127 : 63);
                }
            } else if (cls == 2) {
                box = true, m = 15;
                if (opt & 1) {
                    const uint32_t gx = (w.X >> 5) & 1, gy = (w.Y >> 5) & 1, gz = (w.Z >> 5) & 1;
                    if (!(w.m3 & (0x330033ull << (2 * gx + 8 * gy + 32 * gz)))) m = 31;
                }
            } else if (opt & 4) {  // empty cell: empty brick / 2x2x2 bricks?
                const uint32_t bb = ((w.X >> 2) & 3u) | (((w.Y >> 2) & 3u) << 2) | (((w.Z >> 2) & 3u) << 4);
                if (!((w.m2 >> bb) & 1ull)) {
                    box = true, m = 3;
                    const uint32_t gx = (w.X >> 3) & 1, gy = (w.Y >> 3) & 1, gz = (w.Z >> 3) & 1;
                    if (!(w.m2 & (0x330033ull << (2 * gx + 8 * gy + 32 * gz)))) m = 7;
                }
            }
            if (box && (opt & 8)) {  // adaptive: shrink the box until the lean tier applies (h >= l d per axis)
                auto fits = [&](uint32_t mm) {
                    const float h[3] = {w.tx, w.ty, w.tz}, d[3] = {w.dx, w.dy, w.dz};
                    const int32_t sg[3] = {w.sx, w.sy, w.sz};
                    const uint32_t c3[3] = {w.X, w.Y, w.Z};
                    for (int k = 0; k < 3; ++k) {
                        const uint32_t lo_ = c3[k] & ~mm, hi_ = (c3[k] | mm) < n - 1u ? (c3[k] | mm) : n - 1u;
                        const uint32_t l = sg[k] > 0 ? hi_ - c3[k] : c3[k] - lo_;
                        if (l && !(h[k] >= (float)l * d[k])) return false;
                    }
                    return true;
                };
                if (!fits(m)) {
                    if (m > 15 && fits(15)) m = 15;
                    else box = false;
                }
            }
            if (box) {
                ++skips;
                { Walk t = w; uint32_t cc = 0; uint32_t blo[3], bhi[3];
                  for (int k = 0; k < 3; ++k) { const uint32_t q = k == 0 ? w.X : k == 1 ? w.Y : w.Z; blo[k] = q & ~m; bhi[k] = (q | m) < n - 1u ? (q | m) : n - 1u; }
                  const bool miss = skip_box_fast1(t, blo, bhi, bound, cc) == 2;
                  out[6] += miss;
                  if (miss) {  // crossings needed: max over axes of binades spanned by A(0..l)
                      const float hh[3] = {w.tx, w.ty, w.tz}, dd[3] = {w.dx, w.dy, w.dz};
                      const int32_t sg[3] = {w.sx, w.sy, w.sz};
                      const uint32_t c3[3] = {w.X, w.Y, w.Z};
                      uint32_t worst = 0;
                      for (int k = 0; k < 3; ++k) {
                          const uint32_t l = sg[k] > 0 ? bhi[k] - c3[k] : c3[k] - blo[k];
                          if (!l || !(hh[k] > 0) || !(dd[k] > 0)) continue;
                          const float A = jump(hh[k], dd[k], l);
                          const uint32_t cr = (fbits(A) >> 23) - (fbits(hh[k]) >> 23);
                          worst = cr > worst ? cr : worst;
                      }
                      g_cross[worst < 15 ? worst : 15]++;
                  }
                  if (miss && m > 15) {  // retry with the 16^3 macro box around the cell
                      for (int k = 0; k < 3; ++k) { const uint32_t q = k == 0 ? w.X : k == 1 ? w.Y : w.Z; blo[k] = q & ~15u; bhi[k] = (q | 15u) < n - 1u ? (q | 15u) : n - 1u; }
                      Walk t2 = w; uint32_t c2 = 0;
                      out[7] += skip_box_fast1(t2, blo, bhi, bound, c2) == 2;
                  } else out[7] += miss; }
                for (int k = 0; k < 3; ++k) {
                    const uint32_t cc = k == 0 ? w.X : k == 1 ? w.Y : w.Z;
                    lo[k] = cc & ~m;
                    hi[k] = (cc | m) < n - 1u ? (cc | m) : n - 1u;
                }
                if (skip_box(w, lo, hi, bound, c) == 1) break;
            } else ++steps;
            ++c;
            if (!step1(w, n)) break;
        }
        out[0] += c; out[1] += steps; out[2] += skips; out[3] += hit;
        out[4] += (uint64_t)w.X | ((uint64_t)w.Y << 20) | ((uint64_t)w.Z << 40);  // checksum of end state
        out[5] += fbits(w.t);
        if (tout) tout[r] = hit ? w.t : -1.0f;
    }
}
