// CPU model of the skipping walker for tuning: per-ray counts of plain cell steps and
// distance-field skips, and how often the lean skip tier refuses a box (with the number
// of binade crossings that made it refuse).  Build / driver: tools/walkstats.py
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#include "vpx_skip.hpp"
using namespace vpx::skip;

extern "C" void build_masks(const uint8_t* cells, uint32_t n, uint64_t* l1, uint64_t* l2) {
    build_masks_host(cells, n, l1, l2);
}

static uint64_t g_cross[16];
extern "C" void cross_out(uint64_t* o) {
    for (int i = 0; i < 16; ++i) o[i] = g_cross[i], g_cross[i] = 0;
}

// rays: st = (t, tx, ty, tz, dx, dy, dz), si = (X, Y, Z, sx, sy, sz) per ray; out[8] =
// cells, steps, skips, hits, end-state checksum, sum of t bits, lean refusals, max skips
extern "C" void walk_sim(const uint8_t* cells, const uint64_t* l1, const uint64_t* l2, uint32_t n, const float* st,
                         const int32_t* si, const float* bounds, uint32_t nrays, uint64_t* out, float* tout) {
    const uint32_t nb1 = (n + 3) / 4, nb2 = (nb1 + 3) / 4, nb3 = (nb2 + 3) / 4;
    GridView g{cells, l1, l2, n, nb1, nb2, nb3};
    for (uint32_t r = 0; r < nrays; ++r) {
        Walk w{};
        w.X = si[6 * r], w.Y = si[6 * r + 1], w.Z = si[6 * r + 2];
        w.sx = si[6 * r + 3], w.sy = si[6 * r + 4], w.sz = si[6 * r + 5];
        w.t = st[7 * r], w.tx = st[7 * r + 1], w.ty = st[7 * r + 2], w.tz = st[7 * r + 3];
        w.dx = st[7 * r + 4], w.dy = st[7 * r + 5], w.dz = st[7 * r + 6];
        walk_begin(w);
        const float bound = bounds[r];
        uint32_t c = 0;
        uint64_t steps = 0, skips = 0;
        bool hit = false;
        for (;;) {
            if (!(w.t < bound)) break;
            const int cls = classify(w, g);
            if (cls == 0) { ++c; hit = true; break; }
            if (cls == 2) {
                ++skips;
                uint32_t lo[3], hi[3];
                df_box(w, n, lo, hi);
                Walk t = w;
                uint32_t cc = 0;
                if (skip_box_fast1(t, lo, hi, bound, cc) == 2) {
                    ++out[6];
                    const float hh[3] = {w.tx, w.ty, w.tz}, dd[3] = {w.dx, w.dy, w.dz};
                    const int32_t sg[3] = {w.sx, w.sy, w.sz};
                    const uint32_t c3[3] = {w.X, w.Y, w.Z};
                    uint32_t worst = 0;
                    for (int k = 0; k < 3; ++k) {
                        const uint32_t l = sg[k] > 0 ? hi[k] - c3[k] : c3[k] - lo[k];
                        if (!l || !(hh[k] > 0) || !(dd[k] > 0)) continue;
                        const uint32_t crs = (fbits(jump(hh[k], dd[k], l)) >> 23) - (fbits(hh[k]) >> 23);
                        worst = crs > worst ? crs : worst;
                    }
                    g_cross[worst < 15 ? worst : 15]++;
                }
                if (skip_box(w, lo, hi, bound, c) == 1) break;
            } else {
                ++steps;
            }
            ++c;
            if (!step1(w, n)) break;
        }
        out[0] += c, out[1] += steps, out[2] += skips, out[3] += hit;
        out[4] += (uint64_t)w.X | ((uint64_t)w.Y << 20) | ((uint64_t)w.Z << 40);
        out[5] += fbits(w.t);
        out[7] = out[7] > skips ? out[7] : skips;
        if (tout) tout[r] = hit ? w.t : -1.0f;
    }
}
