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
static uint64_t g_small;
extern "C" uint64_t small_out() { const uint64_t v = g_small; g_small = 0; return v; }
extern "C" void cross_out(uint64_t* o) {
    for (int i = 0; i < 16; ++i) o[i] = g_cross[i], g_cross[i] = 0;
}

// Experimental anisotropic boxes (g_mode 1): per brick, octant and axis a, the side k of
// the largest empty k x k square of bricks in the brick's layer across axis a, growing
// toward the octant (a 1-brick-thick slab).  g_slab[((a * 8 + o) * nb^3) + lin(brick)]
static std::vector<uint8_t> g_slab;
static uint32_t g_nb = 0;
static int g_mode = 0;
static int g_full = 0;
extern "C" void set_full(int f) { g_full = f; }
extern "C" void set_mode(int m) { g_mode = m; }
extern "C" void build_slabs(const uint8_t* bocc, uint32_t nb) {  // bocc[z][y][x] != 0: occupied
    g_nb = nb;
    const size_t n3 = (size_t)nb * nb * nb;
    g_slab.assign(24 * n3, 0);
    auto lin = [&](uint32_t x, uint32_t y, uint32_t z) { return (size_t)z * nb * nb + (size_t)y * nb + x; };
    for (uint32_t a = 0; a < 3; ++a)
        for (uint32_t o = 0; o < 8; ++o) {
            uint8_t* K = &g_slab[(a * 8 + o) * n3];
            const int s[3] = {(o & 1) ? -1 : 1, (o & 2) ? -1 : 1, (o & 4) ? -1 : 1};
            // sweep from the far corner of the octant in the two axes other than a
            for (uint32_t fz = nb; fz-- > 0;)
                for (uint32_t fy = nb; fy-- > 0;)
                    for (uint32_t fx = nb; fx-- > 0;) {
                        const uint32_t x = s[0] < 0 ? nb - 1 - fx : fx, y = s[1] < 0 ? nb - 1 - fy : fy, z = s[2] < 0 ? nb - 1 - fz : fz;
                        if (bocc[lin(x, y, z)]) { K[lin(x, y, z)] = 0; continue; }
                        uint32_t mn = 255;
                        for (uint32_t j = 1; j < 8; ++j) {
                            if (j & (1u << a)) continue;  // stay in the layer
                            const uint32_t p = x + ((j & 1) ? s[0] : 0), q = y + ((j & 2) ? s[1] : 0), r = z + ((j & 4) ? s[2] : 0);
                            const uint32_t v = (p < nb && q < nb && r < nb) ? K[lin(p, q, r)] : 255u;
                            mn = v < mn ? v : mn;
                        }
                        K[lin(x, y, z)] = (uint8_t)(mn < 255 ? mn + 1 : 255);
                    }
        }
}
static uint64_t g_slabskips;
static uint64_t g_seg2[4];  // skips by the number of axes that need the second closed-form segment
extern "C" void seg2_out(uint64_t* o) { for (int i = 0; i < 4; ++i) o[i] = g_seg2[i], g_seg2[i] = 0; }
extern "C" uint64_t slab_out() { const uint64_t v = g_slabskips; g_slabskips = 0; return v; }

// rays: st = (t, tx, ty, tz, dx, dy, dz), si = (X, Y, Z, sx, sy, sz) per ray; out[8] =
// cells, steps, skips, hits, end-state checksum, sum of t bits, lean refusals, max skips
extern "C" void walk_sim(const uint8_t* cells, const uint64_t* l1, const uint64_t* l2, uint32_t n, const float* st,
                         const int32_t* si, const float* bounds, uint32_t nrays, uint64_t* out, float* tout,
                         uint32_t* per = nullptr) {
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
            int cls = classify(w, g);
            if (cls == 0) { ++c; hit = true; break; }
            uint32_t slo[3], shi[3];
            bool slab = false;
            if (g_mode && cls != 0) {
                const uint32_t bb = ((w.X >> 2) & 3u) | (((w.Y >> 2) & 3u) << 2) | (((w.Z >> 2) & 3u) << 4);
                if (!((w.m2 >> bb) & 1ull)) {
                    // candidates: the cube, and the three slabs; pick the farthest approximate exit
                    const uint32_t o = w.osh / 8, nb = g_nb;
                    const uint32_t B[3] = {w.X >> 2, w.Y >> 2, w.Z >> 2};
                    const size_t li = (size_t)B[2] * nb * nb + (size_t)B[1] * nb + B[0], n3 = (size_t)nb * nb * nb;
                    const uint32_t kc = (uint32_t)(w.m1 >> w.osh) & 255u;
                    const float h[3] = {w.tx, w.ty, w.tz}, d[3] = {w.dx, w.dy, w.dz};
                    const int32_t sg[3] = {w.sx, w.sy, w.sz};
                    const uint32_t C3[3] = {w.X, w.Y, w.Z};
                    float best = -1; int bi = -1;
                    for (int cand = 0; cand < 4; ++cand) {
                        uint32_t ext[3];
                        if (cand == 0) ext[0] = ext[1] = ext[2] = kc;
                        else {
                            const uint32_t a = cand - 1, k = g_slab[(a * 8 + o) * n3 + li];
                            for (int q = 0; q < 3; ++q) ext[q] = q == (int)a ? 1u : k;
                        }
                        float ex = 3.4e38f;
                        for (int q = 0; q < 3; ++q) {
                            const uint32_t bq = C3[q] & ~3u;
                            const uint32_t l = sg[q] > 0 ? bq + ext[q] * 4 - 1 - C3[q] : C3[q] - (bq + 4 > ext[q] * 4 ? bq + 4 - ext[q] * 4 : 0);
                            const float e = h[q] + (float)l * d[q];
                            ex = e < ex ? e : ex;
                        }
                        if (ex > best) best = ex, bi = cand;
                    }
                    // worth a skip when the exit is at least g_mode cells ahead along the ray (cheapest axis)
                    const float dmin = std::min(std::min(d[0], d[1]), d[2]);
                    if (bi > 0 && best - w.t >= (float)g_mode * dmin) {
                        const uint32_t a = bi - 1, k = g_slab[(a * 8 + o) * n3 + li];
                        for (int q = 0; q < 3; ++q) {
                            const uint32_t e = q == (int)a ? 1u : k, bq = C3[q] & ~3u;
                            const uint32_t up = bq + e * 4 - 1, dn = bq + 4 > e * 4 ? bq + 4 - e * 4 : 0;
                            slo[q] = sg[q] > 0 ? C3[q] : dn;
                            shi[q] = sg[q] > 0 ? (up < n - 1 ? up : n - 1) : C3[q];
                        }
                        slab = true; cls = 2; ++g_slabskips;
                    } else if (bi == 0 && kc >= 1 && best - w.t >= (float)g_mode * dmin) cls = 2;
                    else cls = 1;
                }
            }
            if (cls == 2) {
                ++skips;
                uint32_t lo[3], hi[3];
                df_box(w, n, cube_l1(w), lo, hi);
                if (slab) for (int q = 0; q < 3; ++q) lo[q] = slo[q], hi[q] = shi[q];
                const uint32_t olo[3] = {lo[0], lo[1], lo[2]}, ohi[3] = {hi[0], hi[1], hi[2]};
                {
                    Axis ax[3];
                    const float hh[3] = {w.tx, w.ty, w.tz}, dd[3] = {w.dx, w.dy, w.dz};
                    const int32_t sg[3] = {w.sx, w.sy, w.sz};
                    const uint32_t c3[3] = {w.X, w.Y, w.Z};
                    int n2 = 0;
                    for (int k = 0; k < 3; ++k) {
                        axis_setup(hh[k], dd[k], sg[k] > 0 ? hi[k] - c3[k] : c3[k] - lo[k], ax[k]);
                        n2 += ax[k].l > ax[k].m1;
                    }
                    g_seg2[n2]++;
                }
                Walk t = w;
                uint32_t cc = 0;
                // g_full: the exact multi-binade tier (skip_box: every box whole, any number of
                // binade crossings) instead of the lean two-segment tier — what a lean tier with
                // more segments could reach
                int sr = g_full ? skip_box(t, lo, hi, bound, cc) : skip_box_lean(t, lo, hi, bound, cc);
                if (g_full && sr == 2) sr = skip_box_lean(t, lo, hi, bound, cc);
                bool clipped = false;
                for (int k = 0; k < 3; ++k) clipped |= lo[k] != olo[k] || hi[k] != ohi[k];
                if (sr == 2 || clipped) {
                    ++out[6];
                    const float hh[3] = {w.tx, w.ty, w.tz}, dd[3] = {w.dx, w.dy, w.dz};
                    const int32_t sg[3] = {w.sx, w.sy, w.sz};
                    const uint32_t c3[3] = {w.X, w.Y, w.Z};
                    uint32_t worst = 0;
                    for (int k = 0; k < 3; ++k) {
                        const uint32_t l = sg[k] > 0 ? ohi[k] - c3[k] : c3[k] - olo[k];
                        if (!l || !(hh[k] > 0) || !(dd[k] > 0)) continue;
                        const uint32_t crs = (fbits(jump(hh[k], dd[k], l)) >> 23) - (fbits(hh[k]) >> 23);
                        worst = crs > worst ? crs : worst;
                    }
                    g_cross[worst < 15 ? worst : 15]++;
                }
                if (sr == 2) { ++c; if (!step1(w, n)) break; continue; }
                w = t; c += cc;
                if (sr == 1) break;
                ++c;
                if (!step1(w, n)) break;
                continue;
            } else {
                ++steps;
                const uint32_t bb = ((w.X >> 2) & 3u) | (((w.Y >> 2) & 3u) << 2) | (((w.Z >> 2) & 3u) << 4);
                if (!((w.m2 >> bb) & 1ull)) ++g_small;  // empty brick whose cube is below kMinCube
            }
            ++c;
            if (!step1(w, n)) break;
        }
        out[0] += c, out[1] += steps, out[2] += skips, out[3] += hit;
        out[4] += (uint64_t)w.X | ((uint64_t)w.Y << 20) | ((uint64_t)w.Z << 40);
        out[5] += fbits(w.t);
        out[7] = out[7] > skips ? out[7] : skips;
        if (tout) tout[r] = hit ? w.t : -1.0f;
        if (per) per[2 * r] = (uint32_t)steps, per[2 * r + 1] = (uint32_t)skips;
    }
}
