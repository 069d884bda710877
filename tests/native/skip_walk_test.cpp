// Randomised equivalence test: vpx::skip::walk_skip (occupancy hierarchy + exact binade
// jumps) against the plain cell-by-cell reference march (template/scene.cpp:751-811).
// Build: g++ -O2 -std=c++17 -ffp-contract=off -I raytracer-voxpopuli_amd/csrc tests/native/skip_walk_test.cpp
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>
#include <xmmintrin.h>
#include "vpx_skip.hpp"

using namespace vpx::skip;

struct World {
    uint32_t n, nb1, nb2, nb3;
    std::vector<uint8_t> cells;
    std::vector<uint64_t> l1, l2;
    std::vector<uint8_t> dfp;  // octant planes (classify_dfp)
    GridView view() const {
        return GridView{cells.data(), l1.data(), l2.data(), n, nb1, nb2, nb3, dfp.data(), 64ull * nb2 * nb2 * nb2};
    }
};

static World make_world(uint32_t n, uint64_t seed, double density) {
    World w;
    w.n = n;
    w.cells.assign((size_t)n * n * n, 255);
    std::mt19937_64 r(seed);
    // clustered boxes of solid voxels with holes
    const int boxes = (int)(density * 400);
    for (int b = 0; b < boxes; ++b) {
        uint32_t x0 = r() % n, y0 = r() % n, z0 = r() % n, sx = 1 + r() % (n / 6 + 1), sy = 1 + r() % (n / 6 + 1), sz = 1 + r() % (n / 6 + 1);
        for (uint32_t z = z0; z < std::min(n, z0 + sz); ++z)
            for (uint32_t y = y0; y < std::min(n, y0 + sy); ++y)
                for (uint32_t x = x0; x < std::min(n, x0 + sx); ++x)
                    if (r() % 5) w.cells[x + (size_t)y * n + (size_t)z * n * n] = (uint8_t)(r() % 200);
    }
    w.nb1 = (n + 3) / 4, w.nb2 = (w.nb1 + 3) / 4, w.nb3 = (w.nb2 + 3) / 4;
    w.l1.assign((size_t)w.nb2 * w.nb2 * w.nb2 * 64, 0);
    w.l2.assign((size_t)w.nb3 * w.nb3 * w.nb3 * 64, 0);
    build_masks_host(w.cells.data(), n, w.l1.data(), w.l2.data());
    w.dfp.assign(8 * 64ull * w.nb2 * w.nb2 * w.nb2, 0);
    build_planes_host(w.l1.data(), w.l2.data(), n, w.dfp.data());
    return w;
}

// classify_dfp (octant plane, then the mask of an occupied brick) == classify_dfp_o == classify (l1 + l2
// words) at sampled cells for every octant: the same class and the same m1 where it is read
// (the cell mask of an occupied brick, the octant's cube byte of an empty one).
static long check_planes(const World& W, std::mt19937_64& r) {
    const GridView g = W.view();
    const uint64_t cells = (uint64_t)W.n * W.n * W.n;
    const uint64_t samples = cells < 3000000 ? cells : 3000000;
    long bad = 0;
    for (uint64_t i = 0; i < samples; ++i) {
        const uint64_t c = samples == cells ? i : r() % cells;
        for (uint32_t o = 0; o < 8; ++o) {
            Walk a{};
            a.X = (uint32_t)(c % W.n), a.Y = (uint32_t)((c / W.n) % W.n), a.Z = (uint32_t)(c / ((uint64_t)W.n * W.n));
            a.sx = (o & 1) ? -1 : 1, a.sy = (o & 2) ? -1 : 1, a.sz = (o & 4) ? -1 : 1;
            walk_begin(a);
            Walk b = a, d = a;
            const int ca = classify(a, g), cb = classify_dfp(b, g, g.dfp + o * g.plane);
            const int cd = classify_dfp_o(d, g, plane_parent(g, o));  // the walkers' form
            const bool m1_read = ca == 1 || ca == 0 ? a.m1 == b.m1 : cube_l1(a) == cube_dfp(b);
            if (ca != cb || !m1_read || cd != cb || d.m1 != b.m1) {
                if (bad < 5) printf("plane mismatch n=%u cell (%u,%u,%u) octant %u: class %d/%d\n", W.n, a.X, a.Y, a.Z, o, ca, cb);
                ++bad;
            }
        }
    }
    return bad;
}

// Setup3DDDA for the unit cube (template/scene.cpp:719-749); false = misses the cube.
static bool setup(uint32_t n, const float O[3], const float D[3], Walk& w) {
    float rD[3], ds[3];
    for (int k = 0; k < 3; ++k) {
        rD[k] = 1.0f / D[k];
        uint32_t b;
        std::memcpy(&b, &D[k], 4);
        ds[k] = (float)(b >> 31);
    }
    float t = 0;
    const bool inside = O[0] >= 0 && O[1] >= 0 && O[2] >= 0 && O[0] <= 1 && O[1] <= 1 && O[2] <= 1;
    if (!inside) {
        float tmin = -1e30f, tmax = 1e30f;
        for (int k = 0; k < 3; ++k) {
            const int sg = D[k] < 0;
            float a = ((sg ? 1.f : 0.f) - O[k]) * rD[k], b = ((sg ? 0.f : 1.f) - O[k]) * rD[k];
            if (k == 0) { tmin = a, tmax = b; continue; }
            if (tmin > b || a > tmax) return false;
            tmin = tmin < a ? a : tmin;
            tmax = b < tmax ? b : tmax;
        }
        if (!(tmin > 0)) return false;
        t = tmin;
    }
    const float g = (float)n, cell = 1.0f / g;
    int P[3], st[3];
    float tm[3], td[3];
    for (int k = 0; k < 3; ++k) {
        st[k] = (int)(1.0f - ds[k] * 2.0f);
        const float pos = ((O[k] - 0.0f) + D[k] * (t + 0.00005f)) * g / 1.0f;
        const float plane = (std::ceil(pos) - ds[k]) * cell;
        int p = (pos > -2147483904.0f && pos < 2147483648.0f) ? (int)pos : (int)0x80000000u;
        P[k] = p < 0 ? 0 : (p > (int)n - 1 ? (int)n - 1 : p);
        td[k] = cell * (float)st[k] * rD[k];
        tm[k] = ((plane * 1.0f) - (O[k] - 0.0f)) * rD[k];
    }
    w = Walk{};
    w.X = P[0], w.Y = P[1], w.Z = P[2];
    w.t = t;
    w.tx = tm[0], w.ty = tm[1], w.tz = tm[2];
    w.dx = td[0], w.dy = td[1], w.dz = td[2];
    w.sx = st[0], w.sy = st[1], w.sz = st[2];
    walk_begin(w);
    return true;
}

// Scene::FindNearest's loop, cell by cell.
static bool walk_naive(const World& W, Walk s, float bound, uint32_t& cells, Walk& out) {
    const uint32_t n = W.n;
    while (s.t < bound) {
        const uint8_t c = W.cells[s.X + (size_t)s.Y * n + (size_t)s.Z * n * n];
        ++cells;
        if (c != 255 && s.t < bound) { out = s; return true; }
        if (s.tx < s.ty) {
            if (s.tx < s.tz) { s.t = s.tx; s.X += s.sx; if (s.X >= n) break; s.tx += s.dx; }
            else { s.t = s.tz; s.Z += s.sz; if (s.Z >= n) break; s.tz += s.dz; }
        } else {
            if (s.ty < s.tz) { s.t = s.ty; s.Y += s.sy; if (s.Y >= n) break; s.ty += s.dy; }
            else { s.t = s.tz; s.Z += s.sz; if (s.Z >= n) break; s.tz += s.dz; }
        }
    }
    return false;
}

// On a mismatch: replay the skipping walk and compare every skip tier against skip_box.
static void debug_walk(const GridView& g, Walk w, float bound) {
    for (int it = 0; it < 100000; ++it) {
        if (!(w.t < bound)) return;
        const int cls = classify(w, g);
        if (cls == 0) return;
        if (cls == 2) {
            uint32_t lo[3], hi[3];
            df_box(w, g.n, cube_l1(w), lo, hi);
            Walk a = w, b = w;
            uint32_t ca = 0, cb = 0;
            const int ra = skip_box_lean(a, lo, hi, bound, ca), rb = skip_box(b, lo, hi, bound, cb);
            if (ra != 2 && (ra != rb || ca != cb || (ra == 0 && memcmp(&a, &b, sizeof(Walk))))) {
                printf("  first bad skip: r %d/%d cells %u/%u X %u %u %u s %d %d %d lo %u %u %u hi %u %u %u\n"
                       "   t %a h %a %a %a d %a %a %a bound %a\n   lean t %a h %a %a %a XYZ %u %u %u\n   ref  t %a h %a %a %a XYZ %u %u %u\n",
                       ra, rb, ca, cb, w.X, w.Y, w.Z, w.sx, w.sy, w.sz, lo[0], lo[1], lo[2], hi[0], hi[1], hi[2], w.t, w.tx, w.ty,
                       w.tz, w.dx, w.dy, w.dz, bound, a.t, a.tx, a.ty, a.tz, a.X, a.Y, a.Z, b.t, b.tx, b.ty, b.tz, b.X, b.Y, b.Z);
                return;
            }
            if (ra == 2) goto step;
            w = a;
            if (ra == 1) return;
        }
    step:
        if (!step1(w, g.n)) return;
    }
}

// step1, both forms (the walkers' branch-free step), against the reference's branches (scene.cpp:773-802)
// on random heads drawn from a small value set, so ties, zeros, infinities and NaNs are common:
// the same axis, t, heads and cell.
static long check_step1(std::mt19937_64& r) {
    const float vals[] = {0.0f, -0.0f, 1.0f, 1.0f, 0.5f, 2.0f, 1e-30f, 3.4e38f, INFINITY, -INFINITY, NAN, 0.25f};
    long bad = 0;
    for (int i = 0; i < 2000000; ++i) {
        Walk a{};
        a.X = 5, a.Y = 6, a.Z = 7, a.sx = (r() & 1) ? 1 : -1, a.sy = (r() & 1) ? 1 : -1, a.sz = (r() & 1) ? 1 : -1;
        float* h[3] = {&a.tx, &a.ty, &a.tz};
        for (int k = 0; k < 3; ++k) *h[k] = (r() % 4) ? vals[r() % 12] : (float)(r() % 1000) * 0.001f;
        a.dx = 0.125f, a.dy = 0.25f, a.dz = 0.5f;
        Walk b = a, c = a;
        step1<true>(a, 64);
        step1<false>(c, 64);
        if (b.tx < b.ty) {
            if (b.tx < b.tz) b.t = b.tx, b.X += b.sx, b.tx += b.dx;
            else b.t = b.tz, b.Z += b.sz, b.tz += b.dz;
        } else {
            if (b.ty < b.tz) b.t = b.ty, b.Y += b.sy, b.ty += b.dy;
            else b.t = b.tz, b.Z += b.sz, b.tz += b.dz;
        }
        if (std::memcmp(&a, &b, sizeof(Walk)) || std::memcmp(&c, &b, sizeof(Walk))) {
            if (bad < 5) printf("step1 mismatch: heads %a %a %a\n", b.tx, b.ty, b.tz);
            ++bad;
        }
    }
    return bad;
}

int main(int argc, char** argv) {
    _mm_setcsr(_mm_getcsr() | 0x8040u);
    {
        std::mt19937_64 r0(12345);
        const long sb = check_step1(r0);
        printf("step1 vs reference branches: 2000000 states, step1 bad=%ld\n", sb);
        if (sb) return 1;
    }
    const long rays = argc > 1 ? atol(argv[1]) : 20000;
    long bad = 0, total = 0;
    uint64_t cells_all = 0;
    const uint32_t sizes[] = {64, 100, 128, 256, 1024};  // 1024: distance-field cubes up to 1020 cells
    for (uint32_t n : sizes) {
        for (double dens : {0.02, 0.2, 1.0}) {
            if (n > 256 && dens > 0.5) continue;
            World W = make_world(n, n * 31 + (uint64_t)(dens * 100), dens);
            std::mt19937_64 r(n + 7);
            bad += check_planes(W, r);
            std::uniform_real_distribution<float> U(0.f, 1.f);
            for (long i = 0; i < rays; ++i) {
                float O[3], T[3], D[3];
                const int kind = i % 4;
                for (int k = 0; k < 3; ++k) {
                    O[k] = kind == 0 ? U(r) : -0.6f + 2.2f * U(r);
                    T[k] = 0.05f + 0.9f * U(r);
                    D[k] = T[k] - O[k];
                }
                if (kind == 3) {  // axis-aligned / grid-aligned directions and origins on planes
                    const int ax = r() % 3;
                    for (int k = 0; k < 3; ++k) if (k != ax) D[k] = (r() % 2) ? 0.0f : D[k];
                    O[r() % 3] = (float)(r() % n) / (float)n;
                }
                const float len = std::sqrt(D[0] * D[0] + D[1] * D[1] + D[2] * D[2]);
                if (!(len > 0)) continue;
                for (int k = 0; k < 3; ++k) D[k] = D[k] * (1.0f / len);
                Walk s;
                if (!setup(n, O, D, s)) continue;
                const float bound = (i % 3 == 0) ? 1e34f : 0.2f + 2.0f * U(r);
                uint32_t c0 = 0, c1 = 0;
                Walk h0{}, h1 = s;
                const bool r0 = walk_naive(W, s, bound, c0, h0);
                const bool r1 = walk_skip(W.view(), h1, bound, c1);
                ++total;
                cells_all += c0;
                bool ok = r0 == r1 && c0 == c1;
                if (ok && r0) ok = std::memcmp(&h0.t, &h1.t, 4) == 0 && h0.X == h1.X && h0.Y == h1.Y && h0.Z == h1.Z;
                if (!ok) {
                    if (bad < 10)
                        printf("n=%u dens=%.2f ray %ld: hit %d/%d cells %u/%u t %a/%a cell (%u,%u,%u)/(%u,%u,%u)\n", n, dens, i, r0, r1, c0, c1,
                               h0.t, h1.t, h0.X, h0.Y, h0.Z, h1.X, h1.Y, h1.Z);
                    if (bad < 3) debug_walk(W.view(), s, bound);
                    ++bad;
                }
            }
        }
    }
    printf("rays=%ld cells=%llu bad=%ld\n", total, (unsigned long long)cells_all, bad);
    return bad ? 1 : 0;
}
