// vpx_persist.hpp — persistent, lane-refilling DDA kernels for single-volume scenes.
//
// A frame's rays differ in length by orders of magnitude (sky misses vs. grazing walks
// through the city), so a wave that owns 64 fixed rays idles most lanes while its longest
// ray finishes (measured: ~20 % lane utilisation in k_nearest).  These kernels keep every
// lane busy instead: a wave pulls rays from a work list in chunks of 256 (one returning
// atomic per chunk, not per ray), and whenever enough lanes have finished it refills them
// from the chunk while the other lanes keep stepping.  Each lane still walks exactly the
// reference DDA (Scene::FindNearest / Scene::IsOccluded, template/scene.cpp:751-811,
// 1009-1047) with the reference float arithmetic, so every result is unchanged.
//
// The single volume's transform, bounds and grid live in kernel arguments (SGPRs); the
// general N-volume path stays in vpx_wavefront.hpp.
#pragma once

#include "vpx_wavefront.hpp"

namespace vpx {

constexpr uint32_t kChunk = 256;        // rays per work-list grab
constexpr uint32_t kRefillMin = 16;     // refill when at least this many lanes are idle
constexpr int kBudget = 6;              // walker iterations between refill checks

struct OneVolume {
    vpx_volume vol;
    DevGrid g;
};

// Chunked work list: lanes of one wave share a chunk [base, base + 256).
struct WorkPool {
    uint32_t base, left;  // wave-uniform
    bool dry;             // the global list is exhausted
};

// Give idle lanes a work index (or 0xffffffff).  Wave-uniform control flow.
__device__ __forceinline__ uint32_t refill(WorkPool& pool, bool idle, uint32_t total, uint32_t* counter) {
    uint64_t mask = __ballot(idle);
    uint32_t got = 0xffffffffu;
    const uint32_t lane = threadIdx.x & 63u;
    while (mask) {
        if (pool.left == 0) {
            if (pool.dry) break;
            uint32_t b = 0;
            if (lane == 0) b = atomicAdd(counter, kChunk);
            b = __shfl(b, 0, 64);
            if (b >= total) {
                pool.dry = true;
                break;
            }
            pool.base = b;
            pool.left = min(kChunk, total - b);
        }
        const uint32_t nidle = (uint32_t)__popcll(mask);
        const uint32_t take = min(nidle, pool.left);
        // rank of this lane among the idle lanes
        const uint32_t rank = (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
        const bool mine = ((mask >> lane) & 1ull) && rank < take;
        if (mine) got = pool.base + rank;
        pool.base += take;
        pool.left -= take;
        // lanes that got work leave the idle mask
        mask &= ~__ballot(mine);
    }
    return got;
}

// ----------------------------------------------------------------------------
// Primary (FIRST) or bounce FindNearest over one volume, persistent.
// Work list: FIRST -> path ids 0..P-1; otherwise the active-path queue `list`.
template <bool FIRST>
__global__ __launch_bounds__(256) void k_nearest1(SceneView sv, OneVolume ov, FrameArgs f, WaveBufs w,
                                                  const uint32_t* __restrict__ list, const uint32_t* __restrict__ list_len,
                                                  uint32_t* __restrict__ counter, unsigned long long* __restrict__ ctr) {
    const uint32_t total = FIRST ? w.P : *list_len;
    const DevGrid g = ov.g;
    const uint32_t n = g.n;
    Counters k{0u, 0u, 0u};
    uint32_t prim = 0;
    WorkPool pool{0u, 0u, false};
    // lane state
    bool busy = false;
    uint32_t p = 0;
    Ray r;        // world ray (O, D, inside) + best hit
    ORay o;       // object-space ray
    skip::Walk wk;
    for (;;) {
        const uint64_t idle = __ballot(!busy);
        if (idle && (__popcll(idle) >= kRefillMin || idle == __ballot(true))) {
            const uint32_t got = refill(pool, !busy, total, counter);
            if (!busy && got != 0xffffffffu) {
                p = FIRST ? got : list[got];
                bool go = true;
                uint32_t flags = 0;
                if (FIRST) {
                    uint32_t x, y;
                    go = path_pixel(f, p, x, y);
                    w.depth[p] = f.max_bounces;
                    w.forms[p] = 0u;
                    w.leaf[p] = make_float4(0.f, 0.f, 0.f, 0.f);
                    uint32_t rng = 0;
                    if (go) {
                        Rng gg{pixel_seed(f.seed_base, f.frame_index, f.width, f.height, x, y)};
                        r = primary_ray(f, x, y, gg);
                        rng = gg.s;
                        ++prim;
                        flags = kActive;
                    } else {
                        r.O = r.D = mk(0.f, 0.f, 0.f);
                        r.inside = false;
                    }
                    if (f.max_bounces < 0) {
                        go = false;
                        flags = 0u;
                    }
                    w.O[p] = make_float4(r.O.x, r.O.y, r.O.z, __uint_as_float(rng));
                    w.D[p] = make_float4(r.D.x, r.D.y, r.D.z, __uint_as_float(flags));
                } else {
                    const float4 oo = w.O[p], dd = w.D[p];
                    r.O = mk(oo.x, oo.y, oo.z);
                    r.D = mk(dd.x, dd.y, dd.z);
                    r.inside = (__float_as_uint(dd.w) & kInside) != 0u;
                }
                if (go) {
                    ++k.nearest;
                    r.t = kBig;
                    r.mat = kNone;
                    r.N = mk(0.f, 0.f, 0.f);
                    o.O = xform_pos_ssem(r.O, ov.vol.inv_matrix);
                    o.D = xform_vec_ssem(r.D, ov.vol.inv_matrix);
                    o.rD = mk(1.0f / o.D.x, 1.0f / o.D.y, 1.0f / o.D.z);
                    Dda s;
                    if (dda_setup(ov.vol, n, o, s)) {
                        wk = to_walk(s);
                        busy = true;
                    } else {
                        busy = false;
                        // miss: no voxel hit; analytic shapes below
                    }
                    if (!busy) {
                        int32_t vox = -2;
                        if (sv.num_spheres | sv.num_triangles) {
                            Ray sh = make_ray(r.O, r.D);
                            for (uint32_t i = 0; i < sv.num_spheres; ++i) sphere_hit(sv.spheres[i], sh);
                            for (uint32_t i = 0; i < sv.num_triangles; ++i) tri_hit(sv.triangles[i], sh);
                            if (r.t > sh.t) {
                                r.t = sh.t, r.mat = sh.mat, r.N = sh.N, r.inside = sh.inside;
                                vox = -1;
                            }
                        }
                        w.H[p] = make_float4(r.t, r.N.x, r.N.y, r.N.z);
                        w.HM[p] = r.mat | ((uint32_t)(vox + 2) << 8) | (r.inside ? 0x80000000u : 0u);
                    }
                }
            }
        }
        if (!__ballot(busy) && pool.dry) break;
        if (!__ballot(busy) && pool.left == 0 && !pool.dry) continue;
        // ---- walk
        if (busy) {
            const int st = skip::walk_skip_some(grid_view(g), wk, r.t, k.cells, kBudget);
            const bool ended = st != 0, hit = st == 1;
            if (ended) {
                int32_t vox = -2;
                if (hit) {
                    r.t = wk.t;
                    r.N = normal_voxel(o, wk.t, n, ov.vol.matrix);
                    r.mat = g.cells[(uint64_t)wk.X + (uint64_t)wk.Y * n + (uint64_t)wk.Z * ((uint64_t)n * n)];
                    vox = 0;
                }
                if (sv.num_spheres | sv.num_triangles) {
                    Ray sh = make_ray(r.O, r.D);
                    for (uint32_t i = 0; i < sv.num_spheres; ++i) sphere_hit(sv.spheres[i], sh);
                    for (uint32_t i = 0; i < sv.num_triangles; ++i) tri_hit(sv.triangles[i], sh);
                    if (r.t > sh.t) {
                        r.t = sh.t, r.mat = sh.mat, r.N = sh.N, r.inside = sh.inside;
                        vox = -1;
                    }
                }
                w.H[p] = make_float4(r.t, r.N.x, r.N.y, r.N.z);
                w.HM[p] = r.mat | ((uint32_t)(vox + 2) << 8) | (r.inside ? 0x80000000u : 0u);
                busy = false;
            }
        }
    }
    flush_counters(k, prim, ctr);
}

// ----------------------------------------------------------------------------
// Renderer::IsOccluded over one volume for a compact list of shadow slots
// (entry = slot << 27 | path); sets kSlotOcc in the slot's flags.
constexpr uint32_t kSlotOcc = 4u;

__global__ __launch_bounds__(256) void k_shadow1(SceneView sv, OneVolume ov, WaveBufs w, const uint32_t* __restrict__ list,
                                                 const uint32_t* __restrict__ list_len, uint32_t* __restrict__ counter,
                                                 unsigned long long* __restrict__ ctr) {
    const uint32_t total = *list_len;
    const DevGrid g = ov.g;
    const uint32_t n = g.n;
    Counters k{0u, 0u, 0u};
    WorkPool pool{0u, 0u, false};
    bool busy = false;
    uint64_t slot = 0;
    float bound = 0.f;
    Ray r;
    skip::Walk wk;
    for (;;) {
        const uint64_t idle = __ballot(!busy);
        if (idle && (__popcll(idle) >= kRefillMin || idle == __ballot(true))) {
            const uint32_t got = refill(pool, !busy, total, counter);
            if (!busy && got != 0xffffffffu) {
                const uint32_t e = list[got];
                const uint32_t p = e & 0x07ffffffu, s_ = e >> 27;
                slot = (uint64_t)s_ * w.P + p;
                const float4 so = w.SO[slot], sd = w.SD[slot];
                r.O = mk(so.x, so.y, so.z);
                r.D = mk(sd.x, sd.y, sd.z);
                r.t = so.w;
                bound = so.w;
                ++k.shadow;
                ORay o;
                o.O = xform_pos(r.O, ov.vol.inv_matrix);
                o.D = xform_vec(r.D, ov.vol.inv_matrix);
                o.rD = mk(1.0f / o.D.x, 1.0f / o.D.y, 1.0f / o.D.z);
                Dda s;
                if (dda_setup(ov.vol, n, o, s)) {
                    wk = to_walk(s);
                    busy = true;
                } else {
                    bool occ = false;
                    for (uint32_t i = 0; i < sv.num_spheres && !occ; ++i) occ = sphere_is_hit(sv.spheres[i], r);
                    for (uint32_t i = 0; i < sv.num_triangles && !occ; ++i) occ = tri_is_hit(sv.triangles[i], r);
                    if (occ) w.SD[slot].w = __uint_as_float(__float_as_uint(sd.w) | kSlotOcc);
                }
            }
        }
        if (!__ballot(busy) && pool.dry) break;
        if (!__ballot(busy) && pool.left == 0 && !pool.dry) continue;
        if (busy) {
            const int st = skip::walk_skip_some(grid_view(g), wk, bound, k.cells, kBudget);
            const bool ended = st != 0;
            bool occ = st == 1;  // Scene::IsOccluded: first non-NONE cell with s.t < ray.t
            if (ended) {
                for (uint32_t i = 0; i < sv.num_spheres && !occ; ++i) occ = sphere_is_hit(sv.spheres[i], r);
                for (uint32_t i = 0; i < sv.num_triangles && !occ; ++i) occ = tri_is_hit(sv.triangles[i], r);
                if (occ) {
                    const float4 sd = w.SD[slot];
                    w.SD[slot].w = __uint_as_float(__float_as_uint(sd.w) | kSlotOcc);
                }
                busy = false;
            }
        }
    }
    flush_counters(k, 0u, ctr);
}

}  // namespace vpx
