// vpx_kernels.hip — gfx950 kernels and the C-ABI of libvpx_hip.so (include/vpx.h).
//
// Kernels:
//   k_nearest / k_shade / k_shadow / k_finish   the frame as a wavefront of small kernels
//                                 per bounce level (vpx_wavefront.hpp); one lane per pixel,
//                                 16x16-pixel tiles per 256-thread workgroup (8x8 pixels per wave)
//   composite_tiles               rank-0 unpack + accumulate + tonemap of gathered tiles.
//   composite_rgb8                rank-0 unpack of gathered RGB8 tiles (sharded accumulator).
//   find_nearest_k / is_occluded_k / trace_k   per-ray unit entries.
//   tiled_world_k / checksum_k    world generator and grid checksum.
#include <hip/hip_runtime.h>
#include <hip/hip_gl_interop.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <array>
#include <atomic>
#include <vector>

#include "vpx_wavefront.hpp"

using namespace vpx;

namespace {

constexpr int kTile = 16;  // 16x16 pixels per tile / 256-thread workgroup
#ifndef VPX_SPLIT_PRIMARY
#define VPX_SPLIT_PRIMARY 1  // multi-volume primary rays: lean world walk + instance pass (k_instances)
#ifndef VPX_DEFER_INSTANCES
#define VPX_DEFER_INSTANCES 1  // depth 0: the world head shades the paths no instance can change (DEFER)
#endif
#endif
#ifndef VPX_LANE_TAIL
#define VPX_LANE_TAIL 1  // frames in flight blend in their own tail launch where they have one (lane_tail_ok)
#endif
#ifndef VPX_LEVEL_FORK
#define VPX_LEVEL_FORK 1  // launch_render: a level's bounce walks beside its shadow walks
#endif
// k_tail: frames of at least VPX_TAIL_MIN_DEPTH bounces run their levels from VPX_TAIL_LEVEL on
// in one launch (0: off).
#ifndef VPX_LANE_DOUBLE
#define VPX_LANE_DOUBLE 1  // frames in flight: two sample buffers per lane (lane_render)
#endif
#ifndef VPX_TAIL_LEVEL
#define VPX_TAIL_LEVEL 7
#endif
#ifndef VPX_TAIL_MIN_DEPTH
#define VPX_TAIL_MIN_DEPTH 8
#endif
constexpr int kThreads = 256;

// One tile per workgroup.  Several tiles per workgroup with their loads issued together
// measured within noise (round 3, four interleaved runs, ms per step: C1 0.5829-0.5888 with 1,
// 0.5808-0.5907 with 2, 0.5780-0.5849 with 4, 0.5847-0.6010 with 8; C3 3.689-3.699 with 1,
// 3.674-3.711 with 4): the blend is not what a frame in flight waits for.
__global__ __launch_bounds__(kThreads) void composite_tiles(FrameArgs f, const float4* __restrict__ gathered,
                                                            float4* __restrict__ accum, uint32_t* __restrict__ rgb8) {
    const uint32_t tile = blockIdx.x;
    uint32_t lx, ly;
    tile_lane_xy(threadIdx.x, lx, ly);
    const uint32_t x = (tile % f.tiles_x) * kTile + lx;
    const uint32_t y = (tile / f.tiles_x) * kTile + ly;
    if (x >= f.width || y >= f.height) return;
    const uint32_t r = tile % f.n_ranks, j = tile / f.n_ranks;
    const float4 s = gathered[((uint64_t)r * f.tiles_per_rank + j) * (kTile * kTile) + threadIdx.x];
    const uint64_t p = (uint64_t)y * f.width + x;
    const float4 a = blend(accum[p], mk(s.x, s.y, s.z), f.weight, f.inv_weight);
    accum[p] = a;
    if (rgb8) rgb8[p] = tonemap_pack(a);
}

// A rank's packed frame folded into its packed accumulator + RGB8 (the frames-in-flight form
// of k_finish<kFinishPackedAccum>: the same blend and tonemap of the same sample, in frame order).
__global__ __launch_bounds__(kThreads) void blend_packed(FrameArgs f, const float4* __restrict__ sample,
                                                         float4* __restrict__ accum, uint32_t* __restrict__ rgb8, uint32_t P) {
    const uint32_t p = blockIdx.x * kThreads + threadIdx.x;
    if (p >= P) return;
    uint32_t x, y;
    if (path_pixel(f, p, x, y)) {
        const float4 s = sample[p];
        const float4 a = blend(accum[p], mk(s.x, s.y, s.z), f.weight, f.inv_weight);
        accum[p] = a;
        rgb8[p] = tonemap_pack(a);
    } else {
        accum[p] = make_float4(0.f, 0.f, 0.f, 0.f);
        rgb8[p] = 0u;
    }
}

// An accumulation window's samples (frame b of the chain at [b*T*256, (b+1)*T*256)) folded
// into the accumulator in frame order: per pixel the same blend of the same samples as B
// calls of k_finish / composite_tiles / blend_packed, and the tonemap of the last.  image:
// the one-GPU image (accum/rgb8 indexed by pixel); else a rank's packed accumulator.
__global__ __launch_bounds__(kThreads) void blend_window(FrameArgs f, const float4* __restrict__ sample, uint32_t B,
                                                         WindowWeights ww, int image, float4* __restrict__ accum,
                                                         uint32_t* __restrict__ rgb8) {
    const uint32_t T = f.batch_tiles;
    const uint32_t p = blockIdx.x * kThreads + threadIdx.x;
    uint32_t x, y;
    const bool valid = path_pixel(f, p, x, y);
    if (image && !valid) return;
    const uint64_t a_at = image ? (uint64_t)y * f.width + x : p;
    if (!valid) {
        accum[a_at] = make_float4(0.f, 0.f, 0.f, 0.f);
        rgb8[a_at] = 0u;
        return;
    }
    float4 a = accum[a_at];
    for (uint32_t b = 0; b < B; ++b) {
        const float4 s = sample[((uint64_t)b * T << 8) + p];
        a = blend(a, mk(s.x, s.y, s.z), ww.w[b], ww.iw[b]);
    }
    accum[a_at] = a;
    if (rgb8) rgb8[a_at] = tonemap_pack(a);
}

// Rank-0 scatter of the gathered packed RGB8 tiles (sharded-accumulator flow).
__global__ __launch_bounds__(kThreads) void composite_rgb8(FrameArgs f, const uint32_t* __restrict__ gathered,
                                                           uint32_t* __restrict__ rgb8) {
    const uint32_t tile = blockIdx.x;
    uint32_t lx, ly;
    tile_lane_xy(threadIdx.x, lx, ly);
    const uint32_t x = (tile % f.tiles_x) * kTile + lx;
    const uint32_t y = (tile / f.tiles_x) * kTile + ly;
    if (x >= f.width || y >= f.height) return;
    const uint32_t r = tile % f.n_ranks, j = tile / f.n_ranks;
    rgb8[(uint64_t)y * f.width + x] = gathered[((uint64_t)r * f.tiles_per_rank + j) * (kTile * kTile) + threadIdx.x];
}

// ------------------------------------------------------------------ unit entries
__device__ __forceinline__ Ray ray_from(const vpx_ray& in) {
    Ray r = make_ray(ld3(in.origin), ld3(in.direction));
    r.t = in.tmax;
    r.inside = in.inside_glass != 0;
    return r;
}

__global__ void find_nearest_k(SceneView sv, const vpx_ray* rays, uint32_t n, vpx_hit* hits) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Ray r = ray_from(rays[i]);
    Counters k{0u, 0u, 0u};
    const int32_t vox = find_nearest(sv, r, k);
    vpx_hit h;
    h.t = r.t;
    h.normal[0] = r.N.x, h.normal[1] = r.N.y, h.normal[2] = r.N.z;
    h.vox_index = vox;
    h.material = r.mat;
    h.cells = k.cells;
    h.inside_glass = r.inside ? 1u : 0u;
    hits[i] = h;
}

__global__ void is_occluded_k(SceneView sv, const vpx_ray* rays, uint32_t n, uint8_t* occ) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Ray r = ray_from(rays[i]);
    Counters k{0u, 0u, 0u};
    occ[i] = is_occluded(sv, r, k) ? 1 : 0;
}

// BasicBVH::IntersectBVH (src/BVH/BasicBVH.cpp:19-70), one ray per lane.  The workgroup
// stages the whole BVH in LDS (nodes, then the triangles already permuted into tri_idx
// order, so a leaf's triangles are contiguous); the recursion (node test, then left
// subtree, then right) becomes an explicit stack that pops the left child first.  Float
// expressions keep the reference's operand order: IEEE divisions, std::min / std::max.
constexpr int kBvhStack = 64;
__global__ __launch_bounds__(256) void bvh_intersect_k(const uint32_t* __restrict__ bvh, uint32_t n_nodes,
                                                       uint32_t n_tris, const vpx_ray* rays, uint32_t n,
                                                       float* t_out) {
    extern __shared__ uint32_t lds_bvh[];
    const uint32_t words = n_nodes * 8u + n_tris * 9u;
    for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) lds_bvh[i] = bvh[i];
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const vpx_bvh_node* nodes = (const vpx_bvh_node*)lds_bvh;
    const vpx_bvh_tri* tris = (const vpx_bvh_tri*)(lds_bvh + n_nodes * 8u);
    Ray r = ray_from(rays[i]);
    uint32_t stack[kBvhStack];
    int sp = 0;
    stack[sp++] = 0;
    while (sp > 0) {
        const vpx_bvh_node& nd = nodes[stack[--sp]];
        // IntersectAABB (BasicBVH.cpp:38-48)
        const float tx1 = (nd.aabb_min[0] - r.O.x) / r.D.x, tx2 = (nd.aabb_max[0] - r.O.x) / r.D.x;
        float tmin = smin(tx1, tx2), tmax = smax(tx1, tx2);
        const float ty1 = (nd.aabb_min[1] - r.O.y) / r.D.y, ty2 = (nd.aabb_max[1] - r.O.y) / r.D.y;
        tmin = smax(tmin, smin(ty1, ty2)), tmax = smin(tmax, smax(ty1, ty2));
        const float tz1 = (nd.aabb_min[2] - r.O.z) / r.D.z, tz2 = (nd.aabb_max[2] - r.O.z) / r.D.z;
        tmin = smax(tmin, smin(tz1, tz2)), tmax = smin(tmax, smax(tz1, tz2));
        if (!(tmax >= tmin && tmin < r.t && tmax > 0)) continue;
        if (nd.tri_count == 0) {  // interior: left subtree first
            stack[sp++] = nd.left_first + 1u;
            stack[sp++] = nd.left_first;
            continue;
        }
        for (uint32_t k = 0; k < nd.tri_count; ++k) {  // IntersectTri (BasicBVH.cpp:19-36)
            const vpx_bvh_tri& t = tris[nd.left_first + k];
            const f3 v0 = ld3(t.v0);
            const f3 e1 = ld3(t.v1) - v0, e2 = ld3(t.v2) - v0;
            const f3 h = cross(r.D, e2);
            const float a = dot(e1, h);
            if (a > -0.0001f && a < 0.0001f) continue;
            const float f = __fdiv_rn(1.0f, a);
            const f3 sv = r.O - v0;
            const float u = f * dot(sv, h);
            if (u < 0 || u > 1) continue;
            const f3 q = cross(sv, e1);
            const float v = f * dot(r.D, q);
            if (v < 0 || u + v > 1) continue;
            const float tt = f * dot(e2, q);
            if (tt > 0.0001f) r.t = smin(r.t, tt);
        }
    }
    t_out[i] = r.t;
}

template <int LEVELS>
__global__ __launch_bounds__(256) void trace_k(SceneView sv, const vpx_ray* rays, const uint32_t* seeds, uint32_t n, int32_t depth,
                        float* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Rng g{seeds[i]};
    Counters k{0u, 0u, 0u};
    const f3 v = trace_path<LEVELS>(sv, ray_from(rays[i]), depth, g, k);
    out[3 * i] = v.x, out[3 * i + 1] = v.y, out[3 * i + 2] = v.z;
}

__global__ void focus_k(SceneView sv, FrameArgs f, float* out) {
    // Renderer::Tick focus ray (renderer.cpp:1987-1991): integer screen centre, no lens
    // jitter, tested against each Scene in WORLD space (no instance transform).
    const float u = (float)(f.width / 2) * __fdiv_rn(1.0f, (float)f.width);
    const float v = (float)(f.height / 2) * __fdiv_rn(1.0f, (float)f.height);
    const f3 tl = ld3(f.cam.top_left), tr = ld3(f.cam.top_right), bl = ld3(f.cam.bottom_left);
    const f3 P = (tl + (tr - tl) * u) + (bl - tl) * v;
    const f3 cp = ld3(f.cam.cam_pos);
    const f3 focal = cp + normalize(P - cp) * f.cam.focal_distance;
    Ray r = make_ray(cp, focal - cp);
    uint32_t cells = 0;
    for (uint32_t i = 0; i < sv.num_volumes; ++i) {
        const vpx_volume& vol = sv.volumes[i];
        ORay o{r.O, r.D, mk(__fdiv_rn(1.0f, r.D.x), __fdiv_rn(1.0f, r.D.y), __fdiv_rn(1.0f, r.D.z))};
        const DevGrid g = sv.grids[vol.grid_id];
        Dda s;
        if (!dda_setup(vol, g.n, o, s)) continue;
        skip::Walk w = to_walk(s);
        if (skip::walk_skip(grid_view(g), w, r.t, cells)) r.t = w.t;
    }
    *out = smax(-1.0f, smin(r.t, 1e4f));
}

// --------------------------------------------------------------- world kernels
__global__ void tiled_world_k(uint8_t* __restrict__ out, uint32_t n, const uint8_t* __restrict__ model, uint32_t mx,
                              uint32_t my, uint32_t mz, uint32_t px, uint32_t py, uint32_t pz, uint32_t ground) {
    // one thread per 16 consecutive x-cells of a row (n % 16 == 0) or per cell otherwise
    const uint64_t n64 = n;
    const bool wide = (n % 16u) == 0;
    const uint64_t per_row = wide ? n64 / 16 : n64;
    const uint64_t total = per_row * n64 * n64;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t row = i / per_row;
        const uint64_t x0 = (i % per_row) * (wide ? 16 : 1);
        const uint64_t y = row % n64, z = row / n64;
        uint8_t vals[16];
        const int cnt = wide ? 16 : 1;
        if (y < ground) {
            for (int c = 0; c < cnt; ++c) vals[c] = VPX_MAT_NON_METAL_WHITE;
        } else {
            const uint64_t ly = (y - ground) % py, lz = z % pz;
            for (int c = 0; c < cnt; ++c) {
                const uint64_t lx = (x0 + c) % px;
                vals[c] = (lx < mx && ly < my && lz < mz) ? model[lx + ly * mx + lz * mx * my] : (uint8_t)kNone;
            }
        }
        uint8_t* dst = out + z * n64 * n64 + y * n64 + x0;
        if (wide) {
            uint4 w;
            memcpy(&w, vals, 16);
            *reinterpret_cast<uint4*>(dst) = w;
        } else {
            dst[0] = vals[0];
        }
    }
}

// ------------------------------------------------------------- occupancy masks
// Layout: vpx_skip.hpp blk_index (l1, l2 blocked by parent) / lin_index (l3).
// l1: one thread per output word (padded space nb2^3 * 64) reads its brick's 64 cells.
__global__ void build_l1_k(const uint8_t* __restrict__ cells, uint32_t n, uint32_t nb1, uint32_t nb2,
                           uint64_t* __restrict__ l1) {
    const uint64_t total = (uint64_t)nb2 * nb2 * nb2 * 64;
    const uint64_t n64 = n;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < total; s += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t parent = s >> 6;
        const uint32_t j = (uint32_t)(s & 63u);
        const uint32_t bx = (uint32_t)(parent % nb2) * 4 + (j & 3u);
        const uint32_t by = (uint32_t)((parent / nb2) % nb2) * 4 + ((j >> 2) & 3u);
        const uint32_t bz = (uint32_t)(parent / ((uint64_t)nb2 * nb2)) * 4 + (j >> 4);
        uint64_t m = 0;
        if (bx < nb1 && by < nb1 && bz < nb1) {
            for (uint32_t lz = 0; lz < 4; ++lz)
                for (uint32_t ly = 0; ly < 4; ++ly) {
                    const uint32_t y = by * 4 + ly, z = bz * 4 + lz;
                    if (y >= n || z >= n) continue;
                    const uint8_t* row = cells + (uint64_t)y * n64 + (uint64_t)z * n64 * n64;
                    for (uint32_t lx = 0; lx < 4; ++lx) {
                        const uint32_t x = bx * 4 + lx;
                        if (x < n && row[x] != kNone) m |= 1ull << (lx + 4 * ly + 16 * lz);
                    }
                }
        }
        l1[s] = m;
    }
}

// One level up: the word of parent block P (np parents per axis, linear P) ORs the 64
// consecutive child words child[P*64 + j] into bit j (child words are fresh cell masks).
// Output blocked by grandparent (ngp per axis, words ngp^3 * 64).
__global__ void build_up_k(const uint64_t* __restrict__ child, uint32_t np, uint32_t ngp, uint64_t* __restrict__ out) {
    const uint64_t total = (uint64_t)ngp * ngp * ngp * 64;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < total; s += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t gp = s >> 6;
        const uint32_t j = (uint32_t)(s & 63u);
        const uint32_t px = (uint32_t)(gp % ngp) * 4 + (j & 3u);
        const uint32_t py = (uint32_t)((gp / ngp) % ngp) * 4 + ((j >> 2) & 3u);
        const uint32_t pz = (uint32_t)(gp / ((uint64_t)ngp * ngp)) * 4 + (j >> 4);
        uint64_t m = 0;
        if (px < np && py < np && pz < np) {
            const uint64_t* c = child + (((uint64_t)pz * np + py) * np + px) * 64;
            for (uint32_t j = 0; j < 64; ++j) m |= (c[j] != 0ull ? 1ull : 0ull) << j;
        }
        out[s] = m;
    }
}

// Region rebuild after an edit: the l1 words of bricks [b0, b0 + cnt) (per axis), then
// the l2 / l3 words of their parents.  Same words as build_l1_k / build_up_k compute.
__global__ void build_l1_box_k(const uint8_t* __restrict__ cells, uint32_t n, uint32_t nb2, uint64_t* __restrict__ l1,
                               uint32_t bx0, uint32_t by0, uint32_t bz0, uint32_t cx, uint32_t cy, uint32_t cz) {
    const uint64_t total = (uint64_t)cx * cy * cz;
    const uint64_t n64 = n;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t bx = bx0 + (uint32_t)(i % cx), by = by0 + (uint32_t)((i / cx) % cy),
                       bz = bz0 + (uint32_t)(i / ((uint64_t)cx * cy));
        uint64_t m = 0;
        for (uint32_t lz = 0; lz < 4; ++lz)
            for (uint32_t ly = 0; ly < 4; ++ly) {
                const uint32_t y = by * 4 + ly, z = bz * 4 + lz;
                if (y >= n || z >= n) continue;
                const uint8_t* row = cells + (uint64_t)y * n64 + (uint64_t)z * n64 * n64;
                for (uint32_t lx = 0; lx < 4; ++lx) {
                    const uint32_t x = bx * 4 + lx;
                    if (x < n && row[x] != kNone) m |= 1ull << (lx + 4 * ly + 16 * lz);
                }
            }
        l1[skip::blk_index(bx, by, bz, nb2)] = m;
    }
}

__global__ void build_up_box_k(const uint64_t* __restrict__ child, uint32_t np, uint32_t ngp, uint64_t* __restrict__ out,
                               uint32_t px0, uint32_t py0, uint32_t pz0, uint32_t cx, uint32_t cy, uint32_t cz) {
    const uint64_t total = (uint64_t)cx * cy * cz;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t px = px0 + (uint32_t)(i % cx), py = py0 + (uint32_t)((i / cx) % cy),
                       pz = pz0 + (uint32_t)(i / ((uint64_t)cx * cy));
        const uint64_t* c = child + (((uint64_t)pz * np + py) * np + px) * 64;
        uint64_t m = 0;
        for (uint32_t j = 0; j < 64; ++j) m |= (c[j] != 0ull ? 1ull : 0ull) << j;
        out[skip::blk_index(px, py, pz, ngp)] = m;
    }
}

// One plane fx + fy + fz = s of the distance-field sweep (build_df), thread = (fx, fy,
// octant o); (fx, fy, fz) are brick coordinates flipped so that octant o's "ahead" is +1.
// Reads bytes o of the words on planes s+1..s+3 (earlier launches), writes plane s.
__global__ void df_plane_k(uint8_t* __restrict__ l1b, const uint64_t* __restrict__ l2, uint32_t nb1, uint32_t nb2,
                           uint32_t nb3, uint32_t s) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t o = (uint32_t)(t & 7u);
    const uint64_t q = t >> 3;
    const uint32_t fx = (uint32_t)(q % nb1), fy = (uint32_t)(q / nb1);
    if (fy >= nb1 || fx + fy > s || s - fx - fy >= nb1) return;
    const uint32_t fz = s - fx - fy;
    const uint32_t x = (o & 1u) ? nb1 - 1u - fx : fx, y = (o & 2u) ? nb1 - 1u - fy : fy, z = (o & 4u) ? nb1 - 1u - fz : fz;
    auto occ = [&](uint32_t a, uint32_t b, uint32_t c) -> bool {
        return (l2[skip::blk_index(a >> 2, b >> 2, c >> 2, nb3)] >> ((a & 3u) | ((b & 3u) << 2) | ((c & 3u) << 4))) & 1ull;
    };
    if (occ(x, y, z)) return;
    auto get = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t oo) -> uint32_t {
        return l1b[(size_t)skip::blk_index(a, b, c, nb2) * 8 + oo];
    };
    l1b[(size_t)skip::blk_index(x, y, z, nb2) * 8 + o] = skip::df_value(x, y, z, o, nb1, occ, get);
}

// The octant planes from the built levels (after build_df): byte o of an empty brick's l1
// word into plane o, 0 for an occupied brick (and for the padding bricks, never walked).
__global__ void build_planes_k(const uint64_t* __restrict__ l1, const uint64_t* __restrict__ l2, uint32_t nb2,
                               uint32_t nb3, uint8_t* __restrict__ dfp) {
    const uint64_t plane = (uint64_t)nb2 * nb2 * nb2 * 64;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < plane; s += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t parent = s >> 6;
        const uint32_t j = (uint32_t)(s & 63u);
        const uint32_t bx = (uint32_t)(parent % nb2) * 4 + (j & 3u);
        const uint32_t by = (uint32_t)((parent / nb2) % nb2) * 4 + ((j >> 2) & 3u);
        const uint32_t bz = (uint32_t)(parent / ((uint64_t)nb2 * nb2)) * 4 + (j >> 4);
        const bool occ = (l2[skip::blk_index(bx >> 2, by >> 2, bz >> 2, nb3)] >> ((bx & 3u) | ((by & 3u) << 2) | ((bz & 3u) << 4))) & 1ull;
        const uint64_t m = occ ? 0ull : l1[s];
#pragma unroll
        for (uint32_t o = 0; o < 8; ++o) dfp[o * plane + s] = (uint8_t)(m >> (8 * o));
    }
}

// Scatter a staged box (x fastest) into the grid.
__global__ void write_box_k(uint8_t* __restrict__ grid, uint32_t n, const uint8_t* __restrict__ src, uint32_t x0,
                            uint32_t y0, uint32_t z0, uint32_t dx, uint32_t dy, uint32_t dz) {
    const uint64_t total = (uint64_t)dx * dy * dz;
    const uint64_t n64 = n;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t x = i % dx, y = (i / dx) % dy, z = i / ((uint64_t)dx * dy);
        grid[(x0 + x) + (y0 + y) * n64 + (z0 + z) * n64 * n64] = src[i];
    }
}

// Scene::CreateEmmisiveSphere (template/scene.cpp:685-711) over the sphere's bounding box:
// point = float3(x, y, z), d = length(float3(worldsize / 2) - point) (sqrtf of the
// left-to-right dot), set when d < radius.
__global__ void emissive_sphere_k(uint8_t* __restrict__ grid, uint32_t n, uint8_t mat, float radius, uint32_t x0,
                                  uint32_t cnt) {
    const uint64_t total = (uint64_t)cnt * cnt * cnt;
    const uint64_t n64 = n;
    const float c = (float)n / 2.0f;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t x = x0 + (uint32_t)(i % cnt), y = x0 + (uint32_t)((i / cnt) % cnt), z = x0 + (uint32_t)(i / ((uint64_t)cnt * cnt));
        const float vx = c - (float)x, vy = c - (float)y, vz = c - (float)z;
        const float d = sqrtf(vx * vx + vy * vy + vz * vz);
        if (d < radius) grid[x + y * n64 + z * n64 * n64] = mat;
    }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

__global__ void checksum_k(const uint8_t* __restrict__ cells, uint64_t count, unsigned long long* out) {
    uint64_t s = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count;
         i += (uint64_t)gridDim.x * blockDim.x)
        s += (uint64_t)(cells[i] + 1u) * splitmix64(i);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)s);
}

}  // namespace

// =========================================================================== host side
struct vpx_ctx {
    int device = 0;
    uint32_t cus = 256;  // compute units of the device (the bounce pool's grid)
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    struct GridBuf {
        uint8_t* ptr = nullptr;
        uint64_t* l1 = nullptr;
        uint64_t* l2 = nullptr;
        uint8_t* dfp = nullptr;  // distance-field octant planes (build_planes_k)
        uint32_t n = 0, nb1 = 0, nb2 = 0, nb3 = 0;
        uint64_t plane() const { return 64ull * nb2 * nb2 * nb2; }
    };
    std::vector<GridBuf> grids;
    DevGrid* d_grids = nullptr;
    uint32_t d_grids_cap = 0;
    std::vector<vpx_volume> volumes;
    vpx_volume* d_volumes = nullptr;
    float4* d_vbounds = nullptr;  // per volume: its cube's inflated world box (lo, hi), see volume_bounds
    void* d_tlas = nullptr;       // instance TLAS: nodes, then the leaf volume list (build_tlas)
    uint32_t tlas_nodes = 0;
    bool tlas_on = false;
    uint64_t tlas_always = 0;
    void* d_bvh = nullptr;        // BasicBVH: nodes, then the triangles in tri_idx order (vpx_bvh_set)
    uint32_t bvh_nodes = 0, bvh_tris = 0;
    uint32_t d_volumes_cap = 0;
    vpx_material* d_materials = nullptr;
    vpx_point_light* d_points = nullptr;
    vpx_spot_light* d_spots = nullptr;
    vpx_area_light* d_areas = nullptr;
    vpx_sphere* d_spheres = nullptr;
    vpx_triangle* d_triangles = nullptr;
    uint32_t n_points = 0, n_spots = 0, n_areas = 0, n_spheres = 0, n_triangles = 0;
    vpx_dir_light dir{{1, 0, 0}, {0, 0, 0}};  // DirectionalLight default (DirectionalLight.h:12)
    vpx_camera cam{};
    bool have_materials = false, have_camera = false;
    // sky dome (vpx_set_sky): RGB float texels, equirectangular
    float* d_sky = nullptr;
    uint32_t sky_w = 0, sky_h = 0;
    float sky_hdr = 1.0f;
    // reference arithmetic (vpx_set_arithmetic): the host's captured rcpss / rsqrtss tables
    uint32_t* d_x86 = nullptr;
    X86Arith x86{nullptr, 0u, 0u, 0u, 0u};
    unsigned long long* d_ctr = nullptr;  // striped work counters (vpx_wavefront.hpp flush_counters)
    // per-stage profile: event pairs around stage launches while enabled
    std::vector<hipEvent_t> prof_ev;
    std::vector<int> prof_stage;
    uint32_t prof_cap = 0, prof_used = 0;
    uint32_t prof_mask = 0xffffffffu;  // stages timed (vpx_profile_select)
    unsigned long long* d_sum = nullptr;
    void* d_scratch = nullptr;
    size_t scratch_bytes = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
    // wavefront path state (vpx_wavefront.hpp), grown on demand: one store per stream that
    // renders (the caller's stream, and each pipeline lane)
    struct WaveStore {
        void* d = nullptr;
        size_t bytes = 0;
        WaveBufs w{};
        // the level fork (launch_render): a second stream for the bounce walks, forked after a
        // level's shade and joined before the next one's, so that they overlap the shadow walks
        hipStream_t fork = nullptr;
        hipEvent_t ev_fork = nullptr, ev_join = nullptr;
        bool fork_dedicated = false;  // on a CU-mask stream, counted in g_lane_queues
    };
    WaveStore wave;
    // frames in flight (vpx_set_pipeline): each lane renders a whole frame on its own library
    // stream into its own path state and packed sample buffer; the caller's stream only runs
    // the frames' composites, in frame order (each waits for its lane's render), so frame f+1's
    // walks fill the GPU while frame f's last tiles drain.  Empty: frames render on the stream.
    struct Lane {
        hipStream_t s = nullptr;
        WaveStore ws;
        float4* packed = nullptr;  // the lane's frame: one float4 sample per path (tile order)
        float4* packed2 = nullptr; // its second buffer (frames alternate: VPX_LANE_DOUBLE)
        size_t packed_len = 0;
        hipEvent_t rendered = nullptr, consumed = nullptr, consumed2 = nullptr;
        bool used2 = false;
        uint32_t flip = 0;
        float4* cur = nullptr;             // the buffer of the lane's latest frame (lane_render)
        hipEvent_t cur_consumed = nullptr; // the event its blend records
        hipEvent_t caller = nullptr;  // the caller's stream at the frame's vpx_render (lane_tail_ok frames)
        bool used = false;
        bool dedicated = false;  // on a CU-mask stream (its own hardware queue), counted in g_lane_queues
    };
    std::vector<Lane> lanes;
    uint32_t lane_next = 0;
    // static-camera path images (float4[W*H] each): albedo, illumination, ray data, temp
    float4* rp_buf = nullptr;
    size_t rp_pixels = 0;
    // a window chain's samples when no lanes run (vpx_render_window)
    float4* win_buf = nullptr;
    size_t win_len = 0;
    // device set (vpx_create_multi): one member context per device; this context only
    // forwards (VPX_GROUP_*) and runs the tile-sharded vpx_render (group_render)
    std::vector<vpx_ctx*> members;
    std::vector<ncclComm_t> comms;      // RCCL, one per member (distinct devices only)
    std::vector<void*> g_packed;        // per member: packed float4 samples / RGB8 (member device)
    std::vector<float*> g_accum;        // per member: packed accumulator (accum == NULL mode)
    void* g_gathered = nullptr;         // member 0's device: the members' packed buffers back to back
    size_t g_len = 0;                   // float4 elements per member buffer the above were sized for
    std::vector<hipEvent_t> g_ev;       // per member: its render done (copy path)
    hipEvent_t g_copied = nullptr;      // member 0: gather copies done (copy path)
    // display interop (vpx_gl_*): a registered GL pixel-unpack buffer on this context's
    // device (device set: devices[0]); mapped between vpx_gl_map and vpx_gl_unmap
    hipGraphicsResource_t gl_res = nullptr;
    bool gl_mapped = false;
};

namespace {

int fail(vpx_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

// Wait for everything the context has queued: its stream and its pipeline lanes (frames in
// flight read the world, tables and path buffers that later calls may replace).
hipError_t sync_all(vpx_ctx* c) {
    for (const auto& l : c->lanes)
        if (l.s) {
            const hipError_t e = hipStreamSynchronize(l.s);
            if (e != hipSuccess) return e;
        }
    return hipStreamSynchronize(c->stream);
}

// The caller's current HIP device, restored when the scope ends: a device-set call sets each
// member's device in turn and must not leave the caller on the last one (torch tensors or
// buffers the caller allocates afterwards belong on devices[0]).
struct DeviceGuard {
    int dev = -1;
    DeviceGuard() {
        if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    }
    ~DeviceGuard() {
        if (dev >= 0) (void)hipSetDevice(dev);
    }
};

// Device-set contexts forward to their members: every member (uploads / state) or member 0
// (unit entries, profiles, the single-image static-camera path, the rank-level primitives).
template <class F>
int group_all(vpx_ctx* c, F f) {
    DeviceGuard keep;
    for (vpx_ctx* m : c->members) {
        if (hipSetDevice(m->device) != hipSuccess) return fail(c, VPX_E_DEVICE, "hipSetDevice");
        const int rc = f(m);
        if (rc) return fail(c, rc, "device " + std::to_string(m->device) + ": " + m->err);
    }
    return VPX_OK;
}
template <class F>
int group_first(vpx_ctx* c, F f) {
    DeviceGuard keep;
    vpx_ctx* m = c->members[0];
    if (hipSetDevice(m->device) != hipSuccess) return fail(c, VPX_E_DEVICE, "hipSetDevice");
    const int rc = f(m);
    return rc ? fail(c, rc, m->err) : VPX_OK;
}
#define VPX_GROUP_ALL(c, call) \
    if ((c) && !(c)->members.empty()) return group_all((c), [&](vpx_ctx* m_) { return call; })
#define VPX_GROUP_FIRST(c, call) \
    if ((c) && !(c)->members.empty()) return group_first((c), [&](vpx_ctx* m_) { return call; })

#define VPX_HIP(c, expr)                                                                            \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess)                                                                       \
            return fail((c), e_ == hipErrorOutOfMemory ? VPX_E_NOMEM : VPX_E_DEVICE,                \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                         \
    } while (0)

template <typename T>
int upload_table(vpx_ctx* c, T*& dst, const T* src, uint32_t n) {
    if (dst) {
        (void)hipFree(dst);
        dst = nullptr;
    }
    if (n == 0) return VPX_OK;
    if (!src) return fail(c, VPX_E_INVALID, "null table with non-zero count");
    VPX_HIP(c, hipMalloc(&dst, sizeof(T) * n));
    VPX_HIP(c, hipMemcpyAsync(dst, src, sizeof(T) * n, hipMemcpyHostToDevice, c->stream));
    return VPX_OK;
}

int ensure_scratch(vpx_ctx* c, size_t bytes) {
    if (bytes <= c->scratch_bytes) return VPX_OK;
    if (c->d_scratch) (void)hipFree(c->d_scratch);
    c->d_scratch = nullptr;
    c->scratch_bytes = 0;
    VPX_HIP(c, hipMalloc(&c->d_scratch, bytes));
    c->scratch_bytes = bytes;
    return VPX_OK;
}

int check_ready(vpx_ctx* c) {
    if (c->volumes.empty()) return fail(c, VPX_E_STATE, "no volumes set (vpx_set_volumes)");
    if (!c->have_materials) return fail(c, VPX_E_STATE, "no materials set (vpx_set_materials)");
    for (const auto& v : c->volumes) {
        if (v.grid_id >= c->grids.size() || !c->grids[v.grid_id].ptr)
            return fail(c, VPX_E_STATE, "volume references a grid that was not uploaded");
    }
    return VPX_OK;
}

int sync_grids(vpx_ctx* c) {
    const uint32_t n = (uint32_t)c->grids.size();
    if (n > c->d_grids_cap) {
        if (c->d_grids) (void)hipFree(c->d_grids);
        c->d_grids = nullptr;
        VPX_HIP(c, hipMalloc(&c->d_grids, sizeof(DevGrid) * n));
        c->d_grids_cap = n;
    }
    std::vector<DevGrid> h(n);
    for (uint32_t i = 0; i < n; ++i) {
        const auto& g = c->grids[i];
        h[i] = DevGrid{g.ptr, g.l1, g.l2, g.n, g.nb1, g.nb2, g.nb3, g.dfp, g.plane()};
    }
    if (n) VPX_HIP(c, hipMemcpy(c->d_grids, h.data(), sizeof(DevGrid) * n, hipMemcpyHostToDevice));
    return VPX_OK;
}

SceneView view_of(const vpx_ctx* c, const float sky[3], int32_t area_samples, bool sky_tex = false) {
    SceneView sv;
    sv.grids = c->d_grids;
    sv.volumes = c->d_volumes;
    sv.vbounds = c->d_vbounds;
    sv.tlas = (const TlasNode*)c->d_tlas;
    sv.tlas_on = c->tlas_on ? 1u : 0u;
    sv.tlas_nodes = c->tlas_nodes;
    sv.tlas_always = c->tlas_always;
    sv.materials = c->d_materials;
    sv.points = c->d_points;
    sv.spots = c->d_spots;
    sv.areas = c->d_areas;
    sv.spheres = c->d_spheres;
    sv.triangles = c->d_triangles;
    sv.num_volumes = (uint32_t)c->volumes.size();
    sv.num_points = c->n_points;
    sv.num_spots = c->n_spots;
    sv.num_areas = c->n_areas;
    sv.num_spheres = c->n_spheres;
    sv.num_triangles = c->n_triangles;
    sv.dir = c->dir;
    sv.sky[0] = sky[0], sv.sky[1] = sky[1], sv.sky[2] = sky[2];
    sv.area_samples = area_samples;
    sv.sky_px = c->d_sky;
    sv.sky_w = c->sky_w, sv.sky_h = c->sky_h;
    sv.sky_hdr = c->sky_hdr;
    sv.sky_tex = (sky_tex && c->d_sky) ? 1u : 0u;
    sv.x86 = c->x86;
    // one grid for every volume after the world: lane_volumes (vpx_trace.hpp)
    sv.inst_grid = -1;
    for (size_t i = 1; i < c->volumes.size(); ++i) {
        const int32_t gi = (int32_t)c->volumes[i].grid_id;
        if (i == 1) sv.inst_grid = gi;
        else if (gi != sv.inst_grid) { sv.inst_grid = -1; break; }
    }
    return sv;
}

FrameArgs frame_of(const vpx_ctx* c, const vpx_frame_params* p, uint32_t rank, uint32_t n_ranks) {
    FrameArgs f;
    f.cam = c->cam;
    f.width = p->width;
    f.height = p->height;
    f.max_bounces = p->max_bounces;
    f.frame_index = p->frame_index;
    f.seed_base = p->seed_base;
    f.flags = p->flags;
    f.aa = p->aa_strength;
    f.weight = 1.0f / ((float)p->frame_index + 1.0f);  // renderer.cpp:1651
    f.inv_weight = 1.0f - f.weight;
    f.tiles_x = (p->width + kTile - 1) / kTile;
    f.tiles_y = (p->height + kTile - 1) / kTile;
    f.num_tiles = f.tiles_x * f.tiles_y;
    f.rank = rank;
    f.n_ranks = n_ranks;
    f.tiles_per_rank = (f.num_tiles + n_ranks - 1) / n_ranks;
    f.batch_tiles = 0;
    return f;
}

int validate_frame(vpx_ctx* c, const vpx_frame_params* p) {
    if (!p) return fail(c, VPX_E_INVALID, "null frame params");
    if (p->width == 0 || p->height == 0 || p->width > 32768 || p->height > 32768)
        return fail(c, VPX_E_INVALID, "frame size out of range");
    // the shadow lists pack a path index into 27 bits beside the slot number (shadow_tile)
    if ((uint64_t)((p->width + kTile - 1) / kTile) * ((p->height + kTile - 1) / kTile) * (uint64_t)kTilePix > (1ull << 27))
        return fail(c, VPX_E_INVALID, "frame larger than 2^27 tile-padded pixels");
    if (p->max_bounces < -1 || p->max_bounces > kMaxLevels - 2)
        return fail(c, VPX_E_INVALID, "max_bounces must be in [-1, 14]");
    if (p->area_samples < 0 || p->area_samples > 15) return fail(c, VPX_E_INVALID, "area_samples must be in [0, 15]");
    if (!c->have_camera) return fail(c, VPX_E_STATE, "no camera set (vpx_set_camera)");
    if ((p->flags & VPX_FLAG_SKY) && !c->d_sky)
        return fail(c, VPX_E_STATE, "VPX_FLAG_SKY without a sky texture (vpx_set_sky)");
    return check_ready(c);
}

// Carve the wavefront buffers for P paths, L levels and S shadow slots out of one
// device allocation (grown on demand; never inside a capture).
int ensure_wave(vpx_ctx* c, vpx_ctx::WaveStore& ws, uint32_t P, uint32_t L, uint32_t S) {
    const size_t f4 = sizeof(float4);
    const size_t bytes = (size_t)P * (f4 * (5 + 2 * (size_t)L + 3 * (size_t)S + 1) + 3 * sizeof(uint32_t)) +
                         sizeof(uint32_t) * (size_t)P * 3 + (size_t)P / 8 + sizeof(uint32_t) * kPoolWords +
                         (size_t)P * S + sizeof(uint32_t) * (size_t)P * S + 22 * 256;
    if (bytes > ws.bytes) {
        if (ws.d) {
            VPX_HIP(c, sync_all(c));
            (void)hipFree(ws.d);
        }
        ws.d = nullptr;
        ws.bytes = 0;
        VPX_HIP(c, hipMalloc(&ws.d, bytes));
        ws.bytes = bytes;
    }
    char* q = (char*)ws.d;
    auto take = [&](size_t n) {
        char* r = q;
        q += (n + 255) & ~(size_t)255;
        return (void*)r;
    };
    WaveBufs& w = ws.w;
    w.P = P;
    w.S = S;
    w.O = (float4*)take(f4 * P);
    w.D = (float4*)take(f4 * P);
    w.H = (float4*)take(f4 * P);
    w.leaf = (float4*)take(f4 * P);
    w.SM = (float4*)take(f4 * P);
    w.LA = (float4*)take(f4 * P * (size_t)L);
    w.LB = (float4*)take(f4 * P * (size_t)L);
    w.SO = (float4*)take(f4 * P * (size_t)S);
    w.SD = (float4*)take(f4 * P * (size_t)S);
    w.SL = (float4*)take(f4 * P * (size_t)S);
    w.HM = (uint32_t*)take(4 * (size_t)P);
    w.depth = (int32_t*)take(4 * (size_t)P);
    w.forms = (uint32_t*)take(4 * (size_t)P);
    w.smask = (uint32_t*)take(4 * (size_t)P);
    w.live0 = (uint32_t*)take(4 * (size_t)P);
    w.live1 = (uint32_t*)take(4 * (size_t)P);
    w.amask = (uint64_t*)take((size_t)P / 8);  // P is a multiple of 256
    w.pool = (uint32_t*)take(sizeof(uint32_t) * kPoolWords);
    w.occb = (uint8_t*)take((size_t)P * S);
    (void)take(sizeof(uint32_t) * (size_t)P * S);  // slot_list (vpx_wavefront.hpp), right after occb
    return VPX_OK;
}

std::atomic<int> g_lane_queues{0};
constexpr int kMaxLaneQueues = 16;

// The level fork's stream and events (created on first use): a CU-mask stream of all the
// device's CUs (a hardware queue of its own) while the process's lane-queue cap allows, else
// a plain non-blocking stream.  Its work always joins back into the owner's stream within the
// frame, so synchronising the owner covers it.
void free_fork(vpx_ctx::WaveStore& ws);
int ensure_fork(vpx_ctx* c, vpx_ctx::WaveStore& ws) {
    if (ws.fork && ws.ev_fork && ws.ev_join) return VPX_OK;
    free_fork(ws);  // a partly created fork (an earlier failure): start clean
    std::vector<uint32_t> all_cus((c->cus + 31u) / 32u, 0xffffffffu);
    ws.fork_dedicated = g_lane_queues.fetch_add(1) < kMaxLaneQueues;
    if (!ws.fork_dedicated) g_lane_queues.fetch_sub(1);
    const hipError_t se = ws.fork_dedicated
                              ? hipExtStreamCreateWithCUMask(&ws.fork, (uint32_t)all_cus.size(), all_cus.data())
                              : hipStreamCreateWithFlags(&ws.fork, hipStreamNonBlocking);
    if (se != hipSuccess) ws.fork = nullptr;
    if (se != hipSuccess || hipEventCreateWithFlags(&ws.ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ws.ev_join, hipEventDisableTiming) != hipSuccess) {
        free_fork(ws);  // releases the counted queue and whatever was created
        return fail(c, VPX_E_DEVICE, "level fork: stream / event creation failed");
    }
    return VPX_OK;
}
void free_fork(vpx_ctx::WaveStore& ws) {
    if (ws.fork) (void)hipStreamSynchronize(ws.fork);
    if (ws.ev_fork) (void)hipEventDestroy(ws.ev_fork);
    if (ws.ev_join) (void)hipEventDestroy(ws.ev_join);
    if (ws.fork) (void)hipStreamDestroy(ws.fork);
    if (ws.fork_dedicated) g_lane_queues.fetch_sub(1);
    ws.fork = nullptr, ws.ev_fork = ws.ev_join = nullptr, ws.fork_dedicated = false;
}

// Profile marks: a stage's start (stage >= 0) or end (-1) event on the stream, while the
// event pool lasts; a start without room for its end is not recorded.
static void prof_mark(vpx_ctx* c, hipStream_t s, int stage) {
    if (!c->prof_cap) return;
    if (stage >= 0 && !((c->prof_mask >> stage) & 1u)) return;  // not selected (its end is dropped too)
    if (stage >= 0 && c->prof_used + 2 > c->prof_cap) return;
    if (stage < 0 && (c->prof_used & 1u) == 0) return;  // its start was dropped
    if (hipEventRecord(c->prof_ev[c->prof_used], s) != hipSuccess) return;
    c->prof_stage[c->prof_used] = stage;
    ++c->prof_used;
}

// The frame: primary -> [shade -> shadow -> resolve -> nearest]* -> finish, all on
// c->stream, one 256-thread workgroup per 16x16 tile in every kernel.
struct Reproj {  // the static-camera tail (vpx_render_reproject)
    PrevCam prev;
    float4 *alb, *ill, *rd, *temp, *hist;
};

// tail_wait: an event the frame's separate tail launch (k_resolve_finish, after the shadow
// pool) waits for — frames in flight that blend on their own lane (lane_tail_ok).  wtail: a
// window chain (tiles = B frames' tiles) whose separate tail blends its frames in order
// (k_finish_window) instead of writing samples.
template <int MODE>
int launch_render(vpx_ctx* c, hipStream_t s, vpx_ctx::WaveStore& ws, const SceneView& sv, const FrameArgs& f,
                  uint32_t tiles, float4* accum, uint32_t* rgb8, float4* packed, const Reproj* rp = nullptr,
                  const hipEvent_t* tail_wait = nullptr, const WindowTail* wtail = nullptr) {
    const uint32_t P = tiles * (uint32_t)kTilePix;
    const uint32_t L = (uint32_t)std::max(1, f.max_bounces + 1);
    // shadow slots per path: an area-light sample each, else one (point / spot / directional
    // lights and the smoke probe use slot 0 only)
    const uint32_t S = sv.num_areas ? (uint32_t)std::max(1, sv.area_samples) : 1u;
    int rc = ensure_wave(c, ws, P, L, S);
    if (rc) return rc;
    WaveBufs w = ws.w;
    if (rp) w.RD = rp->rd;
    const dim3 grid(tiles), block(kThreads);
    const size_t slds = sizeof(uint32_t) * S * kThreads;
    // single volume, no analytic shapes: the DDA kernels' lean instances
    const bool one = sv.num_volumes == 1 && !(sv.num_spheres | sv.num_triangles);
    const bool x86 = sv.x86.tab != nullptr;  // the reference-arithmetic instances of the hot kernels
    // the multi-volume walkers' rcp table in LDS (x86_stage_lds): its dynamic LDS bytes
    const size_t xlds = x86 ? sizeof(uint32_t) * sv.x86.rsq_off : 0;
    // the last level's shadow -> resolve -> finish as one launch (k_shadow_finish), except
    // on the static-camera path, whose tail is the reprojection
    const bool fuse_tail = !rp;
    // The shadow pool (k_shadow_pool, results in occb) for the single-volume walks towards area
    // lights (several slots per path, long walks), except on the static-camera path (its
    // reprojection test reads the tile kernel's SD flags).  Measured (ms per step, two runs
    // each, pool / tile kernels): C3 3.72, 3.71 / 4.96, 4.94; C2 (one point light, one slot per
    // path) 2.83, 2.84 / 2.64, 2.71 (round 3) — so point / spot / directional lights kept the
    // tile kernels; since round 6 single-volume frames in flight use the pool for them too
    // (VPX_SPOOL_ONE_SLOT below: C2 -2.4 %).
    // Multi-volume / shape scenes: the world's walks (volume 0, first in IsOccluded's loop) in
    // the pool, the rest of the loop for the slots the world left unoccluded: k_shadow_inst per
    // tile (round 3: C4 51.7 -> 47.6 ms per 16-spp step), then (round 6) k_shadow_slots over the
    // pool's list of the slots whose segment may meet a later volume.
// Round 6: single-volume frames with one slot per path (C2's point light) through the pool
// too — C2 at 3 lanes 2.294-2.353 vs 2.352-2.400 ms per step (three interleaved runs; at 2
// lanes with forks 2.45-2.47 vs 2.40-2.41).  (Round 3, before the live lists and the lanes'
// double buffers, it had measured 2.83 vs 2.64-2.71.)
#ifndef VPX_SPOOL_ONE_SLOT
#define VPX_SPOOL_ONE_SLOT 1
#endif
// Only for frames in flight: the serial frames (the context's stream, with the level fork)
// keep the tile kernels — C2 serial 3.32-3.33 ms per frame vs 3.51-3.54 with the pool (tile
// kernels everywhere: 3.31-3.35 serial, 2.35-2.39 in flight; three interleaved runs).
#ifndef VPX_SPOOL_ONE_SERIAL
#define VPX_SPOOL_ONE_SERIAL 0
#endif
    const bool spool = !rp && (S > 1 || (one && VPX_SPOOL_ONE_SLOT && (VPX_SPOOL_ONE_SERIAL || &ws != &c->wave)));
    if (wtail && (!spool || f.max_bounces < 0 || !f.batch_tiles || tiles % wtail->B))
        return fail(c, VPX_E_INVALID, "window tail: needs a window chain with the shadow pool");
    if (!spool) w.occb = nullptr;  // k_resolve reads the slots' SD flags
    const uint32_t sgrab = std::max(1u, std::min(4u, kShadowList / (64u * S)));
    // persistent launches over a level's live list (its length is on the device): as many
    // workgroups as the device keeps resident, capped by the frame's tiles
    auto resident = [&](uint32_t waves_per_simd) { return dim3(std::min(tiles, c->cus * waves_per_simd)); };
    auto shadow_pool = [&](int level) {
        const uint32_t grabs = (P / 64u + sgrab - 1u) / sgrab;
        const uint32_t waves = std::min(grabs, c->cus * 4u * (uint32_t)VPX_WPE_SPOOL);
        const uint32_t wpb = kPoolWg / 64u;
        hipLaunchKernelGGL(one ? k_shadow_pool<false> : k_shadow_pool<true>, dim3((waves + wpb - 1u) / wpb), dim3(kPoolWg), 0,
                           s, sv, w, level, sgrab, c->d_ctr);
        if (!one)  // the pool's list of the slots a later volume may occlude
            hipLaunchKernelGGL(k_shadow_slots, dim3(std::min(tiles * S, c->cus * (uint32_t)VPX_WPE_SHADOW_SLOTS)), block, 0, s, sv,
                               w, level, c->d_ctr);
    };
    if (one && fuse_tail && f.max_bounces == 0 && tiles <= kFuseFrameTiles && S == 1 && !f.batch_tiles) {
        // the whole depth-0 frame in one launch (k_frame0), its path state and one shadow slot
        // per path in LDS; with area lights the frame splits to use the shadow pool
        prof_mark(c, s, VPX_STAGE_FRAME);
#ifndef VPX_FRAME_EXTRA_LDS
#define VPX_FRAME_EXTRA_LDS 0  // A/B hook: bytes of unused LDS added per k_frame0 workgroup (occupancy sensitivity)
#endif
        hipLaunchKernelGGL((x86 ? k_frame0<true, MODE, true> : k_frame0<true, MODE, false>), grid, block,
                           slds + VPX_FRAME_EXTRA_LDS, s, sv, f, w, c->d_ctr, accum, rgb8, packed);
        prof_mark(c, s, -1);
        VPX_HIP(c, hipGetLastError());
        return VPX_OK;
    }
    // the frame's level counters (grabs, live-list lengths; kPool*): zeroed before the head,
    // whose level-0 shade appends level 1's list
    VPX_HIP(c, hipMemsetAsync(w.pool, 0, sizeof(uint32_t) * kPoolWords, s));
    prof_mark(c, s, VPX_STAGE_PRIMARY);
    const bool fuse_head = f.max_bounces >= 0;  // level 0's shade at the end of k_primary
    // multi-volume / shape scenes: the world walk in the lean head, then the instance pass
    // (the rest of FindNearest for the rays that can still meet a later volume or a shape, and
    // level 0's shade; k_instances)
    // (scenes with analytic shapes test them on every ray, so no ray skips the second pass
    // there: they keep the one-launch kernel — Z1 2.61-2.62 vs 2.63 ms split, round 4)
    const bool split = !one && fuse_head && VPX_SPLIT_PRIMARY && !(sv.num_spheres | sv.num_triangles);
    // at depth 0 the world head shades the paths that cannot meet an instance itself and the
    // instance pass takes only the others (k_primary / k_instances DEFER)
    const bool defer = split && f.max_bounces == 0 && VPX_DEFER_INSTANCES;
    if (defer)
        hipLaunchKernelGGL((x86 ? k_primary<true, true, true, true> : k_primary<true, true, false, true>), grid, block, 0, s,
                           sv, f, w, c->d_ctr);
    else if (split)
        hipLaunchKernelGGL((x86 ? k_primary<true, false, true> : k_primary<true, false, false>), grid, block, 0, s, sv, f, w,
                           c->d_ctr);
    else if (fuse_head)
        hipLaunchKernelGGL((one ? (x86 ? k_primary<true, true, true> : k_primary<true, true, false>)
                                : (x86 ? k_primary<false, true, true> : k_primary<false, true, false>)),
                           grid, block, 0, s, sv, f, w,
                           c->d_ctr);
    else
        hipLaunchKernelGGL((one ? (x86 ? k_primary<true, false, true> : k_primary<true, false, false>)
                                : (x86 ? k_primary<false, false, true> : k_primary<false, false, false>)),
                           grid, block, 0, s, sv, f,
                           w, c->d_ctr);
    prof_mark(c, s, -1);
    if (split) {
        prof_mark(c, s, VPX_STAGE_INSTANCES);
        if (defer) {  // the deferred paths as a dense list (k_compact), then k_instances_list
            hipLaunchKernelGGL(k_compact, dim3((P / 64u + 255u) / 256u), block, 0, s, w, 0);
            hipLaunchKernelGGL(k_instances_list, grid, block, xlds, s, sv, f, w, c->d_ctr);
        } else {
            hipLaunchKernelGGL(k_instances, grid, block, xlds, s, sv, f, w, c->d_ctr);
        }
        prof_mark(c, s, -1);
    }
    // FindNearest for the traced rays of the next level: the bounce pool (single volume, no
    // shapes) or the tile kernel
    auto bounce = [&](hipStream_t bs, int level) {
        prof_mark(c, bs, VPX_STAGE_BOUNCE);
        if (one) {  // the bounce pool: persistent waves, as many as the device keeps resident
            const uint32_t chunks = (P + kPoolChunk - 1u) / kPoolChunk;
            const uint32_t waves = std::min(chunks, c->cus * 4u * (uint32_t)VPX_WPE_BOUNCE);
            const uint32_t wpb = kPoolWg / 64u;
            hipLaunchKernelGGL(x86 ? k_nearest_pool<true> : k_nearest_pool<false>, dim3((waves + wpb - 1u) / wpb),
                               dim3(kPoolWg), 0, bs, sv, w, level,
                               c->d_ctr);
        } else {  // multi-volume / shape scenes: persistent waves over the live list, 64 rays a grab
            hipLaunchKernelGGL(k_nearest_tile, grid, block, xlds, bs, sv, w, level, c->d_ctr);
        }
        prof_mark(c, bs, -1);
    };
    // Where it pays (ms per step, one MI355X, tools/gpu_r4h/j/k.sh): every frame on the
    // context's stream (serial C2 3.70-3.74 vs 4.49-4.54, Z1 3.44-3.47 vs 3.89-3.90), and
    // single-volume frames in flight with at most two lanes (C2 at 2 lanes 2.50-2.52 vs 2.65-2.67
    // at the 3 lanes without forks).  Not with three or more lanes (C2 3.17-3.28 at 3, 4.0-4.3 at
    // 4: more dedicated queues than the device runs at once; forks from the shared queue pool
    // 2.80-2.86), nor for multi-volume / shape frames in flight (Z1 3.20-3.25 at 2 lanes vs
    // 2.50 at 3 without).
    const bool fork = VPX_LEVEL_FORK && f.max_bounces > 0 && !rp && (&ws == &c->wave || (one && c->lanes.size() <= 2));
    if (fork && (rc = ensure_fork(c, ws))) return rc;
    // deep frames: the levels from tail_from on in one launch (k_tail), then k_finish
    // (frames on the context's stream — a per-frame synchronous Tick — start it a level earlier:
    // with no other frame to overlap, the per-level latency costs more; Z1 serial 2.50 from
    // level 6 vs 2.65 from 7, 2.69 from 5; frames in flight 1.54 from 7 vs 1.56-1.64 from 6)
    const int tail_at = &ws == &c->wave ? VPX_TAIL_LEVEL - 1 : VPX_TAIL_LEVEL;
    const int tail_from = (VPX_TAIL_LEVEL > 0 && f.max_bounces >= VPX_TAIL_MIN_DEPTH && !rp) ? tail_at : -1;
    bool tailed = false;
    // the last level's shadow -> resolve -> finish as one launch (k_shadow_finish)
    for (int level = 0; level <= f.max_bounces; ++level) {
        if (!(fuse_head && level == 0)) {  // (level >= 1: the head shades level 0)
            prof_mark(c, s, VPX_STAGE_SHADE);
            hipLaunchKernelGGL(k_shade, grid, block, 0, s, sv, f, w, level, c->d_ctr);
            prof_mark(c, s, -1);
        }
        if (fuse_tail && level == f.max_bounces) {
            prof_mark(c, s, VPX_STAGE_SHADOW);
            if (spool)
                shadow_pool(level);
            else
                hipLaunchKernelGGL((one ? k_shadow_finish<true, MODE> : k_shadow_finish<false, MODE>), grid, block,
                                   slds, s, sv, f, w, c->d_ctr, accum, rgb8, packed);
            prof_mark(c, s, -1);
            if (spool) {
                if (tail_wait) VPX_HIP(c, hipStreamWaitEvent(s, *tail_wait, 0));
                prof_mark(c, s, VPX_STAGE_FINISH);
                if (wtail)
                    hipLaunchKernelGGL(k_finish_window<true>, dim3(tiles / wtail->B), block, 0, s, sv, f, w, *wtail,
                                       accum, rgb8);
                else
                    hipLaunchKernelGGL((k_resolve_finish<MODE>), grid, block, 0, s, sv, f, w, accum, rgb8, packed);
                prof_mark(c, s, -1);
            }
            break;
        }
        // the next level's live list from this level's shade bits
        if (level < f.max_bounces)
            hipLaunchKernelGGL(k_compact, dim3((P / 64u + 255u) / 256u), block, 0, s, w, level);
        // the level fork: the next level's bounce walks read only the rays and live list this
        // level's shade and k_compact wrote and write only the hit records, which the shadow
        // walks and the light sums do not touch — so they run beside them on the fork stream
        const bool tail_next = level + 1 == tail_from;  // the next levels run in k_tail
        const bool forked = fork && level < f.max_bounces && !tail_next;
        if (forked) {
            VPX_HIP(c, hipEventRecord(ws.ev_fork, s));
            VPX_HIP(c, hipStreamWaitEvent(ws.fork, ws.ev_fork, 0));
            bounce(ws.fork, level);
            VPX_HIP(c, hipEventRecord(ws.ev_join, ws.fork));
        }
        prof_mark(c, s, VPX_STAGE_SHADOW);
        if (spool)
            shadow_pool(level);
        else if (level == 0)
            hipLaunchKernelGGL(one ? k_shadow_tile<true> : k_shadow_tile<false>, grid, block, slds, s, sv, w, c->d_ctr);
        else
            hipLaunchKernelGGL(one ? k_shadow_list<true> : k_shadow_list<false>, grid, block, slds, s, sv, w, level,
                               c->d_ctr);
        prof_mark(c, s, -1);
        prof_mark(c, s, VPX_STAGE_RESOLVE);
        hipLaunchKernelGGL(k_resolve, level ? resident(8) : grid, block, 0, s, sv, w, level);
        prof_mark(c, s, -1);
        if (forked)
            VPX_HIP(c, hipStreamWaitEvent(s, ws.ev_join, 0));
        else if (level < f.max_bounces && !tail_next)
            bounce(s, level);
        if (tail_next) {
            WaveBufs wt = w;
            wt.occb = nullptr;  // k_tail marks occluded slots in their SD words, as the tile kernels do
            prof_mark(c, s, VPX_STAGE_BOUNCE);
            hipLaunchKernelGGL(k_tail, grid, block, xlds, s, sv, f, wt, level + 1, c->d_ctr);
            prof_mark(c, s, -1);
            tailed = true;
            break;
        }
    }
    // (fused tail: k_shadow_finish already finished the frame; max_bounces = -1 runs no
    // level, so the finish folds the zero leaf here)
    const bool finished = fuse_tail && f.max_bounces >= 0 && !tailed;
    // a frame in flight that blends on its lane (tail_wait) blends here when k_tail ran: the
    // blend must follow the caller's earlier writes and the previous frame's blend
    if (!finished && tail_wait) VPX_HIP(c, hipStreamWaitEvent(s, *tail_wait, 0));
    if (!finished) prof_mark(c, s, VPX_STAGE_FINISH);
    if (!rp) {
        if (!finished && wtail)
            hipLaunchKernelGGL(k_finish_window<false>, dim3(tiles / wtail->B), block, 0, s, sv, f, w, *wtail, accum,
                               rgb8);
        else if (!finished)
            hipLaunchKernelGGL((k_finish<MODE>), grid, block, 0, s, f, w, accum, rgb8, packed);
    } else {  // Renderer::Tick static branch, second pass (renderer.cpp:2024-2100)
        hipLaunchKernelGGL(k_finish_reproject, grid, block, 0, s, f, w, rp->alb, rp->ill);
        hipLaunchKernelGGL(k_reproject_setup, grid, block, 0, s, f, w, rp->prev);
        hipLaunchKernelGGL(one ? k_shadow_tile<true> : k_shadow_tile<false>, grid, block, slds, s, sv, w, c->d_ctr);
        hipLaunchKernelGGL(k_reproject_resolve, grid, block, 0, s, f, w, rp->alb, rp->ill, rp->hist, rp->temp,
                           rgb8);
        VPX_HIP(c, hipMemcpyAsync(rp->hist, rp->temp, sizeof(float4) * (size_t)f.width * f.height,
                                  hipMemcpyDeviceToDevice, s));  // history = temp
    }
    if (!finished) prof_mark(c, s, -1);
    VPX_HIP(c, hipGetLastError());
    return VPX_OK;
}

// Whether a frame's blend can run as its own tail launch on the lane (launch_render's spool
// tail, k_resolve_finish): area lights with several samples (the shadow pool).
bool lane_tail_ok(const SceneView& sv, const FrameArgs& f) {
    const uint32_t S = sv.num_areas ? (uint32_t)std::max(1, sv.area_samples) : 1u;
    return VPX_LANE_TAIL && S > 1 && f.max_bounces >= 0;
}

// Frames in flight: render `tiles` tiles of frame f as packed float4 samples (into `out`, or
// the lane's own buffer when null) on the next lane's stream, in that lane's path state; the
// caller's stream waits for the render.  The caller then queues the frame's composite on
// s and records the lane's `consumed` event after it.
int lane_render(vpx_ctx* c, const SceneView& sv, const FrameArgs& f, uint32_t tiles, float4* out, vpx_ctx::Lane*& lane) {
    vpx_ctx::Lane& L = c->lanes[c->lane_next];
    c->lane_next = (c->lane_next + 1u) % (uint32_t)c->lanes.size();
    float4* dst = out;
    // Two sample buffers per lane, alternating: the lane's next frame waits only for the blend
    // of the frame before its previous one, not for the previous one's (which waits for every
    // earlier blend on the caller's stream).  The path state needs no wait: the lane's frames
    // run in its stream's order, and the blends read only the samples.
    const uint32_t b = L.flip;
    L.flip = VPX_LANE_DOUBLE ? L.flip ^ 1u : 0u;
    if (!dst) {
        const size_t need = (size_t)tiles * kTilePix;
        if (L.packed_len < need) {
            VPX_HIP(c, sync_all(c));
            if (L.packed) (void)hipFree(L.packed);
            if (L.packed2) (void)hipFree(L.packed2);
            L.packed = L.packed2 = nullptr;
            L.packed_len = 0;
            VPX_HIP(c, hipMalloc(&L.packed, sizeof(float4) * need));
            if (VPX_LANE_DOUBLE) VPX_HIP(c, hipMalloc(&L.packed2, sizeof(float4) * need));
            L.packed_len = need;
        }
        dst = b ? L.packed2 : L.packed;
    }
    bool& used = b ? L.used2 : L.used;
    L.cur = dst;
    L.cur_consumed = b ? L.consumed2 : L.consumed;
    // this buffer's previous frame has been blended
    if (used) VPX_HIP(c, hipStreamWaitEvent(L.s, L.cur_consumed, 0));
    int rc = launch_render<kFinishPackedSample>(c, L.s, L.ws, sv, f, tiles, nullptr, nullptr, dst);
    if (rc) return rc;
    VPX_HIP(c, hipEventRecord(L.rendered, L.s));
    VPX_HIP(c, hipStreamWaitEvent(c->stream, L.rendered, 0));
    used = true;
    lane = &L;
    return VPX_OK;
}

// Lanes on dedicated hardware queues across the process (every context, every device-set
// member; level forks too): each takes a queue of its own, so the count is capped
// (kMaxLaneQueues, g_lane_queues above); lanes past the cap are plain non-blocking streams
// from the shared pool.

void free_lanes(vpx_ctx* c) {
    for (auto& L : c->lanes) {
        if (L.dedicated) g_lane_queues.fetch_sub(1);
        if (L.s) (void)hipStreamSynchronize(L.s);
        free_fork(L.ws);
        if (L.ws.d) (void)hipFree(L.ws.d);
        if (L.packed) (void)hipFree(L.packed);
        if (L.packed2) (void)hipFree(L.packed2);
        if (L.rendered) (void)hipEventDestroy(L.rendered);
        if (L.consumed) (void)hipEventDestroy(L.consumed);
        if (L.consumed2) (void)hipEventDestroy(L.consumed2);
        if (L.caller) (void)hipEventDestroy(L.caller);
        if (L.s) (void)hipStreamDestroy(L.s);
    }
    c->lanes.clear();
    c->lane_next = 0;
}

int snapshot_counters(vpx_ctx* c, unsigned long long out[kCtrWords]) {
    unsigned long long all[kCtrWords * kCtrStripes];
    VPX_HIP(c, hipMemcpyAsync(all, c->d_ctr, sizeof(all), hipMemcpyDeviceToHost, c->stream));
    VPX_HIP(c, sync_all(c));
    for (uint32_t i = 0; i < kCtrWords; ++i) {
        out[i] = 0;
        for (uint32_t s = 0; s < kCtrStripes; ++s) out[i] += all[kCtrWords * s + i];
    }
    return VPX_OK;
}

void fill_stats(vpx_stats* s, const unsigned long long a[kCtrWords], const unsigned long long b[kCtrWords]) {
    s->shadow_rays = b[0] - a[0];
    s->primary_rays = b[3] - a[3];
    const unsigned long long nearest = b[1] - a[1];  // 0 for Trace(ray, -1): no bounce rays
    s->bounce_rays = nearest > s->primary_rays ? nearest - s->primary_rays : 0;
    s->dda_cells = b[2] - a[2];
}

}  // namespace

// =============================================================================== C-ABI
extern "C" {

int vpx_abi_version(void) { return VPX_ABI_VERSION; }

int vpx_create(int device, vpx_ctx** out) {
    if (!out) return VPX_E_INVALID;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return VPX_E_DEVICE;
    if (device < 0 || device >= count) return VPX_E_INVALID;
    if (hipSetDevice(device) != hipSuccess) return VPX_E_DEVICE;
    vpx_ctx* c = new (std::nothrow) vpx_ctx();
    if (!c) return VPX_E_NOMEM;
    c->device = device;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
        c->cus = (uint32_t)cus;
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&c->d_ctr, kCtrWords * kCtrStripes * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&c->d_sum, sizeof(unsigned long long)) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipEventCreate(&c->ev2) != hipSuccess) {
        vpx_destroy(c);
        return VPX_E_DEVICE;
    }
    c->stream = c->own_stream;
    (void)hipMemset(c->d_ctr, 0, kCtrWords * kCtrStripes * sizeof(unsigned long long));
    *out = c;
    return VPX_OK;
}

int vpx_destroy(vpx_ctx* c) {
    if (!c) return VPX_E_INVALID;
    if (c->gl_res) {  // a context destroyed while its GL buffer is mapped: unmap, then unregister
        vpx_ctx* h = c->members.empty() ? c : c->members[0];
        (void)hipSetDevice(h->device);
        if (c->gl_mapped) (void)hipGraphicsUnmapResources(1, &c->gl_res, h->stream);
        (void)hipGraphicsUnregisterResource(c->gl_res);
        c->gl_res = nullptr;
        c->gl_mapped = false;
    }
    if (!c->members.empty()) {  // device set: its buffers, communicators and members
        DeviceGuard keep;
        for (size_t r = 0; r < c->members.size(); ++r) {
            vpx_ctx* m = c->members[r];
            (void)hipSetDevice(m->device);
            (void)hipStreamSynchronize(m->stream);
            if (r < c->g_packed.size() && c->g_packed[r]) (void)hipFree(c->g_packed[r]);
            if (r < c->g_accum.size() && c->g_accum[r]) (void)hipFree(c->g_accum[r]);
            if (r < c->g_ev.size() && c->g_ev[r]) (void)hipEventDestroy(c->g_ev[r]);
            if (r == 0) {
                if (c->g_gathered) (void)hipFree(c->g_gathered);
                if (c->g_copied) (void)hipEventDestroy(c->g_copied);
            }
        }
        for (ncclComm_t cm : c->comms) (void)ncclCommDestroy(cm);
        for (vpx_ctx* m : c->members) vpx_destroy(m);
        delete c;
        return VPX_OK;
    }
    (void)hipSetDevice(c->device);
    if (c->stream) (void)sync_all(c);
    free_lanes(c);
    free_fork(c->wave);
    for (auto& g : c->grids) {
        if (g.ptr) (void)hipFree(g.ptr);
        if (g.l1) (void)hipFree(g.l1);
        if (g.l2) (void)hipFree(g.l2);
        if (g.dfp) (void)hipFree(g.dfp);
    }
    void* ptrs[] = {c->d_grids, c->d_volumes, c->d_vbounds, c->d_tlas, c->d_bvh, c->d_materials, c->d_points, c->d_spots, c->d_areas,
                    c->d_spheres, c->d_triangles, c->d_ctr, c->d_sum, c->d_scratch, c->wave.d, c->d_sky, c->d_x86};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    for (hipEvent_t e : c->prof_ev) (void)hipEventDestroy(e);
    if (c->rp_buf) (void)hipFree(c->rp_buf);
    if (c->win_buf) (void)hipFree(c->win_buf);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->ev2) (void)hipEventDestroy(c->ev2);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
    return VPX_OK;
}

const char* vpx_last_error(const vpx_ctx* c) { return c ? c->err.c_str() : "null context"; }

int vpx_set_stream(vpx_ctx* c, void* s) {
    if (!c) return VPX_E_INVALID;
    if (!c->members.empty()) return vpx_set_stream(c->members[0], s);  // a stream of the first device
    VPX_HIP(c, sync_all(c));
    // (the context's own stream is kept while unused: releasing it measured slower with
    // pipeline lanes — C2 3.75 vs 2.97 ms at 3 lanes — the lanes' hardware-queue sharing
    // changes with the number of live streams)
    c->stream = s ? (hipStream_t)s : c->own_stream;
    return VPX_OK;
}

int vpx_set_pipeline(vpx_ctx* c, uint32_t depth) {
    VPX_GROUP_ALL(c, vpx_set_pipeline(m_, depth));
    if (!c) return VPX_E_INVALID;
    if (depth > 4) return fail(c, VPX_E_INVALID, "pipeline depth must be in [0, 4]");
    VPX_HIP(c, hipSetDevice(c->device));
    VPX_HIP(c, sync_all(c));
    free_lanes(c);
    if (depth < 2) return VPX_OK;
    // the context's own level fork (taken by a depth > 0 frame on the context's stream) gives
    // its dedicated queue back: the lanes need them, and it is recreated if such a frame comes
    free_fork(c->wave);
    c->lanes.resize(depth);
    // Each lane on a hardware queue of its own.  Plain streams share the process's pool of
    // GPU_MAX_HW_QUEUES (4) queues: a kernel trace shows two of three lanes on one queue and
    // the third on the caller's (blend) queue, so a lane's frame waited behind another's.  A
    // stream with an explicit CU mask (here: every CU) gets a dedicated queue.  Measured on
    // one box (C1 ms, two processes x two contexts, 20 frames): 3 lanes 0.551-0.554 vs
    // 0.578-0.598 on pooled streams (4 pooled lanes 0.567-0.572, 4 dedicated 0.578-0.594).
    int n_cu = 0;
    VPX_HIP(c, hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, c->device));
    std::vector<uint32_t> all_cus(((uint32_t)n_cu + 31u) / 32u, 0xffffffffu);
    // CU-mask streams are blocking streams (no flags argument): they synchronise with the
    // legacy null stream like any default-flag stream (documented in vpx.h).
    for (auto& L : c->lanes) {
        L.dedicated = g_lane_queues.fetch_add(1) < kMaxLaneQueues;
        if (!L.dedicated) g_lane_queues.fetch_sub(1);
        const hipError_t se = L.dedicated
                                  ? hipExtStreamCreateWithCUMask(&L.s, (uint32_t)all_cus.size(), all_cus.data())
                                  : hipStreamCreateWithFlags(&L.s, hipStreamNonBlocking);
        if (se != hipSuccess ||
            hipEventCreateWithFlags(&L.rendered, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&L.consumed, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&L.consumed2, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&L.caller, hipEventDisableTiming) != hipSuccess) {
            free_lanes(c);
            return fail(c, VPX_E_DEVICE, "pipeline lane stream / events");
        }
    }
    return VPX_OK;
}

// ---------------------------------------------------------------- display interop
// GLTexture::CopyFrom (template/opengl.cpp:144-149) uploads the host screen every frame; here
// the RGB8 pack writes into a GL pixel-unpack buffer the host registered once, and the host
// updates its texture from that buffer (glTexSubImage2D with the PBO bound) — the frame stays
// on the GPU.  A device set registers and maps on devices[0], where vpx_render composites.
static vpx_ctx* gl_home(vpx_ctx* c) { return c->members.empty() ? c : c->members[0]; }

int vpx_gl_register_buffer(vpx_ctx* c, unsigned int gl_buffer) {
    if (!c) return VPX_E_INVALID;
    if (c->gl_mapped) return fail(c, VPX_E_STATE, "the GL buffer is mapped (vpx_gl_unmap first)");
    vpx_ctx* h = gl_home(c);
    VPX_HIP(c, hipSetDevice(h->device));
    if (c->gl_res) {
        const hipError_t e = hipGraphicsUnregisterResource(c->gl_res);
        c->gl_res = nullptr;
        if (e != hipSuccess) return fail(c, VPX_E_DEVICE, std::string("hipGraphicsUnregisterResource: ") + hipGetErrorString(e));
    }
    if (gl_buffer == 0u) return VPX_OK;
    hipGraphicsResource_t r = nullptr;
    const hipError_t e = hipGraphicsGLRegisterBuffer(&r, (GLuint)gl_buffer, hipGraphicsRegisterFlagsWriteDiscard);
    if (e != hipSuccess || !r)
        return fail(c, VPX_E_DEVICE, std::string("hipGraphicsGLRegisterBuffer (needs the buffer's GL context current on "
                                                 "this thread, on this context's GPU): ") + hipGetErrorString(e));
    c->gl_res = r;
    return VPX_OK;
}

int vpx_gl_map(vpx_ctx* c, uint32_t** rgb8, size_t* bytes) {
    if (!c || !rgb8) return VPX_E_INVALID;
    if (!c->gl_res) return fail(c, VPX_E_STATE, "no GL buffer registered (vpx_gl_register_buffer)");
    if (c->gl_mapped) return fail(c, VPX_E_STATE, "the GL buffer is already mapped");
    vpx_ctx* h = gl_home(c);
    VPX_HIP(c, hipSetDevice(h->device));
    VPX_HIP(c, hipGraphicsMapResources(1, &c->gl_res, h->stream));
    void* ptr = nullptr;
    size_t n = 0;
    const hipError_t e = hipGraphicsResourceGetMappedPointer(&ptr, &n, c->gl_res);
    if (e != hipSuccess) {
        (void)hipGraphicsUnmapResources(1, &c->gl_res, h->stream);
        return fail(c, VPX_E_DEVICE, std::string("hipGraphicsResourceGetMappedPointer: ") + hipGetErrorString(e));
    }
    c->gl_mapped = true;
    *rgb8 = static_cast<uint32_t*>(ptr);
    if (bytes) *bytes = n;
    return VPX_OK;
}

int vpx_gl_unmap(vpx_ctx* c) {
    if (!c) return VPX_E_INVALID;
    if (!c->gl_mapped) return fail(c, VPX_E_STATE, "the GL buffer is not mapped");
    vpx_ctx* h = gl_home(c);
    VPX_HIP(c, hipSetDevice(h->device));
    c->gl_mapped = false;
    VPX_HIP(c, hipGraphicsUnmapResources(1, &c->gl_res, h->stream));
    return VPX_OK;
}

int vpx_synchronize(vpx_ctx* c) {
    VPX_GROUP_ALL(c, vpx_synchronize(m_));
    if (!c) return VPX_E_INVALID;
    VPX_HIP(c, sync_all(c));
    return VPX_OK;
}

static int alloc_grid(vpx_ctx* c, uint32_t id, uint32_t n) {
    if (id > 4096) return fail(c, VPX_E_INVALID, "grid_id too large");
    if (n == 0 || n > 4096) return fail(c, VPX_E_INVALID, "grid size must be in [1, 4096]");
    VPX_HIP(c, hipSetDevice(c->device));
    if (id >= c->grids.size()) c->grids.resize(id + 1);
    auto& g = c->grids[id];
    const size_t bytes = (size_t)n * n * n;
    if (g.ptr && g.n != n) {
        VPX_HIP(c, sync_all(c));
        (void)hipFree(g.ptr);
        (void)hipFree(g.l1);
        (void)hipFree(g.l2);
        (void)hipFree(g.dfp);
        g.ptr = nullptr, g.l1 = nullptr, g.l2 = nullptr, g.dfp = nullptr;
    }
    g.n = n;
    g.nb1 = (n + 3) / 4;
    g.nb2 = (g.nb1 + 3) / 4;
    g.nb3 = (g.nb2 + 3) / 4;
    if (!g.ptr) {
        VPX_HIP(c, hipMalloc(&g.ptr, bytes));
        VPX_HIP(c, hipMalloc(&g.l1, sizeof(uint64_t) * (size_t)g.nb2 * g.nb2 * g.nb2 * 64));
        VPX_HIP(c, hipMalloc(&g.l2, sizeof(uint64_t) * (size_t)g.nb3 * g.nb3 * g.nb3 * 64));
        VPX_HIP(c, hipMalloc(&g.dfp, 8 * g.plane()));
    }
    return sync_grids(c);
}

// The distance-field words of every empty brick (recurrence: skip::df_value), one
// anti-diagonal plane per launch from the far corner — all 8 octants at once, each in its
// own flipped coordinates and its own byte of the word.  Needs l2 (occupancy) current.
static int build_df(vpx_ctx* c, const vpx_ctx::GridBuf& g) {
    const uint64_t threads = (uint64_t)g.nb1 * g.nb1 * 8;
    const unsigned blocks = (unsigned)((threads + 255) / 256);
    for (uint32_t s = 3 * (g.nb1 - 1) + 1; s-- > 0;) {
        hipLaunchKernelGGL(df_plane_k, dim3(blocks), dim3(256), 0, c->stream, (uint8_t*)g.l1, g.l2, g.nb1, g.nb2, g.nb3, s);
        VPX_HIP(c, hipGetLastError());
    }
    hipLaunchKernelGGL(build_planes_k, dim3(2048), dim3(256), 0, c->stream, g.l1, g.l2, g.nb2, g.nb3, g.dfp);
    VPX_HIP(c, hipGetLastError());
    return VPX_OK;
}

// Rebuild the occupancy levels and the distance field after the grid bytes changed.
static int build_masks(vpx_ctx* c, uint32_t id) {
    auto& g = c->grids[id];
    hipLaunchKernelGGL(build_l1_k, dim3(2048), dim3(256), 0, c->stream, g.ptr, g.n, g.nb1, g.nb2, g.l1);
    VPX_HIP(c, hipGetLastError());
    hipLaunchKernelGGL(build_up_k, dim3(512), dim3(256), 0, c->stream, g.l1, g.nb2, g.nb3, g.l2);
    VPX_HIP(c, hipGetLastError());
    if (int r = build_df(c, g)) return r;
    VPX_HIP(c, sync_all(c));
    return VPX_OK;
}

// Refresh the occupancy levels for the macros that hold the cells [x0, x1) x [y0, y1) x
// [z0, z1) (their bricks' words are recomputed whole, so the l2 words see fresh masks
// only), then the distance field (an edit can change it far behind the box).
static int build_masks_box(vpx_ctx* c, uint32_t id, uint32_t x0, uint32_t y0, uint32_t z0, uint32_t x1, uint32_t y1,
                           uint32_t z1) {
    auto& g = c->grids[id];
    if (x0 >= x1 || y0 >= y1 || z0 >= z1) return VPX_OK;
    uint32_t lo[3] = {(x0 >> 4) * 4, (y0 >> 4) * 4, (z0 >> 4) * 4};
    uint32_t hi[3] = {((x1 - 1) >> 4) * 4 + 3, ((y1 - 1) >> 4) * 4 + 3, ((z1 - 1) >> 4) * 4 + 3};
    for (int k = 0; k < 3; ++k) hi[k] = hi[k] < g.nb1 - 1 ? hi[k] : g.nb1 - 1;
    auto blocks = [](uint64_t a, uint64_t b, uint64_t cc) { return (unsigned)std::min<uint64_t>(4096, (a * b * cc + 255) / 256); };
    hipLaunchKernelGGL(build_l1_box_k, dim3(blocks(hi[0] - lo[0] + 1, hi[1] - lo[1] + 1, hi[2] - lo[2] + 1)), dim3(256), 0,
                       c->stream, g.ptr, g.n, g.nb2, g.l1, lo[0], lo[1], lo[2], hi[0] - lo[0] + 1, hi[1] - lo[1] + 1,
                       hi[2] - lo[2] + 1);
    VPX_HIP(c, hipGetLastError());
    for (int k = 0; k < 3; ++k) lo[k] >>= 2, hi[k] >>= 2;  // macros
    hipLaunchKernelGGL(build_up_box_k, dim3(blocks(hi[0] - lo[0] + 1, hi[1] - lo[1] + 1, hi[2] - lo[2] + 1)), dim3(256), 0,
                       c->stream, g.l1, g.nb2, g.nb3, g.l2, lo[0], lo[1], lo[2], hi[0] - lo[0] + 1, hi[1] - lo[1] + 1,
                       hi[2] - lo[2] + 1);
    VPX_HIP(c, hipGetLastError());
    if (int r = build_df(c, g)) return r;
    VPX_HIP(c, sync_all(c));
    return VPX_OK;
}

int vpx_grid_fill(vpx_ctx* c, uint32_t id, uint8_t value) {
    VPX_GROUP_ALL(c, vpx_grid_fill(m_, id, value));
    if (!c) return VPX_E_INVALID;
    if (id >= c->grids.size() || !c->grids[id].ptr) return fail(c, VPX_E_INVALID, "unknown grid");
    auto& g = c->grids[id];
    VPX_HIP(c, sync_all(c));  // frames in flight still read the grid
    VPX_HIP(c, hipMemsetAsync(g.ptr, value, (size_t)g.n * g.n * g.n, c->stream));
    return build_masks(c, id);
}

int vpx_grid_write_box(vpx_ctx* c, uint32_t id, const uint8_t* src, uint32_t x0, uint32_t y0, uint32_t z0,
                       uint32_t dx, uint32_t dy, uint32_t dz) {
    VPX_GROUP_ALL(c, vpx_grid_write_box(m_, id, src, x0, y0, z0, dx, dy, dz));
    if (!c || !src) return fail(c, VPX_E_INVALID, "null argument");
    if (id >= c->grids.size() || !c->grids[id].ptr) return fail(c, VPX_E_INVALID, "unknown grid");
    auto& g = c->grids[id];
    if ((uint64_t)x0 + dx > g.n || (uint64_t)y0 + dy > g.n || (uint64_t)z0 + dz > g.n)
        return fail(c, VPX_E_INVALID, "box outside the grid");
    const size_t bytes = (size_t)dx * dy * dz;
    if (!bytes) return VPX_OK;
    uint8_t* d = nullptr;
    VPX_HIP(c, sync_all(c));  // frames in flight still read the grid
    VPX_HIP(c, hipMalloc(&d, bytes));
    if (hipMemcpyAsync(d, src, bytes, hipMemcpyHostToDevice, c->stream) != hipSuccess) {
        (void)hipFree(d);
        return fail(c, VPX_E_DEVICE, "box upload failed");
    }
    hipLaunchKernelGGL(write_box_k, dim3((unsigned)std::min<size_t>(4096, (bytes + 255) / 256)), dim3(256), 0, c->stream,
                       g.ptr, g.n, d, x0, y0, z0, dx, dy, dz);
    const hipError_t e = sync_all(c);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(c, VPX_E_DEVICE, hipGetErrorString(e));
    return build_masks_box(c, id, x0, y0, z0, x0 + dx, y0 + dy, z0 + dz);
}

int vpx_grid_emissive_sphere(vpx_ctx* c, uint32_t id, uint8_t mat, float radius) {
    VPX_GROUP_ALL(c, vpx_grid_emissive_sphere(m_, id, mat, radius));
    if (!c) return VPX_E_INVALID;
    if (id >= c->grids.size() || !c->grids[id].ptr) return fail(c, VPX_E_INVALID, "unknown grid");
    auto& g = c->grids[id];
    if (!(radius > 0.0f)) return VPX_OK;  // no cell has length < radius <= 0 (NaN: none either)
    // cells with |c - x| < radius per axis, c = n/2: a conservative integer box
    const double cc = g.n / 2.0, r = std::min<double>(radius, 4.0 * g.n);
    const int64_t a = std::max<int64_t>(0, (int64_t)std::floor(cc - r) - 1);
    const int64_t b = std::min<int64_t>((int64_t)g.n - 1, (int64_t)std::ceil(cc + r) + 1);
    if (b < a) return VPX_OK;
    const uint32_t x0 = (uint32_t)a, cnt = (uint32_t)(b - a + 1);
    VPX_HIP(c, sync_all(c));  // frames in flight still read the grid
    hipLaunchKernelGGL(emissive_sphere_k, dim3((unsigned)std::min<uint64_t>(4096, ((uint64_t)cnt * cnt * cnt + 255) / 256)),
                       dim3(256), 0, c->stream, g.ptr, g.n, mat, radius, x0, cnt);
    VPX_HIP(c, hipGetLastError());
    return build_masks_box(c, id, x0, x0, x0, x0 + cnt, x0 + cnt, x0 + cnt);
}

int vpx_upload_grid(vpx_ctx* c, uint32_t id, const uint8_t* cells, uint32_t n) {
    VPX_GROUP_ALL(c, vpx_upload_grid(m_, id, cells, n));
    if (!c || !cells) return fail(c, VPX_E_INVALID, "null argument");
    VPX_HIP(c, sync_all(c));  // frames in flight still read the grid
    int rc = alloc_grid(c, id, n);
    if (rc) return rc;
    VPX_HIP(c, hipMemcpy(c->grids[id].ptr, cells, (size_t)n * n * n, hipMemcpyHostToDevice));
    return build_masks(c, id);
}

int vpx_generate_tiled_grid(vpx_ctx* c, uint32_t id, uint32_t n, const uint8_t* model, uint32_t mx, uint32_t my,
                            uint32_t mz, uint32_t px, uint32_t py, uint32_t pz, uint32_t ground) {
    VPX_GROUP_ALL(c, vpx_generate_tiled_grid(m_, id, n, model, mx, my, mz, px, py, pz, ground));
    if (!c || !model) return fail(c, VPX_E_INVALID, "null argument");
    if (!mx || !my || !mz || !px || !py || !pz) return fail(c, VPX_E_INVALID, "zero model size or period");
    VPX_HIP(c, sync_all(c));  // frames in flight still read the grid
    int rc = alloc_grid(c, id, n);
    if (rc) return rc;
    const size_t mbytes = (size_t)mx * my * mz;
    uint8_t* dm = nullptr;
    VPX_HIP(c, hipMalloc(&dm, mbytes));
    VPX_HIP(c, hipMemcpy(dm, model, mbytes, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(tiled_world_k, dim3(4096), dim3(256), 0, c->stream, c->grids[id].ptr, n, dm, mx, my, mz, px,
                       py, pz, ground);
    VPX_HIP(c, hipGetLastError());
    VPX_HIP(c, sync_all(c));
    (void)hipFree(dm);
    return build_masks(c, id);
}

int vpx_grid_checksum(vpx_ctx* c, uint32_t id, uint64_t* out) {
    VPX_GROUP_FIRST(c, vpx_grid_checksum(m_, id, out));
    if (!c || !out) return fail(c, VPX_E_INVALID, "null argument");
    if (id >= c->grids.size() || !c->grids[id].ptr) return fail(c, VPX_E_INVALID, "unknown grid");
    const uint64_t count = (uint64_t)c->grids[id].n * c->grids[id].n * c->grids[id].n;
    VPX_HIP(c, hipMemsetAsync(c->d_sum, 0, sizeof(unsigned long long), c->stream));
    hipLaunchKernelGGL(checksum_k, dim3(2048), dim3(256), 0, c->stream, c->grids[id].ptr, count, c->d_sum);
    VPX_HIP(c, hipGetLastError());
    unsigned long long h = 0;
    VPX_HIP(c, hipMemcpyAsync(&h, c->d_sum, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    VPX_HIP(c, sync_all(c));
    *out = (uint64_t)h;
    return VPX_OK;
}

// The world box a volume's walks are culled with (misses_volume, the TLAS): the cube b0..b1
// through the inverse of inv_matrix's affine part (rows 0-2: every transform of the path —
// xform_pos_ssem / xform_pos, TransformPosition(_SSEM), tmpl8math.cpp:345-402 — reads only
// those; SetTransform's inverse leaves m[15] = 1 +- 1 ulp on a third of C4's instances), its 8
// corners in double, padded by 0.1 % of the half-diagonal + 1e-3 of the scale and rounded
// outward to float, so that the reference's float cube test (Setup3DDDA) can only succeed, and
// its walk only read a cell, for rays whose segment meets the box.  A singular 3x3 part gives
// an infinite box (never culled).  [0] = lo, [1] = hi (w = 0).
struct VolBox {
    float4 lo, hi;
};
static VolBox volume_bounds(const vpx_volume& v) {
    const float* m = v.inv_matrix;
    const double a[3][3] = {{m[0], m[1], m[2]}, {m[4], m[5], m[6]}, {m[8], m[9], m[10]}};
    const double det = a[0][0] * (a[1][1] * a[2][2] - a[1][2] * a[2][1]) -
                       a[0][1] * (a[1][0] * a[2][2] - a[1][2] * a[2][0]) +
                       a[0][2] * (a[1][0] * a[2][1] - a[1][1] * a[2][0]);
    const VolBox none{make_float4(-INFINITY, -INFINITY, -INFINITY, 0.f), make_float4(INFINITY, INFINITY, INFINITY, 0.f)};
    if (!(std::fabs(det) > 1e-30)) return none;
    double r[3][3];  // inverse of the 3x3 part
    r[0][0] = (a[1][1] * a[2][2] - a[1][2] * a[2][1]) / det;
    r[0][1] = (a[0][2] * a[2][1] - a[0][1] * a[2][2]) / det;
    r[0][2] = (a[0][1] * a[1][2] - a[0][2] * a[1][1]) / det;
    r[1][0] = (a[1][2] * a[2][0] - a[1][0] * a[2][2]) / det;
    r[1][1] = (a[0][0] * a[2][2] - a[0][2] * a[2][0]) / det;
    r[1][2] = (a[0][2] * a[1][0] - a[0][0] * a[1][2]) / det;
    r[2][0] = (a[1][0] * a[2][1] - a[1][1] * a[2][0]) / det;
    r[2][1] = (a[0][1] * a[2][0] - a[0][0] * a[2][1]) / det;
    r[2][2] = (a[0][0] * a[1][1] - a[0][1] * a[1][0]) / det;
    const double t[3] = {m[3], m[7], m[11]};
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int k = 0; k < 8; ++k) {
        const double q[3] = {(k & 1) ? v.b1[0] : v.b0[0], (k & 2) ? v.b1[1] : v.b0[1], (k & 4) ? v.b1[2] : v.b0[2]};
        for (int i = 0; i < 3; ++i) {
            const double p = r[i][0] * (q[0] - t[0]) + r[i][1] * (q[1] - t[1]) + r[i][2] * (q[2] - t[2]);
            lo[i] = std::min(lo[i], p), hi[i] = std::max(hi[i], p);
        }
    }
    double half = 0.0, cen = 0.0;
    for (int i = 0; i < 3; ++i) {
        half += (hi[i] - lo[i]) * (hi[i] - lo[i]) / 4.0;
        cen += std::fabs((lo[i] + hi[i]) / 2.0);
    }
    half = std::sqrt(half);
    const double pad = half * 1e-3 + 1e-3 * (1.0 + cen + half);
    VolBox b;
    float* out[2] = {&b.lo.x, &b.hi.x};
    for (int i = 0; i < 3; ++i) {
        if (!std::isfinite(lo[i] - pad) || !std::isfinite(hi[i] + pad)) return none;
        out[0][i] = std::nextafter((float)(lo[i] - pad), -INFINITY);
        out[1][i] = std::nextafter((float)(hi[i] + pad), INFINITY);
    }
    b.lo.w = b.hi.w = 0.f;
    return b;
}

// Instance TLAS (the C4 lattice of 64 instances over the world volume): a BVH over the
// inflated world boxes (volume_bounds) of volumes 1..n-1, built once per
// vpx_set_volumes (volume 0, first in the reference's loop, is walked before the tree is
// asked, so the instances' candidates are bounded by its hit).
// Boxes are the volumes' boxes widened by a further 1e-4 of the scale and rounded outward to
// float, so every volume misses_volume keeps is a candidate.  Median split on the
// longest centroid axis (ties by index), leaves of <= 4 volumes (their bit mask), nodes in
// depth-first order with skip links (TlasNode).  Volumes without finite bounds go to the
// always-set.
#ifndef VPX_TLAS_LEAF
#define VPX_TLAS_LEAF 4  // volumes per TLAS leaf
#endif
struct TlasBuild {
    std::vector<TlasNode> nodes;
    struct Item {
        double lo[3], hi[3], c[3];
        uint32_t id;
    };
    std::vector<Item> items;
    void build(uint32_t first, uint32_t count) {
        const uint32_t me = (uint32_t)nodes.size();
        nodes.push_back(TlasNode{});
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (uint32_t i = first; i < first + count; ++i)
            for (int k = 0; k < 3; ++k) {
                lo[k] = std::min(lo[k], items[i].lo[k]), hi[k] = std::max(hi[k], items[i].hi[k]);
                clo[k] = std::min(clo[k], items[i].c[k]), chi[k] = std::max(chi[k], items[i].c[k]);
            }
        TlasNode nd{};
        for (int k = 0; k < 3; ++k) {
            nd.lo[k] = std::nextafter((float)lo[k], -INFINITY);
            nd.hi[k] = std::nextafter((float)hi[k], INFINITY);
        }
        if (count <= (uint32_t)VPX_TLAS_LEAF) {
            nd.leaf = 1;
            for (uint32_t i = first; i < first + count; ++i) nd.mask |= 1ull << (items[i].id - 1u);
            nodes[me] = nd;
            return;
        }
        int axis = 0;
        for (int k = 1; k < 3; ++k)
            if (chi[k] - clo[k] > chi[axis] - clo[axis]) axis = k;
        std::stable_sort(items.begin() + first, items.begin() + first + count,
                         [axis](const Item& x, const Item& y) { return x.c[axis] < y.c[axis]; });
        const uint32_t half = count / 2;
        build(first, half);
        build(first + half, count - half);
        nd.skip = (uint32_t)nodes.size();  // the node after this subtree
        nodes[me] = nd;
    }
};

int build_tlas(vpx_ctx* c, const std::vector<VolBox>& bounds) {
    c->tlas_on = false;
    c->tlas_nodes = 0;
    c->tlas_always = 0;
    const uint32_t count = (uint32_t)bounds.size();
    if (count < 2 || count > kTlasMaxVolumes) return VPX_OK;  // one volume / too many: the linear loop
    TlasBuild b;
    for (uint32_t i = 1; i < count; ++i) {  // volume 0 is walked first, outside the tree
        const VolBox& vb = bounds[i];
        const double lo[3] = {vb.lo.x, vb.lo.y, vb.lo.z}, hi[3] = {vb.hi.x, vb.hi.y, vb.hi.z};
        if (!std::isfinite(lo[0] + lo[1] + lo[2] + hi[0] + hi[1] + hi[2])) {
            c->tlas_always |= 1ull << (i - 1u);
            continue;
        }
        double half = 0.0, cen = 0.0;
        for (int k = 0; k < 3; ++k) half += (hi[k] - lo[k]) * (hi[k] - lo[k]) / 4.0, cen += std::fabs((lo[k] + hi[k]) / 2.0);
        half = std::sqrt(half);
        const double pad = half * 1e-4 + 1e-4 * (1.0 + cen + half);
        TlasBuild::Item it{};
        for (int k = 0; k < 3; ++k) it.lo[k] = lo[k] - pad, it.hi[k] = hi[k] + pad, it.c[k] = (lo[k] + hi[k]) / 2.0;
        it.id = i;
        b.items.push_back(it);
    }
    if (!b.items.empty()) b.build(0, (uint32_t)b.items.size());
    if (b.nodes.size() > kTlasMaxNodes) return fail(c, VPX_E_INVALID, "TLAS node budget exceeded");
    if (!c->d_tlas) VPX_HIP(c, hipMalloc(&c->d_tlas, sizeof(TlasNode) * kTlasMaxNodes));
    if (!b.nodes.empty())
        VPX_HIP(c, hipMemcpy(c->d_tlas, b.nodes.data(), sizeof(TlasNode) * b.nodes.size(), hipMemcpyHostToDevice));
    c->tlas_nodes = (uint32_t)b.nodes.size();
    c->tlas_on = true;
    return VPX_OK;
}

int vpx_set_volumes(vpx_ctx* c, const vpx_volume* v, uint32_t count) {
    VPX_GROUP_ALL(c, vpx_set_volumes(m_, v, count));
    if (!c || (!v && count)) return fail(c, VPX_E_INVALID, "null argument");
    if (count > 65536) return fail(c, VPX_E_INVALID, "too many volumes");
    VPX_HIP(c, sync_all(c));
    if (count > c->d_volumes_cap) {
        if (c->d_volumes) (void)hipFree(c->d_volumes);
        if (c->d_vbounds) (void)hipFree(c->d_vbounds);
        c->d_volumes = nullptr;
        c->d_vbounds = nullptr;
        VPX_HIP(c, hipMalloc(&c->d_volumes, sizeof(vpx_volume) * count));
        VPX_HIP(c, hipMalloc(&c->d_vbounds, sizeof(VolBox) * count));
        c->d_volumes_cap = count;
    }
    // Invariant: d_volumes, d_vbounds and the TLAS (d_tlas) describe the same volumes.  The
    // instance kernels cull by the TLAS root box and the bounding spheres (FindNearest's
    // candidates, the shadow pool's slot list), so a volume update that skipped build_tlas would
    // silently drop instance hits and shadows: every writer of d_volumes goes through here.
    c->volumes.assign(v, v + count);
    std::vector<VolBox> bounds(count);
    for (uint32_t i = 0; i < count; ++i) bounds[i] = volume_bounds(v[i]);
    if (count) {
        VPX_HIP(c, hipMemcpy(c->d_volumes, v, sizeof(vpx_volume) * count, hipMemcpyHostToDevice));
        VPX_HIP(c, hipMemcpy(c->d_vbounds, bounds.data(), sizeof(VolBox) * count, hipMemcpyHostToDevice));
    }
    return build_tlas(c, bounds);
}

int vpx_volume_bounds(const vpx_volume* v, float out[6]) {
    if (!v || !out) return VPX_E_INVALID;
    const VolBox b = volume_bounds(*v);
    out[0] = b.lo.x, out[1] = b.lo.y, out[2] = b.lo.z, out[3] = b.hi.x, out[4] = b.hi.y, out[5] = b.hi.z;
    return VPX_OK;
}

int vpx_set_materials(vpx_ctx* c, const vpx_material* m, uint32_t count) {
    VPX_GROUP_ALL(c, vpx_set_materials(m_, m, count));
    if (!c || !m) return fail(c, VPX_E_INVALID, "null argument");
    if (count == 0 || count > VPX_NUM_MATERIALS) return fail(c, VPX_E_INVALID, "material count must be 1..256");
    vpx_material full[VPX_NUM_MATERIALS];
    // entries past `count` behave like MaterialSetUp's padding: white, roughness 1
    for (auto& e : full) e = vpx_material{{1, 1, 1}, 1.0f, 0.0f, 1.5f, {0, 0}};
    std::memcpy(full, m, sizeof(vpx_material) * count);
    VPX_HIP(c, sync_all(c));
    int rc = upload_table(c, c->d_materials, full, VPX_NUM_MATERIALS);
    if (rc) return rc;
    VPX_HIP(c, sync_all(c));
    c->have_materials = true;
    return VPX_OK;
}

int vpx_set_lights(vpx_ctx* c, const vpx_point_light* p, uint32_t np, const vpx_spot_light* s, uint32_t ns,
                   const vpx_area_light* a, uint32_t na, const vpx_dir_light* d) {
    VPX_GROUP_ALL(c, vpx_set_lights(m_, p, np, s, ns, a, na, d));
    if (!c) return VPX_E_INVALID;
    VPX_HIP(c, sync_all(c));
    int rc;
    if ((rc = upload_table(c, c->d_points, p, np))) return rc;
    if ((rc = upload_table(c, c->d_spots, s, ns))) return rc;
    if ((rc = upload_table(c, c->d_areas, a, na))) return rc;
    VPX_HIP(c, sync_all(c));
    c->n_points = np, c->n_spots = ns, c->n_areas = na;
    if (d) c->dir = *d;
    return VPX_OK;
}

int vpx_set_shapes(vpx_ctx* c, const vpx_sphere* s, uint32_t ns, const vpx_triangle* t, uint32_t nt) {
    VPX_GROUP_ALL(c, vpx_set_shapes(m_, s, ns, t, nt));
    if (!c) return VPX_E_INVALID;
    VPX_HIP(c, sync_all(c));
    int rc;
    if ((rc = upload_table(c, c->d_spheres, s, ns))) return rc;
    if ((rc = upload_table(c, c->d_triangles, t, nt))) return rc;
    VPX_HIP(c, sync_all(c));
    c->n_spheres = ns, c->n_triangles = nt;
    return VPX_OK;
}

int vpx_set_sky(vpx_ctx* c, const float* rgb, uint32_t width, uint32_t height, float hdr_contribution) {
    VPX_GROUP_ALL(c, vpx_set_sky(m_, rgb, width, height, hdr_contribution));
    if (!c) return VPX_E_INVALID;
    VPX_HIP(c, hipSetDevice(c->device));
    if (!rgb || !width || !height) {  // remove the texture (misses use the constant sky)
        if (c->d_sky) {
            VPX_HIP(c, sync_all(c));
            (void)hipFree(c->d_sky);
        }
        c->d_sky = nullptr;
        c->sky_w = c->sky_h = 0;
        return VPX_OK;
    }
    if ((uint64_t)width * height > (1ull << 28)) return fail(c, VPX_E_INVALID, "sky texture too large");
    const size_t bytes = sizeof(float) * 3 * (size_t)width * height;
    if ((size_t)c->sky_w * c->sky_h != (size_t)width * height) {
        VPX_HIP(c, sync_all(c));
        if (c->d_sky) (void)hipFree(c->d_sky);
        c->d_sky = nullptr;
        c->sky_w = c->sky_h = 0;
        VPX_HIP(c, hipMalloc(&c->d_sky, bytes));
    }
    VPX_HIP(c, sync_all(c));  // frames in flight still read the texture
    VPX_HIP(c, hipMemcpyAsync(c->d_sky, rgb, bytes, hipMemcpyHostToDevice, c->stream));
    VPX_HIP(c, sync_all(c));
    c->sky_w = width, c->sky_h = height;
    c->sky_hdr = hdr_contribution;
    return VPX_OK;
}

int vpx_set_arithmetic(vpx_ctx* c, uint32_t mode) {
    VPX_GROUP_ALL(c, vpx_set_arithmetic(m_, mode));
    if (!c) return VPX_E_INVALID;
    if (mode != VPX_ARITH_EXACT && mode != VPX_ARITH_X86_HOST) return fail(c, VPX_E_INVALID, "unknown arithmetic mode");
    VPX_HIP(c, hipSetDevice(c->device));
    VPX_HIP(c, sync_all(c));  // frames in flight read the tables
    if (c->d_x86) (void)hipFree(c->d_x86);
    c->d_x86 = nullptr;
    c->x86 = X86Arith{nullptr, 0u, 0u, 0u, 0u};
    if (mode == VPX_ARITH_EXACT) return VPX_OK;
    uint32_t info[4];
    if (vpx_x86_arith_tables(nullptr, 0, info) != VPX_OK)
        return fail(c, VPX_E_STATE, "the host's rcpss / rsqrtss do not follow the table model (or the host is not x86)");
    if (23u - info[0] > kX86LdsBits)  // the multi-volume walkers stage the rcp table in LDS
        return fail(c, VPX_E_STATE, "the host's rcpss key is wider than the LDS-staged table allows");
    std::vector<uint32_t> tab(info[3]);
    if (vpx_x86_arith_tables(tab.data(), tab.size(), info) != VPX_OK) return fail(c, VPX_E_STATE, "table capture failed");
    VPX_HIP(c, hipMalloc(&c->d_x86, sizeof(uint32_t) * tab.size()));
    VPX_HIP(c, hipMemcpy(c->d_x86, tab.data(), sizeof(uint32_t) * tab.size(), hipMemcpyHostToDevice));
    c->x86 = X86Arith{c->d_x86, info[0], info[1], info[2], 0u};
    return VPX_OK;
}

int vpx_set_camera(vpx_ctx* c, const vpx_camera* cam) {
    VPX_GROUP_ALL(c, vpx_set_camera(m_, cam));
    if (!c || !cam) return fail(c, VPX_E_INVALID, "null argument");
    c->cam = *cam;
    c->have_camera = true;
    return VPX_OK;
}

static int group_render(vpx_ctx* c, const vpx_frame_params* p, float* accum, uint32_t* rgb8, vpx_stats* stats);

int vpx_render(vpx_ctx* c, const vpx_frame_params* p, float* accum, uint32_t* rgb8, vpx_stats* stats) {
    if (!c) return VPX_E_INVALID;
    if (!c->members.empty()) return group_render(c, p, accum, rgb8, stats);
    int rc = validate_frame(c, p);
    if (rc) return rc;
    if (!accum) return fail(c, VPX_E_INVALID, "accum (device float4[W*H]) is required");
    VPX_HIP(c, hipSetDevice(c->device));
    const SceneView sv = view_of(c, p->sky, p->area_samples, (p->flags & VPX_FLAG_SKY) != 0);
    const FrameArgs f = frame_of(c, p, 0, 1);
    if (!c->lanes.empty() && !stats && !(p->flags & VPX_FLAG_NO_TONEMAP) && lane_tail_ok(sv, f)) {
        // frames in flight whose tail is a launch of its own (k_resolve_finish after the shadow
        // pool): the whole frame runs on its lane, the tail blending straight into the caller's
        // accumulator once the caller's stream has reached this call (which orders it after
        // the previous frame's tail): no packed sample, no composite (32 B per pixel less)
        vpx_ctx::Lane& L = c->lanes[c->lane_next];
        c->lane_next = (c->lane_next + 1u) % (uint32_t)c->lanes.size();
        if (L.used) VPX_HIP(c, hipStreamWaitEvent(L.s, L.consumed, 0));
        VPX_HIP(c, hipEventRecord(L.caller, c->stream));
        if ((rc = launch_render<kFinishImage>(c, L.s, L.ws, sv, f, f.num_tiles, reinterpret_cast<float4*>(accum), rgb8,
                                              nullptr, nullptr, &L.caller)))
            return rc;
        VPX_HIP(c, hipEventRecord(L.rendered, L.s));
        VPX_HIP(c, hipStreamWaitEvent(c->stream, L.rendered, 0));
        VPX_HIP(c, hipEventRecord(L.consumed, L.s));
        L.used = true;
        return VPX_OK;
    }
    if (!c->lanes.empty() && !stats && !(p->flags & VPX_FLAG_NO_TONEMAP)) {
        // frames in flight: the frame renders on a lane; its accumulate / tonemap runs on the
        // caller's stream after the previous frame's (the same blend of the same sample)
        vpx_ctx::Lane* L = nullptr;
        if ((rc = lane_render(c, sv, f, f.num_tiles, nullptr, L))) return rc;
        hipLaunchKernelGGL(composite_tiles, dim3(f.num_tiles), dim3(kThreads), 0, c->stream, f, L->cur,
                           reinterpret_cast<float4*>(accum), rgb8);
        VPX_HIP(c, hipGetLastError());
        VPX_HIP(c, hipEventRecord(L->cur_consumed, c->stream));
        return VPX_OK;
    }
    unsigned long long before[kCtrWords] = {};
    if (stats && (rc = snapshot_counters(c, before))) return rc;
    if (stats) VPX_HIP(c, hipEventRecord(c->ev0, c->stream));
    if ((rc = launch_render<kFinishImage>(c, c->stream, c->wave, sv, f, f.num_tiles, reinterpret_cast<float4*>(accum), rgb8,
                                          nullptr)))
        return rc;
    if (stats) {
        VPX_HIP(c, hipEventRecord(c->ev1, c->stream));
        unsigned long long after[kCtrWords];
        if ((rc = snapshot_counters(c, after))) return rc;
        std::memset(stats, 0, sizeof(*stats));
        fill_stats(stats, before, after);
        float ms = 0.f;
        VPX_HIP(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
        stats->kernel_ms = ms;
        stats->total_ms = ms;
    }
    return VPX_OK;
}

int vpx_render_reproject(vpx_ctx* c, const vpx_frame_params* p, const vpx_prev_camera* prev, float* history,
                         uint32_t* rgb8, vpx_stats* stats) {
    VPX_GROUP_FIRST(c, vpx_render_reproject(m_, p, prev, history, rgb8, stats));
    if (!c) return VPX_E_INVALID;
    int rc = validate_frame(c, p);
    if (rc) return rc;
    if (!prev || !history) return fail(c, VPX_E_INVALID, "prev camera and history (device float4[W*H]) are required");
    VPX_HIP(c, hipSetDevice(c->device));
    const size_t pix = (size_t)p->width * p->height;
    if (pix > c->rp_pixels) {
        VPX_HIP(c, sync_all(c));
        if (c->rp_buf) (void)hipFree(c->rp_buf);
        c->rp_buf = nullptr;
        c->rp_pixels = 0;
        VPX_HIP(c, hipMalloc(&c->rp_buf, sizeof(float4) * 4 * pix));
        c->rp_pixels = pix;
    }
    Reproj rp;
    auto h3 = [](const float* v) { return f3{v[0], v[1], v[2]}; };
    rp.prev = PrevCam{h3(prev->cam_pos), h3(prev->left_normal), h3(prev->right_normal), h3(prev->top_normal),
                      h3(prev->bottom_normal)};
    rp.alb = c->rp_buf, rp.ill = c->rp_buf + pix, rp.rd = c->rp_buf + 2 * pix, rp.temp = c->rp_buf + 3 * pix;
    rp.hist = reinterpret_cast<float4*>(history);
    unsigned long long before[kCtrWords] = {};
    if (stats && (rc = snapshot_counters(c, before))) return rc;
    const SceneView sv = view_of(c, p->sky, p->area_samples, (p->flags & VPX_FLAG_SKY) != 0);
    FrameArgs f = frame_of(c, p, 0, 1);
    f.flags = (f.flags & ~(VPX_FLAG_AA | VPX_FLAG_DOF)) | kFlagReproject;  // GetPrimaryRayNoDOF
    if (stats) VPX_HIP(c, hipEventRecord(c->ev0, c->stream));
    if ((rc = launch_render<kFinishImage>(c, c->stream, c->wave, sv, f, f.num_tiles, nullptr, rgb8, nullptr, &rp))) return rc;
    if (stats) {
        VPX_HIP(c, hipEventRecord(c->ev1, c->stream));
        unsigned long long after[kCtrWords];
        if ((rc = snapshot_counters(c, after))) return rc;
        std::memset(stats, 0, sizeof(*stats));
        fill_stats(stats, before, after);
        float ms = 0.f;
        VPX_HIP(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
        stats->kernel_ms = ms;
        stats->total_ms = ms;
    }
    return VPX_OK;
}

uint64_t vpx_tiles_packed_len(uint32_t width, uint32_t height, uint32_t tile_w, uint32_t tile_h, uint32_t n_ranks) {
    if (!width || !height || !n_ranks || tile_w != kTile || tile_h != kTile) return 0;
    const uint64_t tiles = (uint64_t)((width + kTile - 1) / kTile) * ((height + kTile - 1) / kTile);
    return ((tiles + n_ranks - 1) / n_ranks) * (uint64_t)(kTile * kTile);
}

// Shared body of vpx_render_tiles (packed samples) and vpx_render_tiles_accum (this rank's
// packed accumulator + RGB8); MODE is a FinishMode.
static int render_tiles_impl(int MODE, vpx_ctx* c, const vpx_frame_params* p, uint32_t tile_w, uint32_t tile_h,
                             uint32_t rank, uint32_t n_ranks, float4* accum, uint32_t* rgb8, float4* packed,
                             vpx_stats* stats) {
    if (!c) return VPX_E_INVALID;
    int rc = validate_frame(c, p);
    if (rc) return rc;
    if (tile_w != kTile || tile_h != kTile) return fail(c, VPX_E_INVALID, "tiles must be 16x16");
    if (n_ranks == 0 || rank >= n_ranks) return fail(c, VPX_E_INVALID, "bad rank");
    if (MODE == kFinishPackedSample ? !packed : (!accum || !rgb8))
        return fail(c, VPX_E_INVALID, "null packed buffer");
    VPX_HIP(c, hipSetDevice(c->device));
    const SceneView sv = view_of(c, p->sky, p->area_samples, (p->flags & VPX_FLAG_SKY) != 0);
    const FrameArgs f = frame_of(c, p, rank, n_ranks);
    // frames in flight (vpx_set_pipeline) for the sharded accumulator: the frame renders into
    // the lane's own samples and only the blend runs on the caller's stream.  Packed samples
    // into the caller's buffer stay serial: a lane would not wait for the caller's use of the
    // previous frame's samples (e.g. a gather queued on its stream).
    if (MODE == kFinishPackedAccum && !c->lanes.empty() && !stats) {
        vpx_ctx::Lane* L = nullptr;
        if ((rc = lane_render(c, sv, f, f.tiles_per_rank, nullptr, L))) return rc;
        const uint32_t P = f.tiles_per_rank * (uint32_t)kTilePix;  // this rank's running average, in frame order
        hipLaunchKernelGGL(blend_packed, dim3(f.tiles_per_rank), dim3(kThreads), 0, c->stream, f, L->cur, accum, rgb8,
                           P);
        VPX_HIP(c, hipGetLastError());
        VPX_HIP(c, hipEventRecord(L->cur_consumed, c->stream));
        return VPX_OK;
    }
    unsigned long long before[kCtrWords] = {};
    if (stats && (rc = snapshot_counters(c, before))) return rc;
    if (stats) VPX_HIP(c, hipEventRecord(c->ev0, c->stream));
    rc = MODE == kFinishPackedSample
             ? launch_render<kFinishPackedSample>(c, c->stream, c->wave, sv, f, f.tiles_per_rank, accum, rgb8, packed)
             : launch_render<kFinishPackedAccum>(c, c->stream, c->wave, sv, f, f.tiles_per_rank, accum, rgb8, packed);
    if (rc) return rc;
    if (stats) {
        VPX_HIP(c, hipEventRecord(c->ev1, c->stream));
        unsigned long long after[kCtrWords];
        if ((rc = snapshot_counters(c, after))) return rc;
        std::memset(stats, 0, sizeof(*stats));
        fill_stats(stats, before, after);
        float ms = 0.f;
        VPX_HIP(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
        stats->kernel_ms = ms;
        stats->total_ms = ms;
    }
    return VPX_OK;
}

// Tiles per window chain: frames join a chain while it holds at most this many tiles, and
// (with lanes) a window keeps at least one chain per lane.  C4 (32400 tiles a frame, 16 spp,
// 4 lanes): one GPU renders 4 chains of 4 frames (26.9 ms a step against 28.5 frame by
// frame), rank 0 of 8 (4050 tiles) 4 chains of 4 frames (3.7 ms against 7.3): profiles/r06_window_ab.txt.
#ifndef VPX_WINDOW_TILES
#define VPX_WINDOW_TILES 131072
#endif
// Window chains of big frames (at least this many tiles a frame) whose tail is a launch of
// its own blend in that tail (k_finish_window), once the previous chain's tail has run: C4 one
// GPU 26.60-26.66 vs 26.95 ms per step.  Small shares keep the blend on the caller's stream
// (blend_window): the tail's wait for the previous chain held each lane (C4 rank 0 of 8: 4.12
// vs 3.68 ms), profiles/r06_window_ab.txt.  0 = never.
#ifndef VPX_WINDOW_FUSED
#define VPX_WINDOW_FUSED 16384
#endif
#ifndef VPX_WINDOW_LANE_CAP
#define VPX_WINDOW_LANE_CAP 1
#endif

static int render_window_impl(vpx_ctx* c, const vpx_frame_params* p, uint32_t n, uint32_t rank, uint32_t n_ranks,
                              bool image, float* accum, uint32_t* rgb8) {
    if (!c) return VPX_E_INVALID;
    int rc = validate_frame(c, p);
    if (rc) return rc;
    if (n == 0) return VPX_OK;
    if (image ? !accum : (!accum || !rgb8)) return fail(c, VPX_E_INVALID, "null accumulator buffer");
    if (n_ranks == 0 || rank >= n_ranks) return fail(c, VPX_E_INVALID, "bad rank");
    const FrameArgs f0 = frame_of(c, p, rank, n_ranks);
    const uint32_t T = image ? f0.num_tiles : f0.tiles_per_rank;
    uint32_t bmax = std::min<uint32_t>(kMaxWindow, std::max<uint32_t>(1u, VPX_WINDOW_TILES / T));
    // at least one chain per lane, so the lanes keep chains in flight as they do frames
    if (VPX_WINDOW_LANE_CAP && c->lanes.size() > 1)
        bmax = std::min<uint32_t>(bmax, std::max<uint32_t>(1u, (n + (uint32_t)c->lanes.size() - 1) / (uint32_t)c->lanes.size()));
    // the shadow lists pack a path index into 27 bits (validate_frame's bound per chain)
    while (bmax > 1 && (uint64_t)bmax * T * kTilePix > (1ull << 27)) --bmax;
    const bool per_frame = bmax == 1 || n == 1 || (p->flags & VPX_FLAG_NO_TONEMAP) || !c->members.empty();
    for (uint32_t i = 0; i < n;) {
        vpx_frame_params q = *p;
        q.frame_index = p->frame_index + i;
        if (per_frame) {
            rc = image ? vpx_render(c, &q, accum, rgb8, nullptr)
                       : vpx_render_tiles_accum(c, &q, kTile, kTile, rank, n_ranks, accum, rgb8, nullptr);
            if (rc) return rc;
            ++i;
            continue;
        }
        const uint32_t B = std::min(bmax, n - i);
        VPX_HIP(c, hipSetDevice(c->device));
        const SceneView sv = view_of(c, q.sky, q.area_samples, (q.flags & VPX_FLAG_SKY) != 0);
        FrameArgs f = frame_of(c, &q, rank, n_ranks);
        f.batch_tiles = T;
        WindowWeights ww;
        for (uint32_t b = 0; b < B; ++b) {  // frame_of's weight per frame
            ww.w[b] = 1.0f / ((float)(q.frame_index + b) + 1.0f);
            ww.iw[b] = 1.0f - ww.w[b];
        }
        float4* samples = nullptr;
        vpx_ctx::Lane* L = nullptr;
        if (!c->lanes.empty() && VPX_WINDOW_FUSED && T >= VPX_WINDOW_FUSED && lane_tail_ok(sv, f)) {
            // the chain's own tail blends its frames into the accumulator (k_finish_window) on
            // its lane, once the caller's stream has reached this call — which orders it after
            // the previous chain's tail, as vpx_render's lane_tail_ok frames
            vpx_ctx::Lane& FL = c->lanes[c->lane_next];
            c->lane_next = (c->lane_next + 1u) % (uint32_t)c->lanes.size();
            if (FL.used) VPX_HIP(c, hipStreamWaitEvent(FL.s, FL.consumed, 0));
            VPX_HIP(c, hipEventRecord(FL.caller, c->stream));
            WindowTail wt;
            wt.B = B;
            wt.image = image ? 1 : 0;
            wt.ww = ww;
            if ((rc = launch_render<kFinishPackedSample>(c, FL.s, FL.ws, sv, f, B * T, reinterpret_cast<float4*>(accum),
                                                         rgb8, nullptr, nullptr, &FL.caller, &wt)))
                return rc;
            VPX_HIP(c, hipEventRecord(FL.rendered, FL.s));
            VPX_HIP(c, hipStreamWaitEvent(c->stream, FL.rendered, 0));
            VPX_HIP(c, hipEventRecord(FL.consumed, FL.s));
            FL.used = true;
            i += B;
            continue;
        }
        if (!c->lanes.empty()) {
            if ((rc = lane_render(c, sv, f, B * T, nullptr, L))) return rc;
            samples = L->cur;
        } else {
            const size_t need = (size_t)B * T * kTilePix;
            if (c->win_len < need) {
                VPX_HIP(c, hipStreamSynchronize(c->stream));
                if (c->win_buf) (void)hipFree(c->win_buf);
                c->win_buf = nullptr;
                c->win_len = 0;
                VPX_HIP(c, hipMalloc(&c->win_buf, sizeof(float4) * need));
                c->win_len = need;
            }
            samples = c->win_buf;
            if ((rc = launch_render<kFinishPackedSample>(c, c->stream, c->wave, sv, f, B * T, nullptr, nullptr,
                                                         samples)))
                return rc;
        }
        hipLaunchKernelGGL(blend_window, dim3(T), dim3(kThreads), 0, c->stream, f, samples, B, ww, image ? 1 : 0,
                           reinterpret_cast<float4*>(accum), rgb8);
        VPX_HIP(c, hipGetLastError());
        if (L) VPX_HIP(c, hipEventRecord(L->cur_consumed, c->stream));
        i += B;
    }
    return VPX_OK;
}

int vpx_render_window(vpx_ctx* c, const vpx_frame_params* p, uint32_t n_frames, float* accum, uint32_t* rgb8) {
    return render_window_impl(c, p, n_frames, 0, 1, true, accum, rgb8);
}

int vpx_render_tiles_accum_window(vpx_ctx* c, const vpx_frame_params* p, uint32_t n_frames, uint32_t tile_w,
                                  uint32_t tile_h, uint32_t rank, uint32_t n_ranks, float* accum_packed,
                                  uint32_t* rgb8_packed) {
    VPX_GROUP_FIRST(c, vpx_render_tiles_accum_window(m_, p, n_frames, tile_w, tile_h, rank, n_ranks, accum_packed,
                                                     rgb8_packed));
    if (c && (tile_w != kTile || tile_h != kTile)) return fail(c, VPX_E_INVALID, "tiles must be 16x16");
    return render_window_impl(c, p, n_frames, rank, n_ranks, false, accum_packed, rgb8_packed);
}

int vpx_render_tiles(vpx_ctx* c, const vpx_frame_params* p, uint32_t tile_w, uint32_t tile_h, uint32_t rank,
                     uint32_t n_ranks, float* packed, vpx_stats* stats) {
    VPX_GROUP_FIRST(c, vpx_render_tiles(m_, p, tile_w, tile_h, rank, n_ranks, packed, stats));
    return render_tiles_impl(kFinishPackedSample, c, p, tile_w, tile_h, rank, n_ranks, nullptr, nullptr,
                                                  reinterpret_cast<float4*>(packed), stats);
}

int vpx_render_tiles_accum(vpx_ctx* c, const vpx_frame_params* p, uint32_t tile_w, uint32_t tile_h, uint32_t rank,
                           uint32_t n_ranks, float* accum_packed, uint32_t* rgb8_packed, vpx_stats* stats) {
    VPX_GROUP_FIRST(c, vpx_render_tiles_accum(m_, p, tile_w, tile_h, rank, n_ranks, accum_packed, rgb8_packed, stats));
    return render_tiles_impl(kFinishPackedAccum, c, p, tile_w, tile_h, rank, n_ranks,
                                                 reinterpret_cast<float4*>(accum_packed), rgb8_packed, nullptr, stats);
}

int vpx_composite_rgb8(vpx_ctx* c, const vpx_frame_params* p, uint32_t tile_w, uint32_t tile_h, uint32_t n_ranks,
                       const uint32_t* gathered, uint32_t* rgb8) {
    VPX_GROUP_FIRST(c, vpx_composite_rgb8(m_, p, tile_w, tile_h, n_ranks, gathered, rgb8));
    if (!c || !p || !gathered || !rgb8) return fail(c, VPX_E_INVALID, "null argument");
    if (tile_w != kTile || tile_h != kTile || n_ranks == 0) return fail(c, VPX_E_INVALID, "tiles must be 16x16");
    if (p->width == 0 || p->height == 0) return fail(c, VPX_E_INVALID, "empty frame");
    VPX_HIP(c, hipSetDevice(c->device));
    const FrameArgs f = frame_of(c, p, 0, n_ranks);
    hipLaunchKernelGGL(composite_rgb8, dim3(f.num_tiles), dim3(kThreads), 0, c->stream, f, gathered, rgb8);
    VPX_HIP(c, hipGetLastError());
    return VPX_OK;
}

int vpx_composite_tiles(vpx_ctx* c, const vpx_frame_params* p, uint32_t tile_w, uint32_t tile_h, uint32_t n_ranks,
                        const float* gathered, float* accum, uint32_t* rgb8) {
    VPX_GROUP_FIRST(c, vpx_composite_tiles(m_, p, tile_w, tile_h, n_ranks, gathered, accum, rgb8));
    if (!c || !p || !gathered || !accum) return fail(c, VPX_E_INVALID, "null argument");
    if (tile_w != kTile || tile_h != kTile || n_ranks == 0) return fail(c, VPX_E_INVALID, "tiles must be 16x16");
    if (p->width == 0 || p->height == 0) return fail(c, VPX_E_INVALID, "empty frame");
    VPX_HIP(c, hipSetDevice(c->device));
    const FrameArgs f = frame_of(c, p, 0, n_ranks);
    hipLaunchKernelGGL(composite_tiles, dim3(f.num_tiles), dim3(kThreads), 0, c->stream, f,
                       reinterpret_cast<const float4*>(gathered), reinterpret_cast<float4*>(accum), rgb8);
    VPX_HIP(c, hipGetLastError());
    return VPX_OK;
}

int vpx_get_counters(vpx_ctx* c, vpx_stats* out, int reset) {
    if (!c || !out) return fail(c, VPX_E_INVALID, "null argument");
    if (!c->members.empty()) {  // sum over the devices
        std::memset(out, 0, sizeof(*out));
        return group_all(c, [&](vpx_ctx* m) {
            vpx_stats one;
            const int rc = vpx_get_counters(m, &one, reset);
            out->primary_rays += one.primary_rays, out->shadow_rays += one.shadow_rays;
            out->bounce_rays += one.bounce_rays, out->dda_cells += one.dda_cells;
            return rc;
        });
    }
    unsigned long long now[kCtrWords];
    int rc = snapshot_counters(c, now);
    if (rc) return rc;
    const unsigned long long zero[kCtrWords] = {};
    std::memset(out, 0, sizeof(*out));
    fill_stats(out, zero, now);
    if (reset) {
        VPX_HIP(c, hipMemsetAsync(c->d_ctr, 0, kCtrWords * kCtrStripes * sizeof(unsigned long long), c->stream));
        VPX_HIP(c, sync_all(c));
    }
    return VPX_OK;
}

int vpx_find_nearest(vpx_ctx* c, const vpx_ray* rays, uint32_t n, vpx_hit* hits) {
    VPX_GROUP_FIRST(c, vpx_find_nearest(m_, rays, n, hits));
    if (!c || (n && (!rays || !hits))) return fail(c, VPX_E_INVALID, "null argument");
    int rc = check_ready(c);
    if (rc) return rc;
    if (n == 0) return VPX_OK;
    const size_t rb = sizeof(vpx_ray) * n, hb = sizeof(vpx_hit) * n;
    if ((rc = ensure_scratch(c, rb + hb))) return rc;
    vpx_ray* dr = (vpx_ray*)c->d_scratch;
    vpx_hit* dh = (vpx_hit*)((char*)c->d_scratch + rb);
    VPX_HIP(c, hipMemcpyAsync(dr, rays, rb, hipMemcpyHostToDevice, c->stream));
    const float sky[3] = {0.392f, 0.584f, 0.829f};
    hipLaunchKernelGGL(find_nearest_k, dim3((n + 255) / 256), dim3(256), 0, c->stream, view_of(c, sky, 3), dr, n, dh);
    VPX_HIP(c, hipGetLastError());
    VPX_HIP(c, hipMemcpyAsync(hits, dh, hb, hipMemcpyDeviceToHost, c->stream));
    VPX_HIP(c, sync_all(c));
    return VPX_OK;
}

int vpx_is_occluded(vpx_ctx* c, const vpx_ray* rays, uint32_t n, uint8_t* occ) {
    VPX_GROUP_FIRST(c, vpx_is_occluded(m_, rays, n, occ));
    if (!c || (n && (!rays || !occ))) return fail(c, VPX_E_INVALID, "null argument");
    int rc = check_ready(c);
    if (rc) return rc;
    if (n == 0) return VPX_OK;
    const size_t rb = sizeof(vpx_ray) * n;
    if ((rc = ensure_scratch(c, rb + n))) return rc;
    vpx_ray* dr = (vpx_ray*)c->d_scratch;
    uint8_t* doc = (uint8_t*)c->d_scratch + rb;
    VPX_HIP(c, hipMemcpyAsync(dr, rays, rb, hipMemcpyHostToDevice, c->stream));
    const float sky[3] = {0.392f, 0.584f, 0.829f};
    hipLaunchKernelGGL(is_occluded_k, dim3((n + 255) / 256), dim3(256), 0, c->stream, view_of(c, sky, 3), dr, n, doc);
    VPX_HIP(c, hipGetLastError());
    VPX_HIP(c, hipMemcpyAsync(occ, doc, n, hipMemcpyDeviceToHost, c->stream));
    VPX_HIP(c, sync_all(c));
    return VPX_OK;
}

int vpx_trace(vpx_ctx* c, const vpx_ray* rays, const uint32_t* seeds, uint32_t n, int32_t depth, const float sky[3],
              int32_t area_samples, float* radiance) {
    VPX_GROUP_FIRST(c, vpx_trace(m_, rays, seeds, n, depth, sky, area_samples, radiance));
    if (!c || (n && (!rays || !seeds || !radiance))) return fail(c, VPX_E_INVALID, "null argument");
    if (depth < -1 || depth > kMaxLevels - 2) return fail(c, VPX_E_INVALID, "depth must be in [-1, 14]");
    if (!sky && !c->d_sky) return fail(c, VPX_E_STATE, "sky == NULL (textured sky) without vpx_set_sky");
    int rc = check_ready(c);
    if (rc) return rc;
    static const float kNoSky[3] = {0.f, 0.f, 0.f};
    if (n == 0) return VPX_OK;
    const size_t rb = sizeof(vpx_ray) * n, sb = 4ull * n, ob = 12ull * n;
    if ((rc = ensure_scratch(c, rb + sb + ob))) return rc;
    vpx_ray* dr = (vpx_ray*)c->d_scratch;
    uint32_t* ds = (uint32_t*)((char*)c->d_scratch + rb);
    float* dout = (float*)((char*)c->d_scratch + rb + sb);
    VPX_HIP(c, hipMemcpyAsync(dr, rays, rb, hipMemcpyHostToDevice, c->stream));
    VPX_HIP(c, hipMemcpyAsync(ds, seeds, sb, hipMemcpyHostToDevice, c->stream));
    const SceneView sv = view_of(c, sky ? sky : kNoSky, area_samples, sky == nullptr);
    const dim3 g((n + 255) / 256), b(256);
    if (depth <= 0)
        hipLaunchKernelGGL(trace_k<1>, g, b, 0, c->stream, sv, dr, ds, n, depth, dout);
    else if (depth <= 4)
        hipLaunchKernelGGL(trace_k<5>, g, b, 0, c->stream, sv, dr, ds, n, depth, dout);
    else
        hipLaunchKernelGGL(trace_k<kMaxLevels>, g, b, 0, c->stream, sv, dr, ds, n, depth, dout);
    VPX_HIP(c, hipGetLastError());
    VPX_HIP(c, hipMemcpyAsync(radiance, dout, ob, hipMemcpyDeviceToHost, c->stream));
    VPX_HIP(c, sync_all(c));
    return VPX_OK;
}

int vpx_bvh_set(vpx_ctx* c, const vpx_bvh_tri* tris, uint32_t n) {
    VPX_GROUP_ALL(c, vpx_bvh_set(m_, tris, n));
    if (!c || (n && !tris)) return fail(c, VPX_E_INVALID, "null argument");
    if (n > VPX_BVH_MAX_TRIS) return fail(c, VPX_E_INVALID, "more triangles than VPX_BVH_MAX_TRIS");
    VPX_HIP(c, sync_all(c));
    if (c->d_bvh) (void)hipFree(c->d_bvh);
    c->d_bvh = nullptr;
    c->bvh_nodes = c->bvh_tris = 0;
    if (!n) return VPX_OK;
    std::vector<vpx_bvh_node> nodes(2 * (size_t)n - 1);
    std::vector<uint32_t> idx(n);
    uint32_t used = 0;
    int rc = vpx_bvh_build_host(tris, n, nodes.data(), idx.data(), &used);
    if (rc) return fail(c, rc, "vpx_bvh_build_host failed");
    // the traversal pushes both children of every interior node it enters
    static_assert(VPX_BVH_MAX_DEPTH + 1 <= kBvhStack, "traversal stack: one pending sibling per level + the root");
    if (vpx_bvh_depth(nodes.data(), used) > VPX_BVH_MAX_DEPTH)
        return fail(c, VPX_E_INVALID, "BVH deeper than VPX_BVH_MAX_DEPTH (the traversal stack)");
    std::vector<uint32_t> img(used * 8u + n * 9u);
    std::memcpy(img.data(), nodes.data(), sizeof(vpx_bvh_node) * used);
    for (uint32_t k = 0; k < n; ++k) std::memcpy(&img[used * 8u + k * 9u], &tris[idx[k]], sizeof(vpx_bvh_tri));
    VPX_HIP(c, hipMalloc(&c->d_bvh, sizeof(uint32_t) * img.size()));
    VPX_HIP(c, hipMemcpy(c->d_bvh, img.data(), sizeof(uint32_t) * img.size(), hipMemcpyHostToDevice));
    c->bvh_nodes = used, c->bvh_tris = n;
    return VPX_OK;
}

int vpx_bvh_intersect(vpx_ctx* c, const vpx_ray* rays, uint32_t n, float* t_out) {
    VPX_GROUP_FIRST(c, vpx_bvh_intersect(m_, rays, n, t_out));
    if (!c || (n && (!rays || !t_out))) return fail(c, VPX_E_INVALID, "null argument");
    if (!c->d_bvh) return fail(c, VPX_E_STATE, "no BVH set (vpx_bvh_set)");
    if (n == 0) return VPX_OK;
    const size_t rb = sizeof(vpx_ray) * n, tb = sizeof(float) * n;
    int rc = ensure_scratch(c, rb + tb);
    if (rc) return rc;
    vpx_ray* dr = (vpx_ray*)c->d_scratch;
    float* dt = (float*)((char*)c->d_scratch + rb);
    VPX_HIP(c, hipMemcpyAsync(dr, rays, rb, hipMemcpyHostToDevice, c->stream));
    const size_t lds = sizeof(uint32_t) * (c->bvh_nodes * 8u + c->bvh_tris * 9u);  // <= 51 KiB (512 triangles)
    hipLaunchKernelGGL(bvh_intersect_k, dim3((n + 255) / 256), dim3(256), lds, c->stream, (const uint32_t*)c->d_bvh,
                       c->bvh_nodes, c->bvh_tris, dr, n, dt);
    VPX_HIP(c, hipGetLastError());
    VPX_HIP(c, hipMemcpyAsync(t_out, dt, tb, hipMemcpyDeviceToHost, c->stream));
    VPX_HIP(c, sync_all(c));
    return VPX_OK;
}

int vpx_focus_distance(vpx_ctx* c, uint32_t width, uint32_t height, float* fd) {
    VPX_GROUP_FIRST(c, vpx_focus_distance(m_, width, height, fd));
    if (!c || !fd || !width || !height) return fail(c, VPX_E_INVALID, "bad argument");
    int rc = check_ready(c);
    if (rc) return rc;
    if (!c->have_camera) return fail(c, VPX_E_STATE, "no camera set");
    if ((rc = ensure_scratch(c, 16))) return rc;
    vpx_frame_params p{};
    p.width = width, p.height = height;
    const float sky[3] = {0, 0, 0};
    hipLaunchKernelGGL(focus_k, dim3(1), dim3(1), 0, c->stream, view_of(c, sky, 3), frame_of(c, &p, 0, 1),
                       (float*)c->d_scratch);
    VPX_HIP(c, hipGetLastError());
    VPX_HIP(c, hipMemcpyAsync(fd, c->d_scratch, sizeof(float), hipMemcpyDeviceToHost, c->stream));
    VPX_HIP(c, sync_all(c));
    return VPX_OK;
}

uint32_t vpx_pixel_seed(uint32_t base, uint32_t frame, uint32_t w, uint32_t h, uint32_t x, uint32_t y) {
    return pixel_seed(base, frame, w, h, x, y);
}


// ------------------------------------------------------------------ device sets
// One frame on a device set (vpx_create_multi): the 16x16 tiles are dealt round-robin to
// the members (tile t -> member t % n, as dist.py deals them to ranks), each member renders
// its tiles on its own device and stream, and the packed results are gathered to member 0
// over RCCL (grouped ncclSend / ncclRecv: n - 1 point-to-point transfers into device 0,
// each on its own xGMI link on an MI355X node) — or by device copies when the set repeats
// a device (RCCL communicators need distinct devices).  Member 0 then composites:
//   accum != NULL: float4 samples (16 B/pixel) -> vpx_composite_tiles into the caller's
//     accumulator + screen, bit-identical to vpx_render on one device;
//   accum == NULL: each member keeps the running average of ITS tiles (sharded
//     accumulator, reset by frame_index 0) and only packed RGB8 (4 B/pixel) travels ->
//     vpx_composite_rgb8 into the screen.
static int group_render(vpx_ctx* c, const vpx_frame_params* p, float* accum, uint32_t* rgb8, vpx_stats* stats) {
    DeviceGuard keep;
    if (!p) return fail(c, VPX_E_INVALID, "null params");
    if (!accum && !rgb8) return fail(c, VPX_E_INVALID, "accum or rgb8 (device pointers on the first device) required");
    const uint32_t n = (uint32_t)c->members.size();
    const uint64_t L = vpx_tiles_packed_len(p->width, p->height, kTile, kTile, n);
    if (!L) return fail(c, VPX_E_INVALID, "empty frame");
    const bool samples = accum != nullptr;
    const size_t elem = samples ? sizeof(float4) : sizeof(uint32_t);
    int rc;
    if (c->g_len < L) {  // (re)size the per-member buffers
        for (uint32_t r = 0; r < n; ++r) {
            vpx_ctx* m = c->members[r];
            VPX_HIP(c, hipSetDevice(m->device));
            VPX_HIP(c, hipStreamSynchronize(m->stream));
            if (c->g_packed[r]) (void)hipFree(c->g_packed[r]);
            if (c->g_accum[r]) (void)hipFree(c->g_accum[r]);
            c->g_packed[r] = nullptr, c->g_accum[r] = nullptr;
            VPX_HIP(c, hipMalloc(&c->g_packed[r], sizeof(float4) * L));
            VPX_HIP(c, hipMalloc((void**)&c->g_accum[r], sizeof(float4) * L));
            VPX_HIP(c, hipMemsetAsync(c->g_accum[r], 0, sizeof(float4) * L, m->stream));
            if (r == 0) {
                if (c->g_gathered) (void)hipFree(c->g_gathered);
                c->g_gathered = nullptr;
                VPX_HIP(c, hipMalloc(&c->g_gathered, sizeof(float4) * L * n));
            }
        }
        c->g_len = L;
    }
    vpx_ctx* m0 = c->members[0];
    if (stats) std::memset(stats, 0, sizeof(*stats));
    // stats: every member's counters are read BEFORE any member launches and after the whole
    // set is done, and each member's render is bracketed by events on its own stream, so
    // taking stats does not serialise the members (their launches still overlap)
    std::vector<std::array<unsigned long long, kCtrWords>> before(stats ? n : 0);
    if (stats)
        for (uint32_t r = 0; r < n; ++r) {
            VPX_HIP(c, hipSetDevice(c->members[r]->device));
            if ((rc = snapshot_counters(c->members[r], before[r].data()))) return fail(c, rc, c->members[r]->err);
        }
    // 1. every member renders its tiles (launches are asynchronous: the devices overlap)
    for (uint32_t r = 0; r < n; ++r) {
        vpx_ctx* m = c->members[r];
        VPX_HIP(c, hipSetDevice(m->device));
        if (c->comms.empty())  // copy path: the previous frame's copy of this buffer is done
            VPX_HIP(c, hipStreamWaitEvent(m->stream, c->g_copied, 0));
        if (stats) VPX_HIP(c, hipEventRecord(m->ev0, m->stream));
        rc = samples ? vpx_render_tiles(m, p, kTile, kTile, r, n, (float*)c->g_packed[r], nullptr)
                     : vpx_render_tiles_accum(m, p, kTile, kTile, r, n, c->g_accum[r], (uint32_t*)c->g_packed[r],
                                              nullptr);
        if (rc) return fail(c, rc, "device " + std::to_string(m->device) + ": " + m->err);
        if (stats) VPX_HIP(c, hipEventRecord(m->ev1, m->stream));
        if (c->comms.empty()) VPX_HIP(c, hipEventRecord(c->g_ev[r], m->stream));
    }
    // 2. gather the packed buffers to member 0
    char* dst = (char*)c->g_gathered;
    const size_t bytes = elem * L;
    if (!c->comms.empty()) {
        VPX_HIP(c, hipSetDevice(m0->device));
        VPX_HIP(c, hipMemcpyAsync(dst, c->g_packed[0], bytes, hipMemcpyDeviceToDevice, m0->stream));
        if (ncclGroupStart() != ncclSuccess) return fail(c, VPX_E_DEVICE, "ncclGroupStart");
        for (uint32_t r = 1; r < n; ++r) {
            if (ncclRecv(dst + bytes * r, bytes, ncclChar, (int)r, c->comms[0], m0->stream) != ncclSuccess ||
                ncclSend(c->g_packed[r], bytes, ncclChar, 0, c->comms[r], c->members[r]->stream) != ncclSuccess) {
                (void)ncclGroupEnd();
                return fail(c, VPX_E_DEVICE, "RCCL gather");
            }
        }
        if (ncclGroupEnd() != ncclSuccess) return fail(c, VPX_E_DEVICE, "ncclGroupEnd");
    } else {
        VPX_HIP(c, hipSetDevice(m0->device));
        for (uint32_t r = 0; r < n; ++r) {
            vpx_ctx* m = c->members[r];
            VPX_HIP(c, hipStreamWaitEvent(m0->stream, c->g_ev[r], 0));
            VPX_HIP(c, hipMemcpyPeerAsync(dst + bytes * r, m0->device, c->g_packed[r], m->device, bytes, m0->stream));
        }
        VPX_HIP(c, hipEventRecord(c->g_copied, m0->stream));
    }
    // 3. member 0 composites into the caller's buffers
    rc = samples ? vpx_composite_tiles(m0, p, kTile, kTile, n, (const float*)dst, accum, rgb8)
                 : vpx_composite_rgb8(m0, p, kTile, kTile, n, (const uint32_t*)dst, rgb8);
    if (rc) return fail(c, rc, m0->err);
    if (stats) {  // kernel_ms: the slowest member's render; total_ms: member 0's start to the composite's end
        VPX_HIP(c, hipSetDevice(m0->device));
        VPX_HIP(c, hipEventRecord(m0->ev2, m0->stream));
        for (uint32_t r = 0; r < n; ++r) {
            vpx_ctx* m = c->members[r];
            VPX_HIP(c, hipSetDevice(m->device));
            unsigned long long after[kCtrWords];
            if ((rc = snapshot_counters(m, after))) return fail(c, rc, m->err);  // synchronises m's stream
            vpx_stats one;
            std::memset(&one, 0, sizeof(one));
            fill_stats(&one, before[r].data(), after);
            stats->primary_rays += one.primary_rays, stats->shadow_rays += one.shadow_rays;
            stats->bounce_rays += one.bounce_rays, stats->dda_cells += one.dda_cells;
            float ms = 0.f;
            VPX_HIP(c, hipEventElapsedTime(&ms, m->ev0, m->ev1));
            stats->kernel_ms = std::max(stats->kernel_ms, ms);
        }
        VPX_HIP(c, hipSetDevice(m0->device));
        float tot = 0.f;
        VPX_HIP(c, hipEventElapsedTime(&tot, m0->ev0, m0->ev2));
        stats->total_ms = std::max(tot, stats->kernel_ms);
    }
    return VPX_OK;
}

int vpx_create_multi(const int* devices, int ndev, vpx_ctx** out) {
    if (!out) return VPX_E_INVALID;
    *out = nullptr;
    if (!devices || ndev < 1 || ndev > 64) return VPX_E_INVALID;
    DeviceGuard keep;
    vpx_ctx* c = new (std::nothrow) vpx_ctx();
    if (!c) return VPX_E_NOMEM;
    c->device = devices[0];
    bool distinct = true;
    for (int r = 0; r < ndev; ++r) {
        for (int q = 0; q < r; ++q) distinct &= devices[q] != devices[r];
        vpx_ctx* m = nullptr;
        const int rc = vpx_create(devices[r], &m);
        if (rc) {
            vpx_destroy(c);
            return rc;
        }
        c->members.push_back(m);
        c->g_packed.push_back(nullptr);
        c->g_accum.push_back(nullptr);
        c->g_ev.push_back(nullptr);
        if (hipEventCreateWithFlags(&c->g_ev.back(), hipEventDisableTiming) != hipSuccess) {
            vpx_destroy(c);
            return VPX_E_DEVICE;
        }
    }
    (void)hipSetDevice(devices[0]);
    if (hipEventCreateWithFlags(&c->g_copied, hipEventDisableTiming) != hipSuccess) {
        vpx_destroy(c);
        return VPX_E_DEVICE;
    }
    if (distinct && ndev > 1) {  // one RCCL communicator per device, all in this process
        c->comms.assign(ndev, nullptr);
        if (ncclCommInitAll(c->comms.data(), ndev, devices) != ncclSuccess) {
            c->comms.clear();
            vpx_destroy(c);
            return VPX_E_DEVICE;
        }
    }
    *out = c;
    return VPX_OK;
}

}  // extern "C"

extern "C" int vpx_profile_select(vpx_ctx* c, uint32_t stage_mask) {
    VPX_GROUP_FIRST(c, vpx_profile_select(m_, stage_mask));
    if (!c) return VPX_E_INVALID;
    c->prof_mask = stage_mask;
    return VPX_OK;
}

extern "C" int vpx_profile_enable(vpx_ctx* c, uint32_t max_launches) {
    VPX_GROUP_FIRST(c, vpx_profile_enable(m_, max_launches));
    if (!c) return VPX_E_INVALID;
    VPX_HIP(c, sync_all(c));
    for (hipEvent_t e : c->prof_ev) (void)hipEventDestroy(e);
    c->prof_ev.clear();
    c->prof_stage.clear();
    c->prof_cap = c->prof_used = 0;
    if (!max_launches) return VPX_OK;
    if (max_launches > 1u << 16) return fail(c, VPX_E_INVALID, "max_launches too large");
    c->prof_ev.resize(2 * (size_t)max_launches, nullptr);
    c->prof_stage.resize(2 * (size_t)max_launches, -1);
    for (auto& e : c->prof_ev) VPX_HIP(c, hipEventCreate(&e));
    c->prof_cap = 2 * max_launches;
    return VPX_OK;
}

// Length of the union of [first, second) intervals (any sign), overlaps counted once.
static float interval_union_ms(std::vector<std::pair<float, float>>& iv) {
    if (iv.empty()) return 0.f;
    std::sort(iv.begin(), iv.end());
    float busy = 0.f, lo = iv[0].first, hi = iv[0].second;
    for (const auto& v : iv) {
        if (v.first > hi) {
            busy += hi - lo;
            lo = v.first, hi = v.second;
        } else if (v.second > hi) {
            hi = v.second;
        }
    }
    return busy + (hi - lo);
}

// Host check of the union (tests/test_abi.py): n intervals as (start, end) pairs.
extern "C" float vpx_profile_busy_union(const float* se, uint32_t n) {
    std::vector<std::pair<float, float>> iv;
    for (uint32_t i = 0; i < n; ++i) iv.emplace_back(se[2 * i], se[2 * i + 1]);
    return interval_union_ms(iv);
}

extern "C" int vpx_profile_read(vpx_ctx* c, vpx_profile* out, int reset) {
    VPX_GROUP_FIRST(c, vpx_profile_read(m_, out, reset));
    if (!c || !out) return fail(c, VPX_E_INVALID, "null argument");
    std::memset(out, 0, sizeof(*out));
    unsigned long long now[kCtrWords];
    int rc = snapshot_counters(c, now);  // synchronises the stream
    if (rc) return rc;
    for (uint32_t st = 0; st < 8; ++st) out->stage_cells[st] = now[8 + st];
    std::vector<std::pair<float, float>> iv[8];  // per stage: launch intervals, ms after the first event
    for (uint32_t i = 0; i + 1 < c->prof_used; i += 2) {
        float ms = 0.f, t0 = 0.f;
        VPX_HIP(c, hipEventElapsedTime(&ms, c->prof_ev[i], c->prof_ev[i + 1]));
        VPX_HIP(c, hipEventElapsedTime(&t0, c->prof_ev[0], c->prof_ev[i]));
        const int st = c->prof_stage[i];
        if (st >= 0 && st < 8) {
            out->stage_ms[st] += ms;
            ++out->stage_launches[st];
            iv[st].emplace_back(t0, t0 + ms);
        }
    }
    // busy time: the union of the intervals.  Offsets are measured from prof_ev[0], which may
    // sit on another lane's stream, so a launch can start before it (a negative offset): the
    // union starts from the first sorted interval, not from a sentinel at 0.
    for (uint32_t st = 0; st < 8; ++st) out->stage_busy_ms[st] = interval_union_ms(iv[st]);
    if (reset) {
        c->prof_used = 0;
        unsigned long long* d = c->d_ctr;
        std::vector<unsigned long long> h(kCtrWords * kCtrStripes);
        VPX_HIP(c, hipMemcpy(h.data(), d, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
        for (uint32_t s = 0; s < kCtrStripes; ++s)
            for (uint32_t st = 8; st < 16; ++st) h[kCtrWords * s + st] = 0;
        VPX_HIP(c, hipMemcpy(d, h.data(), sizeof(unsigned long long) * h.size(), hipMemcpyHostToDevice));
    }
    return VPX_OK;
}

#ifdef VPX_PHASE_PROF
extern "C" int vpx_debug_phase(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(vpx::g_phase), sizeof(unsigned long long) * 32) != hipSuccess) return -1;
    if (reset) {
        const unsigned long long z[32] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(vpx::g_phase), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
