// vpx_wavefront.hpp — the per-frame render as a wavefront of small kernels.
//
// Renderer::Trace (renderer.cpp:1076-1328) is one chain per pixel.  Instead of one big
// kernel that carries the whole chain (VGPR-heavy, 2 waves/SIMD), each bounce level runs
//   nearest  — primary/bounce ray -> Renderer::FindNearest               (DDA, lean)
//   shade    — material dispatch: RNG, next ray, light choice, and the shadow rays the
//              light evaluation would cast, with their unoccluded contributions
//   shadow   — Renderer::IsOccluded for those rays, then the light's sum    (DDA, lean)
// and a final `finish` folds the per-level (a, b, form) records bottom-up exactly as the
// recursion does and accumulates / tonemaps (or packs tiles for the multi-GPU gather).
// The RNG is consumed only in `shade`, in the reference order, and no RNG draw depends on
// an occlusion result (renderer.cpp:102-207 draw before they test), so splitting the
// chain changes no value: results stay bit-identical to the restatement.
//
// Path state lives in HBM as structure-of-arrays float4 streams (coalesced 16-B lanes).
#pragma once

#include "vpx_trace.hpp"

namespace vpx {

constexpr int kTileW = 16;
constexpr int kTilePix = kTileW * kTileW;



// flags word of a path (stored in D.w)
constexpr uint32_t kActive = 1u;
constexpr uint32_t kInside = 2u;

// shadow-slot flags (stored in SH_D.w)
constexpr uint32_t kSlotValid = 1u;
constexpr uint32_t kSlotDiscard = 2u;  // smoke player probe: traced for the count, result unused

// internal frame flag: the static-camera path (Renderer::TraceReproject + reprojection)
constexpr uint32_t kFlagReproject = 0x80000000u;
// pending-light bit: the level adds its light to a zero first (TraceNonMetal's
// `illumination{0}; illumination += incLight`, renderer.cpp:1343-1357)
constexpr uint32_t kPendZeroAdd = 1u << 13;

// light kinds of a level's pending incLight
constexpr uint32_t kLightNone = 0, kLightSingle = 1, kLightArea = 2;

struct FrameArgs {
    vpx_camera cam;
    uint32_t width, height;
    int32_t max_bounces;
    uint32_t frame_index;
    uint32_t seed_base;
    uint32_t flags;
    float aa;
    float weight;      // 1/(n+1)
    float inv_weight;  // 1 - weight
    uint32_t tiles_x, tiles_y, num_tiles;
    uint32_t rank, n_ranks;
    uint32_t tiles_per_rank;
    // an accumulation window rendered in one chain (vpx_render_window): paths of frame
    // frame_index + b fill tile blocks [b*batch_tiles, (b+1)*batch_tiles); 0 = one frame
    uint32_t batch_tiles;
};

// Per-path level forms: level l's 2-bit form at bits 2l..2l+1 and a sentinel 1 just above
// the last recorded level, so a count of up to kMaxLevels - 1 = 15 levels (max_bounces 14)
// takes bits 0..30 (a separate count field would not fit beside 30 form bits).
// Bit 31 says the path ended on a leaf value (sky / emissive) held in `leaf`; without it the
// leaf is 0 (Trace(ray, -1)) and is not read, so no kernel zero-fills the leaf buffer.
constexpr uint32_t kLeafBit = 0x80000000u;
static_assert(2 * (kMaxLevels - 1) < 31, "forms word: 2 bits per level + sentinel + leaf bit must fit 32 bits");
__device__ __forceinline__ uint32_t forms_count(uint32_t forms) {
    return (31u - (uint32_t)__clz(forms & ~kLeafBit)) >> 1;
}

// Where a kernel finds the ray (O, D) and hit record (H, HM) of the path it works on: the
// global path buffers, or the workgroup's LDS in the fused head (k_primary<.., true>), whose
// walkers and level-0 shade hand them over inside the workgroup (base = the tile's first
// path).  Only the fused head uses LDS; every later kernel reads the global buffers.
struct PathRay {
    float4* O;
    float4* D;
    float4* H;
    uint32_t* HM;
    uint32_t base;
    __device__ __forceinline__ uint32_t at(uint32_t p) const { return p - base; }
};

struct WaveBufs {
    float4* O;     // [P] ray origin, w = rng state bits
    float4* D;     // [P] ray direction, w = flags bits (kActive | kInside)
    float4* H;     // [P] hit: t, normal
    uint32_t* HM;  // [P] hit: material | (vox + 2) << 8
    int32_t* depth;  // [P] remaining Trace depth
    uint32_t* forms; // [P] form of level l in bits 2l..2l+1, sentinel 1 at bit 2*count (forms_count)
    float4* LA;    // [L][P] level multiplier a (xyz)
    float4* LB;    // [L][P] level addend b (xyz)
    float4* leaf;  // [P] leaf radiance (sky / emissive / 0)
    float4* SO;    // [S][P] shadow origin, w = tmax
    float4* SD;    // [S][P] shadow direction, w = slot flags bits
    float4* SL;    // [S][P] unoccluded contribution of the slot
    float4* SM;    // [P] pending light: xyz = kd (area), w = bits(kind | discard<<3 | count<<4 | level<<8 | lc<<16)
    uint32_t* smask;  // [P] shadow slots emitted this level (bit s = slot s, s < 15) | light key << 16
    uint32_t* live0;  // [P] live-path lists: the paths that trace a ray at level l (l >= 1) are
    uint32_t* live1;  //     live{l & 1}[0 .. pool[kPoolLive + l]) (k_compact after level l - 1's shade)
    uint64_t* amask;  // [P/64] bit i of word i >> 6: the path at list position i of the level being
                      // shaded (level 0: path i) traces a next ray (the shades write it, k_compact reads it)
    uint32_t* pool;   // [kPoolWords] the level counters (kPool*), zeroed at the start of every frame that
                      // uses them (launch_render)
    uint8_t* occb;    // [S][P] the shadow pool's result per slot: 1 = occluded (valid slots only),
                      // followed by slot_list's [S * P] words
    float4* RD;    // [W*H] reprojection: level-0 intersection point, w = material bits (image order)
    uint32_t P;    // paths (pixels) this call
    uint32_t S;    // shadow slots per path
};

// Multi-volume scenes: the slots the shadow pool left unoccluded whose segment may meet a later
// volume (slot << 27 | path), pool[kPoolSlots + level * kLineWords] of them; stored after occb
// (ensure_wave) rather than in a WaveBufs field of its own (the pool's registers: a bigger
// kernel argument block cost k_shadow_pool two more spilled VGPRs).
__device__ __forceinline__ uint32_t* slot_list(const WaveBufs& w) {
    return reinterpret_cast<uint32_t*>(w.occb + (((size_t)w.P * w.S + 255u) & ~(size_t)255u));
}

// Level counters in WaveBufs::pool: the length of level l's live-path list, and the pools'
// chunk grabs (kGrabStripes counters per level) of its shadow walks and its bounce walks.
// (Spreading the pools' grabs over 16 counters per level — stripe s dealing chunks s, s + 16,
// ... — measured much slower: C2 5.64 vs 2.54 ms, C3 3.93 vs 3.65, C4 49.7 vs 43.1.  The
// counters share a cache line, so the L2 still serialises them, the tail takes up to 16 atomics
// per wave, and the frame is no longer swept in order, so the waves' lines are spread further.)
// The pools' grab counters: kGrabLines counters per level, each on its own 128-byte line (the
// L2 serialises atomics per line), counter k dealing chunks k, k + kGrabLines, ...; a wave
// starts on its own counter and moves to the next when it runs dry, and an exhausted counter
// sets its bit in the level's mask word (its own line) so that later waves skip it.
#ifndef VPX_GRAB_LINES
#define VPX_GRAB_LINES 1
#endif
constexpr uint32_t kGrabLines = VPX_GRAB_LINES, kLineWords = 32;
constexpr uint32_t kGrabBlock = (kGrabLines + 1u) * kLineWords;  // per level: the counters, then the mask
constexpr uint32_t kPoolLive = 0, kPoolShadow = kLineWords, kPoolBounce = kPoolShadow + kMaxLevels * kGrabBlock,
                   kPoolSlots = kPoolBounce + kMaxLevels * kGrabBlock,  // per level, its own line: slist's length
                   kPoolWords = kPoolSlots + kMaxLevels * kLineWords;

// The next of `chunks` chunks for this wave (wave-uniform; lane 0 takes it), ~0u when none is
// left.  blk: the level's grab block; line: the wave's current counter (wave-uniform).
__device__ __forceinline__ uint32_t pool_grab(uint32_t* blk, uint32_t chunks, uint32_t& line) {
    const bool lead = (threadIdx.x & 63u) == 0u;
    if (kGrabLines == 1u) {
        uint32_t g = 0u;
        if (lead) g = atomicAdd(blk, 1u);
        g = __builtin_amdgcn_readfirstlane(g);
        return g < chunks ? g : ~0u;
    }
    for (uint32_t t = 0; t < kGrabLines; ++t) {
        const uint32_t done = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(blk + kGrabLines * kLineWords, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if (!((done >> line) & 1u)) {
            uint32_t k = 0u;
            if (lead) k = atomicAdd(blk + line * kLineWords, 1u);
            k = __builtin_amdgcn_readfirstlane(k);
            const uint32_t c = line + k * kGrabLines;
            if (c < chunks) return c;
            if (lead) atomicOr(blk + kGrabLines * kLineWords, 1u << line);
        }
        line = line + 1u == kGrabLines ? 0u : line + 1u;
    }
    return ~0u;
}
__device__ __forceinline__ uint32_t pool_line0() {
    return __builtin_amdgcn_readfirstlane((blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) % kGrabLines);
}

// The scene view a kernel instance works with: X86 = false drops the reference-arithmetic
// tables (a constant null tab, so the exact arithmetic is inlined without its runtime branch:
// the branch cost C1 1.2 %, 0.5527-0.5563 vs 0.5445-0.5477 ms); X86 = true keeps them.
template <bool X86>
__device__ __forceinline__ SceneView arith_view(const SceneView& sv) {
    SceneView v = sv;
    if (!X86) v.x86.tab = nullptr;
    return v;
}

// Level l's paths: level 0 is every path of the launch (p = i); a later level's are the paths
// that trace a ray there, listed by the previous level's shade (put_live).  Every kernel after
// level 0's head walks / shades / resolves the list, so a level costs its live paths — Z1's
// deep levels hold a few thousand of the frame's two million.
__device__ __forceinline__ const uint32_t* live_list(const WaveBufs& w, int level) {
    return (level & 1) ? w.live1 : w.live0;
}
__device__ __forceinline__ uint32_t live_count(const WaveBufs& w, int level) {
    return level ? __builtin_amdgcn_readfirstlane(w.pool[kPoolLive + level]) : w.P;
}
__device__ __forceinline__ uint32_t live_path(const WaveBufs& w, int level, uint32_t i) {
    return level ? live_list(w, level)[i] : i;
}

// ------------------------------------------------------------------ primary rays
// Camera::GetPrimaryRayNoDOF (camera.h:103-110) / GetPrimaryRay + thin lens (:68-83);
// AA jitter as the AVX path: fma(rand, aa, x) (renderer.cpp:1699-1708).
// Reference arithmetic (xa.tab set, not the static-camera path, whose GetPrimaryRayNoDOF goes
// through the Ray constructor): the AVX loop's normalize(__m128) = v * rsqrtps(dpps(v, v,
// 0x7F)) (tmpl8math.h:2356-2360, renderer.cpp:1735-1765), the dot product summed
// (x*x + y*y) + z*z as dpps does, rsqrtps from the host's captured table (vpx_x86.hpp).
__device__ __forceinline__ Ray primary_make_ray(f3 o, f3 dir, const X86Arith& xa, bool x86) {
#ifdef VPX_DEBUG_X86_NO_RSQ  // timing probe only (wrong results)
    x86 = false;
#endif
    if (!x86) return make_ray(o, dir);
    Ray r = make_ray(o, dir);
    const float dp = (dir.x * dir.x + dir.y * dir.y) + dir.z * dir.z;
    const float inv = __uint_as_float(x86_rsq_bits(__float_as_uint(dp), xa.tab + xa.rsq_off, xa.rsq_shift));
    r.D = dir * inv;
    return r;
}
__device__ __forceinline__ Ray primary_ray(const FrameArgs& f, uint32_t x, uint32_t y, Rng& g, const X86Arith& xa) {
#ifndef VPX_NO_X86
    const bool x86 = xa.tab && !(f.flags & kFlagReproject);
#else
    const bool x86 = false;
#endif
    float fx = (float)x, fy = (float)y;
    if (f.flags & VPX_FLAG_AA) {
        const float rx = g.next(), ry = g.next();
        fx = fmaf(rx, f.aa, fx);
        fy = fmaf(ry, f.aa, fy);
    }
    const float u = fx * (1.0f / (float)f.width);
    const float v = fy * (1.0f / (float)f.height);
    const f3 tl = ld3(f.cam.top_left), tr = ld3(f.cam.top_right), bl = ld3(f.cam.bottom_left);
    const f3 P = (tl + (tr - tl) * u) + (bl - tl) * v;
    const f3 cp = ld3(f.cam.cam_pos);
    if (f.flags & VPX_FLAG_DOF) {
        const float rr = sqrtf(g.next());
        const float theta = g.next() * (2.0f * kPi);
        float st, ct;
        dm::sincos(theta, st, ct);
        const float cx = ct * rr, cy = st * rr;
        const float jx = (cx * f.cam.defocus_jitter) / (float)f.width;
        const float jy = (cy * f.cam.defocus_jitter) / (float)f.width;
        const f3 focal = cp + normalize(P - cp) * f.cam.focal_distance;
        const f3 o = (cp + ld3(f.cam.right) * jx) + ld3(f.cam.up) * jy;
        return primary_make_ray(o, focal - o, xa, x86);
    }
    return primary_make_ray(cp, P - cp, xa, x86);
}

// Lane -> pixel inside a 16x16 tile: the tile's four waves take its four 8x8 quadrants
// (row-major quadrant order), each row-major inside — a wave's rays leave from an 8x8 block
// rather than a 16x4 strip, so their walks overlap more (C1 / C3 -0.3 / -0.5 %, three
// interleaved A/B rounds).  Also the order of a tile's 256 entries in the packed buffers.
__device__ __forceinline__ void tile_lane_xy(uint32_t lane, uint32_t& lx, uint32_t& ly) {
    lx = ((lane >> 6) & 1u) * 8u + (lane & 7u);
    ly = (lane >> 7) * 8u + ((lane >> 3) & 7u);
}
// Path index -> pixel: path p = j*256 + lane covers the j-th tile of this rank
// (tile = rank + j*n_ranks), lane as tile_lane_xy.
__device__ __forceinline__ bool tile_pixel(const FrameArgs& f, uint32_t j, uint32_t lane, uint32_t& x, uint32_t& y) {
    const uint32_t tile = f.rank + j * f.n_ranks;
    uint32_t lx, ly;
    tile_lane_xy(lane, lx, ly);
    x = (tile % f.tiles_x) * kTileW + lx;
    y = (tile / f.tiles_x) * kTileW + ly;
    return tile < f.num_tiles && x < f.width && y < f.height;
}
// A window chain's frame b holds tile blocks [b*batch_tiles, (b+1)*batch_tiles).
__device__ __forceinline__ bool path_pixel(const FrameArgs& f, uint32_t p, uint32_t& x, uint32_t& y) {
    const uint32_t j = p >> 8;
    return tile_pixel(f, f.batch_tiles ? j % f.batch_tiles : j, p & 255u, x, y);
}
// Paths of frames that never join a window chain (the static-camera path).
__device__ __forceinline__ bool path_pixel_single(const FrameArgs& f, uint32_t p, uint32_t& x, uint32_t& y) {
    return tile_pixel(f, p >> 8, p & 255u, x, y);
}
// The frame of path p in a window chain (FrameArgs::batch_tiles).
__device__ __forceinline__ uint32_t path_frame(const FrameArgs& f, uint32_t p) {
    return f.frame_index + (f.batch_tiles ? (p >> 8) / f.batch_tiles : 0u);
}

// Sum over the wave (every lane gets it).  DPP row shifts / mirrors rather than __shfl_xor:
// the shuffles' lane-address registers were hoisted and kept live (spilled) across
// k_frame0's walks, since the three counter flushes share them.
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) { return __reduce_add_sync(~0ull, v); }

// Work counters: [0] shadow rays, [1] FindNearest calls, [2] DDA cells, [3] primary rays,
// [8 + s] DDA cells of stage s (VPX_STAGE_*), striped over kCtrStripes copies of
// kCtrWords words (one 64-bit atomic per counter per wave, spread over addresses by
// workgroup so that waves do not serialise on one word); summed on readout.
constexpr uint32_t kCtrStripes = 64;
constexpr uint32_t kCtrWords = 16;
__device__ __forceinline__ void flush_counters(const Counters& k, uint32_t primary, unsigned long long* ctr,
                                               uint32_t stage = 7u) {
    const uint32_t sh = wave_sum(k.shadow), ne = wave_sum(k.nearest), ce = wave_sum(k.cells);
    const uint32_t pr = wave_sum(primary);
    if ((threadIdx.x & 63) == 0) {
        unsigned long long* c = ctr + kCtrWords * ((blockIdx.x * 4u + (threadIdx.x >> 6)) & (kCtrStripes - 1u));
        if (sh) atomicAdd(&c[0], (unsigned long long)sh);
        if (ne) atomicAdd(&c[1], (unsigned long long)ne);
        if (ce) {
            atomicAdd(&c[2], (unsigned long long)ce);
            atomicAdd(&c[8 + stage], (unsigned long long)ce);
        }
        if (pr) atomicAdd(&c[3], (unsigned long long)pr);
    }
}

// The tile (logical block) a workgroup of the walking kernels takes.  Workgroups are dealt
// round-robin to the 8 XCDs (blocks b and b + 8 share one, MI355X_MICROARCH.md "Workgroup
// dispatch"), so consecutive tiles land in 8 different L2s.  Launches of more than
// kXcdBigTiles tiles (C3 / C4 at 3840x2160: 32400) deal runs of kXcdRunBig consecutive tiles
// to each XCD, the runs round-robin: block b = 8k + x takes tile ((k / R) * 8 + x) * R + k % R
// (the last partial round keeps t = b).  8-tile strips per XCD measured C3 5.61 -> 5.52 ms
// (runs of 4: 5.62, of 30 — a column band per XCD — 10.1).  C1-sized launches keep t = b
// (runs of 8: 0.705 -> 0.716 ms; runs of 2 / 4 within noise; a contiguous band per XCD:
// primary 0.46 -> 0.80 ms — the image's cost is spatially uneven, most XCDs idled).
// A permutation of the tiles: any kernel may use it or not.
constexpr uint32_t kXcdRunBig = 8;
constexpr uint32_t kXcdBigTiles = 16384;
__device__ __forceinline__ uint32_t tile_block() {
    if (gridDim.x > kXcdBigTiles) {
        constexpr uint32_t R = kXcdRunBig;
        const uint32_t b = blockIdx.x, full = (gridDim.x / (8u * R)) * 8u * R;
        if (b >= full) return b;
        const uint32_t x = b & 7u, k = b >> 3;
        return ((k / R) * 8u + x) * R + k % R;
    }
    return blockIdx.x;
}

// ------------------------------------------------------------------- stage 2
// Slot bookkeeping: a shadow slot's validity is the path's smask bit (written by every shade
// for every path), so a rejected area-light sample writes no slot and resolve does not
// re-zero the SM word (every shade rewrites it before the next resolve reads it).  The fused
// tails (k_shadow_finish, k_frame0) keep the tile's occluded flags in an LDS bitmap and hand
// the last level's light sum from resolve to finish in registers.
__device__ __forceinline__ void put_slot(const WaveBufs& w, uint32_t s, uint32_t p, f3 o, f3 d, float tmax, f3 val,
                                         uint32_t fl) {
    const uint64_t i = (uint64_t)s * w.P + p;
    w.SO[i] = make_float4(o.x, o.y, o.z, tmax);
    w.SD[i] = make_float4(d.x, d.y, d.z, __uint_as_float(fl));
    w.SL[i] = make_float4(val.x, val.y, val.z, 0.f);
}

// Light keys of the shadow-list buckets (the light index modulo this): a tile's shadow rays
// are walked grouped by the light they go to, so a wave's lanes head the same way and read
// the same distance-field words.
constexpr uint32_t kLightKeys = 16;
constexpr uint32_t kSlotBits = 0x7fffu;  // smask: slots 0..14 (area_samples <= 15)

// Renderer::Illumination (renderer.cpp:738-764) up to the IsOccluded calls: draws the
// light index (and the area-light sample directions), computes each shadow ray exactly as
// the evaluators build it, and the contribution it adds when unoccluded.  Returns the
// pending-light word; discard = the smoke player probe (result thrown away).
__device__ __forceinline__ uint32_t emit_illumination(const SceneView& sv, const Ray& r, Rng& g, const WaveBufs& w,
                                                      uint32_t p, bool discard, f3& kd_out, uint32_t& slots) {
    const uint64_t pc = sv.num_points, scn = sv.num_spots, ac = sv.num_areas;
    const uint64_t lc = pc + scn + ac + 1;
    const uint64_t idx = (uint64_t)(g.next() * (float)lc);
    const f3 ip = ray_point(r);
    const f3 n = r.N;
    const f3 kd = albedo(sv, r.mat);
    kd_out = kd;
    const uint32_t extra = discard ? kSlotDiscard : 0u;
    uint32_t kind = kLightSingle, count = 0;
    if (idx < pc) {  // PointLightEvaluate :102-131
        const vpx_point_light& l = sv.points[idx];
        const f3 dir = ld3(l.position) - ip;
        const float dst = length(dir);
        const f3 dn = dir * (1.0f / dst);
        const float c = dot(dn, n);
        if (!(c <= 0.0f)) {
            const f3 li = (ld3(l.color) * smax(0.0f, c)) * (1.0f / (dst * dst));
            const Ray sh = make_ray(offset_ray(ip, n), dn);
            put_slot(w, 0, p, sh.O, sh.D, dst, li * kd, kSlotValid | extra);
            count = 1;
            slots |= 1u;
        }
    } else if (idx < ac + pc) {  // AreaLightEvaluation :161-207
        const vpx_area_light& l = sv.areas[idx - pc];
        const f3 center = ld3(l.position);
        const float radius = l.radius;
        const f3 point = offset_ray(ip, n);
        kind = kLightArea;
        count = (uint32_t)sv.area_samples;
        for (int i = 0; i < sv.area_samples; ++i) {  // count <= 15 slots (API caps area_samples)
            f3 rp = random_direction(g);
            rp = rp * radius;
            rp = rp + center;
            const f3 dir = rp - ip;
            const float dst = length(dir);
            const f3 dn = dir * (1.0f / dst);
            const float c = dot(dn, n);
            if (c <= 0) continue;  // rejected: no shadow ray (its smask bit stays clear, nothing written)
            f3 li = ld3(l.color) * c;
            li = li * l.color_multiplier;
            li = li * (radius * radius);
            li = li * kPi;
            li = li * 4.0f;
            li = li / (dst * dst);
            const Ray sh = make_ray(point, dn);
            put_slot(w, i, p, sh.O, sh.D, dst, li, kSlotValid | extra);
            slots |= 1u << i;
        }
    } else if (idx < ac + scn + pc) {  // SpotLightEvaluate :133-159
        const vpx_spot_light& l = sv.spots[idx - ac - pc];
        const f3 dir = ld3(l.position) - ip;
        const float dst = length(dir);
        const f3 dn = dir / dst;
        const float c = dot(dn, ld3(l.direction));
        if (!(c <= l.angle)) {
            const float alpha = 1.0f - ((1.0f - c) * 1.0f) / (1.0f - l.angle);
            const f3 li = (ld3(l.color) * smax(0.0f, c)) / (dst * dst);
            const Ray sh = make_ray(offset_ray(ip, n), dn);
            put_slot(w, 0, p, sh.O, sh.D, dst, (li * kd) * alpha, kSlotValid | extra);
            count = 1;
            slots |= 1u;
        }
    } else {  // DirectionalLightEvaluate :315-338
        const f3 dir = -ld3(sv.dir.direction);
        const float c = dot(dir, n);
        if (!(c <= 0)) {
            const f3 li = ld3(sv.dir.color) * smax(0.0f, c);
            const Ray sh = make_ray(offset_ray(ip, n), dir);
            put_slot(w, 0, p, sh.O, sh.D, kBig, li * kd, kSlotValid | extra);
            count = 1;
            slots |= 1u;
        }
    }
    // every slot of this call goes to light `idx`: the tile's shadow list is bucketed by it
    if (slots) slots |= ((uint32_t)idx & (kLightKeys - 1u)) << 16;
    return kind | (discard ? 8u : 0u) | (count << 4) | ((uint32_t)lc << 16);
}

// One Trace level of the material switch (renderer.cpp:1100-1327) for an active path.
// Exclusive wave prefix sum (inclusive scan by shuffles, minus self).
// DPP form (no lane-address registers, see wave_sum): an inclusive scan inside each row of
// 16 lanes by row shifts of 1, 2, 4, 8 (lanes shifted in from outside the row read 0), then
// the rows' totals carried by row_bcast:15 (into rows 1 and 3) and row_bcast:31 (rows 2, 3).
// Needs the whole wave active (every caller runs it in uniform control flow).
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ uint32_t dpp_add(uint32_t x) {
    return x + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xf, true);
}
__device__ __forceinline__ uint32_t wave_prefix(uint32_t v, uint32_t& total) {
    uint32_t x = v;
    x = dpp_add<0x111>(x);        // row_shr:1
    x = dpp_add<0x112>(x);        // row_shr:2
    x = dpp_add<0x114>(x);        // row_shr:4
    x = dpp_add<0x118>(x);        // row_shr:8
    x = dpp_add<0x142, 0xa>(x);   // row_bcast:15
    x = dpp_add<0x143, 0xc>(x);   // row_bcast:31
    total = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
    return x - v;
}

// Order a wave's LDS / global writes before its lanes read each other's (the wave-local
// counterpart of __syncthreads: the same workgroup-scope release / acquire, no s_barrier).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// L0: the call shades level 0 (the fused head in k_primary).  Level 0 rays are primary
// rays, which never start inside glass or smoke, so the interior exit marches (a whole DDA
// walker each) drop out of that instance; the forms word is known (no levels yet).
// Returns whether the path traces a next ray (the bounce pool's mask bit).
template <bool L0 = false>
__device__ __forceinline__ bool shade_path(const SceneView& sv, const FrameArgs& f, const WaveBufs& w,
                                           const PathRay& pr, uint32_t p, int level, Counters& k) {
    uint32_t slots = 0;
    bool cont = false;
    if (p < w.P) {
        float4 od = pr.D[pr.at(p)];
        uint32_t flags = __float_as_uint(od.w);
        uint32_t pending = 0;  // SM word; 0 = no light sample this level
        if (flags & kActive) {
            const float4 oo = pr.O[pr.at(p)];
            const float4 hh = pr.H[pr.at(p)];
            const uint32_t hm = pr.HM[pr.at(p)];
            Ray ray;
            ray.O = mk(oo.x, oo.y, oo.z);
            ray.D = mk(od.x, od.y, od.z);
            ray.t = hh.x;
            ray.N = mk(hh.y, hh.z, hh.w);
            ray.mat = hm & 0xffu;
            ray.inside = L0 ? false : (hm & 0x80000000u) != 0u;
            if ((f.flags & kFlagReproject) && level == 0) {  // RayDataReproject::GetRayInfo (renderer.h:31-34)
                uint32_t x, y;
                if (path_pixel_single(f, p, x, y)) {
                    const f3 ip = ray_point(ray);
                    w.RD[(uint64_t)y * f.width + x] = make_float4(ip.x, ip.y, ip.z, __uint_as_float(ray.mat));
                }
            }
            const int32_t vox = (int32_t)((hm >> 8) & 0xffffu) - 2;
            Rng g{__float_as_uint(oo.w)};
            int depth = L0 ? f.max_bounces : w.depth[p];  // the fused head's k_primary writes no depth
            // a path being shaded at `level` has recorded exactly `level` forms
            uint32_t forms = (L0 || level == 0) ? 1u : w.forms[p];
            const uint32_t nl = forms_count(forms);
            bool done = false;
            f3 leaf = mk(0.f, 0.f, 0.f);
            if (ray.mat == kNone) {  // SampleSky, :1092-1095
                leaf = sample_sky(sv, ray.D);
                done = true;
            } else if (ray.mat == VPX_MAT_EMISSIVE) {  // :1315-1316
                leaf = albedo(sv, ray.mat) * sv.materials[ray.mat].emissive;
                done = true;
            } else {
                const uint32_t m = ray.mat;
                const vpx_material& mat = sv.materials[m];
                f3 a = mk(1.f, 1.f, 1.f);
                uint32_t form;
                Ray next;
                f3 kd;
                if (m >= VPX_MAT_METAL_HIGH && m <= VPX_MAT_METAL_LOW) {  // :1103-1114
                    const f3 refl = reflect(ray.D, ray.N);
                    const f3 o = offset_ray(ray_point(ray), ray.N);
                    next = make_ray(o, refl + random_sphere_sample(g) * mat.roughness);
                    a = albedo(sv, m);
                    form = kFormMul;
                } else if (m <= VPX_MAT_NON_METAL_PINK && (f.flags & kFlagReproject)) {
                    // TraceNonMetal (renderer.cpp:1343-1357): no Schlick branch; Lambertian
                    // direction first, then Illumination; albedo * ((0 + incLight) + child)
                    const f3 rdir = ray.N + random_sphere_sample(g);
                    pending = emit_illumination(sv, ray, g, w, p, false, kd, slots);
                    if (pending) pending |= kPendZeroAdd;
                    next = make_ray(offset_ray(ray_point(ray), ray.N), rdir);
                    a = albedo(sv, m);
                    form = kFormAddMul;
                } else if (m <= VPX_MAT_NON_METAL_PINK) {  // :1117-1144
                    if (g.next() > schlick_nonmetal(dot(-ray.D, ray.N))) {
                        const f3 rdir = ray.N + random_sphere_sample(g);
                        pending = emit_illumination(sv, ray, g, w, p, false, kd, slots);
                        next = make_ray(offset_ray(ray_point(ray), ray.N), rdir);
                        a = albedo(sv, m);
                        form = kFormMulAdd;
                    } else {
                        const f3 refl = reflect(ray.D, ray.N);
                        const f3 o = offset_ray(ray_point(ray), ray.N);
                        next = make_ray(o, refl + random_sphere_sample(g) * mat.roughness);
                        form = kFormPass;
                    }
                } else if (m == VPX_MAT_GLASS) {  // :1146-1209
                    bool in_glass = ray.inside;
                    const float ior = mat.ior;
                    const float ratio = in_glass ? ior : 1.0f / ior;
                    bool inside_volume = true;
                    if (in_glass) {
                        a = albedo(sv, m);
                        if (vox >= 0) inside_volume = exit_march<kGlassExit>(sv, ray, vox, k);
                    }
                    if (!inside_volume) {
                        ray.O = ray.O + ray.D * ray.t;
                        ray.t = 0;
                    }
                    const float c = smin(dot(-ray.D, ray.N), 1.0f);
                    const float s = sqrtf(1.0f - c * c);
                    const bool cannot = ratio * s > 1.0f;
                    f3 rdir, rn;
                    if (cannot || schlick(c, ratio) > g.next()) {
                        rdir = reflect(ray.D, ray.N);
                        rn = ray.N;
                    } else {
                        rdir = refract(ray.D, ray.N, ratio);
                        in_glass = !in_glass;
                        rn = -ray.N;
                    }
                    next = make_ray(offset_ray(ray_point(ray), rn), rdir);
                    next.inside = in_glass;
                    form = kFormMul;
                } else if (m <= VPX_MAT_SMOKE_PLAYER) {  // smoke :1210-1314
                    f3 color = mk(1.f, 1.f, 1.f);
                    const bool in_glass = ray.inside;
                    bool inside_volume = true;
                    float intensity = 0.f, dist = 0.f;
                    if (vox == 0) {  // player light probe :1228-1240 (rays cast, result unused)
                        pending = emit_illumination(sv, ray, g, w, p, true, kd, slots);
                    }
                    if (in_glass) {
                        intensity = mat.emissive;
                        color = albedo(sv, m);
                        if (vox >= 0) inside_volume = exit_march<kSmokeExit>(sv, ray, vox, k);
                        dist = ray.t;
                    }
                    const float threshold = g.next() * 100.0f - intensity;
                    if (g.next() * dist > threshold) {
                        const float lo = ray.t * .45f, hi = ray.t;
                        const float tt = lo + g.next() * (hi - lo);
                        ray.O = ray.O + ray.D * tt;
                        ray.D = random_direction(g);
                        ray.t = 0;
                    }
                    const f3 flipped = mk(1.f, 1.f, 1.f) - color;
                    const f3 e = flipped * ((-dist) * intensity);
                    a = mk(cr_exp(e.x), cr_exp(e.y), cr_exp(e.z));
                    if (!inside_volume) {
                        ray.O = ray.O + ray.D * ray.t;
                        ray.t = 0;
                    }
                    const f3 rdir = refract(ray.D, ray.N, 1.0f);
                    next = make_ray(offset_ray(ray_point(ray), -ray.N), rdir);
                    next.inside = !in_glass;
                    form = kFormMul;
                } else {  // model materials :1319-1326
                    const f3 rdir = diffuse_reflection(g, ray.N);
                    pending = emit_illumination(sv, ray, g, w, p, false, kd, slots);
                    next = make_ray(offset_ray(ray_point(ray), ray.N), rdir);
                    a = albedo(sv, m);
                    form = kFormAddMul;
                }
                // LB is read by k_finish only for the MulAdd / AddMul forms, and those
                // levels always carry a pending light whose k_resolve writes LB: no zero fill
                const uint64_t li = (uint64_t)nl * w.P + p;
                w.LA[li] = make_float4(a.x, a.y, a.z, 0.f);
                forms = (forms ^ (1u << (2 * nl))) | (form << (2 * nl)) | (1u << (2 * nl + 2));
                if (pending) {
                    pending |= (nl << 8);
                    w.SM[p] = make_float4(kd.x, kd.y, kd.z, __uint_as_float(pending));
                }
                --depth;
                if (depth >= 0) {
                    flags = (next.inside ? kInside : 0u) | kActive;
                    w.O[p] = make_float4(next.O.x, next.O.y, next.O.z, __uint_as_float(g.s));
                    w.D[p] = make_float4(next.D.x, next.D.y, next.D.z, __uint_as_float(flags));
                    w.depth[p] = depth;
                    cont = true;
                }
                // else: the child Trace(depth < 0) returns 0 (the leaf k_primary zeroed).
                // Only the last level gets here (depth starts at max_bounces) and no kernel
                // after it reads the path's ray, flags or depth, so they are not written.
                w.forms[p] = forms;
            }
            if (done) {  // sky / emissive leaf; the path stops
                w.leaf[p] = make_float4(leaf.x, leaf.y, leaf.z, 0.f);
                w.forms[p] = forms | kLeafBit;
                // later levels' kernels skip it (after the last level no kernel reads D)
                if (level < f.max_bounces) w.D[p] = make_float4(od.x, od.y, od.z, __uint_as_float(0u));
            }
        }
        if (!pending) w.SM[p] = make_float4(0.f, 0.f, 0.f, __uint_as_float(0u));
    }
    if (p < w.P) w.smask[p] = slots;
    return cont;
}

__device__ __forceinline__ uint32_t lane_rank(uint64_t m) {  // set bits of m below this lane
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// Whether the path at list position i (level 0: the path i itself) traces a next ray: bit
// i & 63 of amask word i >> 6, one ballot per wave (its lanes hold consecutive positions, no
// atomics).  k_compact turns the bits into the next level's list.  (Appending each wave's
// paths to the list with one atomic per wave serialised on the shared count: Z1's level-0
// head 0.21 -> 0.41 ms, C2's shades 0.057 -> 0.132 ms.)
__device__ __forceinline__ void put_amask(const WaveBufs& w, uint32_t i, bool cont) {
    const uint64_t b = __ballot(cont);
    if ((threadIdx.x & 63u) == 0 && i < w.P) w.amask[i >> 6] = b;
}

// Level l >= 1's material switch over its live list: the launch is sized for the largest list
// (the count is on the device), workgroups past the list's end return at once (a grid-stride
// loop kept more registers live: 113 VGPRs and scratch instead of 90).
__global__ __launch_bounds__(256) void k_shade(SceneView sv, FrameArgs f, WaveBufs w, int level,
                                               unsigned long long* ctr) {
    Counters k{0u, 0u, 0u};
    const uint32_t n = live_count(w, level);
    if (blockIdx.x * 256u >= n) return;
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const uint32_t p = i < n ? live_path(w, level, i) : ~0u;  // ~0u: shade_path does nothing
    const bool cont = shade_path(sv, f, w, PathRay{w.O, w.D, w.H, w.HM, 0u}, p, level, k);
    if (level < f.max_bounces) put_amask(w, i, cont);
    flush_counters(k, 0u, ctr, VPX_STAGE_SHADE);
}

// Light sum of a level once its shadow rays are resolved (kSlotOcc set by k_shadow1):
// the evaluators' accumulation (renderer.cpp:102-207) and Illumination's *lightCount.
// occ (fused tails): the tile's occluded bits in LDS, bit s * 256 + (p & 255);
// out: the light sum and its level are returned instead of written to LB (the caller's
// finish_path takes them), out->lvl = ~0u when the path has none.
struct LightSum {
    uint32_t lvl;
    f3 inc;
};
// is_occ(s, i): whether slot s (element i of the slot arrays) was occluded.
template <class OccFn>
__device__ __forceinline__ void resolve_path_by(const SceneView& sv, const WaveBufs& w, uint32_t p, OccFn is_occ,
                                                LightSum* out) {
    if (out) out->lvl = ~0u;
    if (p >= w.P) return;
    const float4 sm = w.SM[p];
    const uint32_t pend = __float_as_uint(sm.w);
    if (!pend) return;
    const uint32_t kind = pend & 7u, count = (pend >> 4) & 15u, lvl = (pend >> 8) & 31u, lc = pend >> 16;
    if (pend & 8u) return;  // discarded probe
    const uint32_t valid = w.smask[p];
    f3 acc = mk(0.f, 0.f, 0.f);
    for (uint32_t s = 0; s < count; ++s) {
        const uint64_t i = (uint64_t)s * w.P + p;
        if (!((valid >> s) & 1u)) continue;
        if (is_occ(s, i)) continue;
        const float4 v = w.SL[i];
        if (kind == kLightArea)
            acc = acc + mk(v.x, v.y, v.z);
        else
            acc = mk(v.x, v.y, v.z);
    }
    f3 inc = acc;
    if (kind == kLightArea) inc = (acc / (float)sv.area_samples) * mk(sm.x, sm.y, sm.z);
    inc = inc * (float)lc;
    if (pend & kPendZeroAdd) inc = mk(0.f, 0.f, 0.f) + inc;
    if (out) {
        out->lvl = lvl;
        out->inc = inc;
    } else {
        w.LB[(uint64_t)lvl * w.P + p] = make_float4(inc.x, inc.y, inc.z, 0.f);
    }
}
// occ (fused tails): the tile's LDS bitmap, bit s * 256 + (p & 255); else the shadow pool's
// occb bytes, else the tile kernels' kSlotOcc bit in the slot's SD word.
__device__ __forceinline__ void resolve_path(const SceneView& sv, const WaveBufs& w, uint32_t p,
                                             const uint32_t* occ = nullptr, LightSum* out = nullptr) {
    resolve_path_by(
        sv, w, p,
        [&](uint32_t s, uint64_t i) -> bool {
            const uint32_t b = s * 256u + (p & 255u);
            return occ ? (occ[b >> 5] >> (b & 31u)) & 1u
                       : w.occb ? (uint32_t)w.occb[i] : __float_as_uint(w.SD[i].w) & 4u /* kSlotOcc */;
        },
        out);
}

__global__ __launch_bounds__(256) void k_resolve(SceneView sv, WaveBufs w, int level) {
    const uint32_t n = live_count(w, level);
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u)
        resolve_path(sv, w, live_path(w, level, i));
}

// ------------------------------------------------------------ tile kernels
// Minimum waves per SIMD requested for the DDA kernels (caps their VGPRs: the walks are
// bound by dependent mask loads, so residency matters more than a few spilled values).
// Measured (ms, C1 / C3): 4 -> 0.927 / 7.66, 5 -> 0.899 / 7.22, 6 -> 0.898 / 7.03.
#ifndef VPX_WPE_NEAREST
#define VPX_WPE_NEAREST 6
#endif
// The bounce pool (k_nearest_pool) at 5 (96 VGPRs, no spills): C2 2.62 / 2.64 vs 2.67 / 2.68 ms
// at 6 (4 spills), 7: 2.78 / 2.82.
#ifndef VPX_WPE_BOUNCE
#define VPX_WPE_BOUNCE 5
#endif
// Shadow kernels (k_shadow_tile, k_shadow_finish) at 7 with the octant planes (13 spilled
// VGPRs): C3 5.68 -> 5.60 ms, C2 unchanged; 8 measured 6.03 / 4.51.
#ifndef VPX_WPE_SHADOW
#define VPX_WPE_SHADOW 7
#endif
// The multi-volume / shape instances (C4) carry the volume loop's state across the walks:
// at 6 waves/SIMD they spilled 45-53 VGPRs.  Measured C4 (ms, FindNearest / IsOccluded
// stages): 6 -> 2.98 / 2.50, 5 -> 2.13 / 2.40, 4 (no spills) -> 1.72 / 2.59.
#ifndef VPX_WPE_MULTI_NEAREST
#define VPX_WPE_MULTI_NEAREST 4
#endif
// The multi-volume shadow kernels (k_shadow_tile<false>, k_shadow_finish<false>; round 4 also k_shadow_inst)
// at 6 (80 VGPRs, 15-18 spilled): C4 42.91 / 42.60 / 42.84 vs 43.18 / 42.94 / 44.99 ms at 5,
// Z1 within noise (round 4, tools/gpu_r4n.sh); k_nearest_tile at 5 (49 spilled VGPRs): Z1
// 2.66 vs 2.50-2.52.
#ifndef VPX_WPE_MULTI_SHADOW
#define VPX_WPE_MULTI_SHADOW 6
#endif

#define VPX_WPE(n) __attribute__((amdgpu_waves_per_eu(n)))

// The multi-volume kernels read the instance TLAS nodes with scalar loads (the traversal is
// wave-uniform); staging them in LDS measured slower (C4 FindNearest 1.70 vs 1.68 ms,
// IsOccluded 2.81 vs 2.68).

// One 256-thread workgroup per 16x16 tile.  Work is compacted inside the tile through LDS
// (no global atomics), so a DDA wave only carries rays that will actually march, and the
// waves of a sparse tile retire at once.

// Rank of this thread's `cnt` items among the workgroup's (exclusive), and the total.
__device__ __forceinline__ uint32_t block_scan(uint32_t cnt, uint32_t& total, uint32_t* sh) {
    uint32_t wt;
    const uint32_t off = wave_prefix(cnt, wt);
    const uint32_t wid = threadIdx.x >> 6;
    if ((threadIdx.x & 63u) == 0) sh[wid] = wt;
    __syncthreads();
    uint32_t base = 0;
    total = 0;
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
        const uint32_t v = sh[i];
        base += i < wid ? v : 0u;
        total += v;
    }
    __syncthreads();
    return base + off;
}

template <uint32_t SKIPW = kSkipwNearest, uint32_t MINC = kMincNearest, uint32_t RUN = kRunNearest>
__device__ __forceinline__ void nearest_record(SceneView sv, const PathRay& pr, uint32_t p, Ray& r, Counters& k) {
    r.t = kBig;
    r.mat = kNone;
    r.N = mk(0.f, 0.f, 0.f);
    const int32_t vox = find_nearest<SKIPW, MINC, RUN>(sv, r, k);
    pr.H[pr.at(p)] = make_float4(r.t, r.N.x, r.N.y, r.N.z);
    pr.HM[pr.at(p)] = r.mat | ((uint32_t)(vox + 2) << 8) | (r.inside ? 0x80000000u : 0u);
}

// Object-space ray of path p in the single volume (FindNearest's SSE transforms).
__device__ __forceinline__ ORay path_oray(const vpx_volume& vol, const PathRay& pr, uint32_t p,
                                          const X86Arith& xa = X86Arith{}) {
    const float4 o = pr.O[pr.at(p)], d = pr.D[pr.at(p)];
    ORay r;
    r.O = xform_pos_ssem(mk(o.x, o.y, o.z), vol.inv_matrix);
    r.D = xform_vec_ssem(mk(d.x, d.y, d.z), vol.inv_matrix);
    r.rD = nearest_rd(r.D, xa);
    return r;
}

// nearest_record for the single-volume, shape-free scene: the same result, but only the
// walk state lives across the walk — the ray is read back from the path buffers and
// transformed again for the normal (the same operations, so the same values), which
// keeps the walker's registers from spilling.
// Its two halves (walk continuations, k_nearest_tile): the walk state of path p's ray
// (false: Setup3DDDA fails, no cell is read) and the hit record from the finished walk.
__device__ __forceinline__ bool nearest_begin_v(const vpx_volume& vol, uint32_t n, const PathRay& w, uint32_t p,
                                                Counters& k, skip::Walk& wk, const X86Arith& xa) {
    ++k.nearest;
    const ORay o = path_oray(vol, w, p, xa);
    Dda s;
    if (!dda_setup(vol, n, o, s)) return false;
    wk = to_walk(s);
    return true;
}
__device__ __forceinline__ bool nearest_begin_1v(const SceneView& sv, const PathRay& w, uint32_t p, Counters& k,
                                                 skip::Walk& wk) {
    const vpx_volume* vol = uni_ptr(&sv.volumes[0]);
    return nearest_begin_v(*vol, sv.grids[vol->grid_id].n, w, p, k, wk, sv.x86);
}
__device__ __forceinline__ void nearest_end_v(const vpx_volume& vol, const uint8_t* cells, uint32_t n, const PathRay& w,
                                              uint32_t p, const skip::Walk& wk, bool hit);
__device__ __forceinline__ void nearest_end_1v(const SceneView& sv, const PathRay& w, uint32_t p, const skip::Walk& wk,
                                               bool hit) {
    const vpx_volume* vol = uni_ptr(&sv.volumes[0]);
    const DevGrid g = sv.grids[vol->grid_id];
    nearest_end_v(*vol, g.cells, g.n, w, p, wk, hit);
}

template <uint32_t SKIPW = kSkipwNearest, uint32_t MINC = kMincNearest, uint32_t RUN = kRunNearest>
__device__ __forceinline__ void nearest_record_1v(const SceneView& sv, const PathRay& w, uint32_t p, Counters& k) {
    bool hit = false;
    skip::Walk wk;
    if (nearest_begin_1v(sv, w, p, k, wk))
        hit = walk_wave<0, SKIPW, MINC, RUN>(grid_view(sv.grids[uni_ptr(&sv.volumes[0])->grid_id]), wk, kBig, k.cells);
    nearest_end_1v(sv, w, p, wk, hit);
}

__device__ __forceinline__ void nearest_end_v(const vpx_volume& vol, const uint8_t* cells, uint32_t n, const PathRay& w,
                                              uint32_t p, const skip::Walk& wk, bool hit) {
    asm volatile("" ::: "memory");  // re-read the ray below instead of keeping it live
    const uint32_t inside = __float_as_uint(w.D[w.at(p)].w) & kInside ? 0x80000000u : 0u;
    if (!hit) {
        w.H[w.at(p)] = make_float4(kBig, 0.f, 0.f, 0.f);
        w.HM[w.at(p)] = kNone | inside;  // vox -2
        return;
    }
    const ORay o = path_oray(vol, w, p);
    const f3 N = normal_voxel(o, wk.t, n, vol.matrix);
    const uint32_t mat = cells[(uint64_t)wk.X + (uint64_t)wk.Y * n + (uint64_t)wk.Z * ((uint64_t)n * n)];
    w.H[w.at(p)] = make_float4(wk.t, N.x, N.y, N.z);
    w.HM[w.at(p)] = mat | (2u << 8) | inside;  // vox 0
}

// Primary rays + Renderer::FindNearest.  Every path's ray / RNG state is written; rays
// that cannot hit a voxel or shape (one volume, no shapes, Setup3DDDA fails: the
// reference returns before reading a cell) get their miss record directly.
// SHADE: the fused head keeps the tile's rays and hit records in LDS (its walkers and its
// level-0 shade are the only readers).  Ordering the tile's walkers by their pixel's walk
// length in the previous frame measured faster per wave but not per tile (C1 0.697-0.704 vs
// 0.712-0.715 ms with, C3 5.43 vs 5.54 — a tile costs its longest walk) and adds a
// frame-to-frame dependency, so walkers run in pixel order.
// The head's LDS: the compacted walker list, and with SHADE the tile's rays (O, D, H) and hit
// records.  Declared by the kernel, so that k_frame0 can hand the regions on to its tail once
// the head is done with them.
template <bool SHADE>
struct HeadLds {
    uint32_t sh[4];
    uint32_t lst[256];
    float4 ray[SHADE ? 3 * 256 : 1];
    uint32_t hm[SHADE ? 256 : 1];
};

// Whether FindNearest may still find something after volume 0 for a ray whose world walk
// ended at t: the TLAS root box within its segment [0, t] (conservative, tlas_box), or always
// when there are shapes, volumes outside the tree or no TLAS (the instance pass's candidates).
__device__ __forceinline__ bool meets_later_volume(const SceneView& sv, f3 o, f3 d, float t) {
    if (!(sv.tlas_on && !sv.tlas_always && !(sv.num_spheres | sv.num_triangles) && sv.tlas_nodes)) return true;
    return tlas_box(sv.tlas[0], o, world_inv(d), t);
}

// DEFER (multi-volume scenes without shapes at Trace depth 0, the head of k_instances_list):
// after the world walk a path whose ray cannot meet a later volume (meets_later_volume) is
// final — the head shades it from its LDS records like a single-volume head; the others are
// written to HBM and flagged in amask (one ballot word per wave, unused at depth 0) for the
// instance pass, which continues FindNearest and shades only them.  C4: ~15 % of the primary
// rays reach the instance lattice's box.
template <bool ONE, bool SHADE, uint32_t RUN = kRunNearest, bool DEFER = false>
__device__ __forceinline__ void primary_tile(const SceneView& sv, const FrameArgs& f, const WaveBufs& w,
                                             HeadLds<SHADE>& L, unsigned long long* __restrict__ ctr) {
    uint32_t* sh = L.sh;
    uint32_t* lst = L.lst;
    const uint32_t tb = tile_block() * 256u;
    const uint32_t p = tb + threadIdx.x;
    const PathRay pr = SHADE ? PathRay{L.ray, L.ray + 256, L.ray + 512, L.hm, tb} : PathRay{w.O, w.D, w.H, w.HM, 0u};
    Counters k{0u, 0u, 0u};
    uint32_t prim = 0;
    bool walk = false;
    if (p < w.P) {
        uint32_t x, y;
        bool go = path_pixel(f, p, x, y);
        if (!SHADE) {  // the fused shade writes depth (paths that continue) and forms itself
            w.depth[p] = f.max_bounces;
            w.forms[p] = 1u;  // no levels recorded, no leaf
        }
        Ray r;
        r.O = r.D = mk(0.f, 0.f, 0.f);
        uint32_t rng = 0, flags = 0;
        if (go) {
            Rng g{pixel_seed(f.seed_base, path_frame(f, p), f.width, f.height, x, y)};
            r = primary_ray(f, x, y, g, sv.x86);
            rng = g.s;
            prim = 1;
            flags = kActive;
        }
        if (f.max_bounces < 0) {  // Trace(ray, -1) returns 0 without a lookup
            go = false;
            flags = 0u;
        }
        pr.O[pr.at(p)] = make_float4(r.O.x, r.O.y, r.O.z, __uint_as_float(rng));
        pr.D[pr.at(p)] = make_float4(r.D.x, r.D.y, r.D.z, __uint_as_float(flags));
        // an inactive path (no pixel) must read as such in the later levels' kernels
        if (SHADE && !flags && f.max_bounces > 0) w.D[p] = make_float4(0.f, 0.f, 0.f, __uint_as_float(0u));
        if (go) {
            walk = true;
            if (ONE) {
                const vpx_volume& vol = sv.volumes[0];
                ORay o;
                o.O = xform_pos_ssem(r.O, vol.inv_matrix);
                o.D = xform_vec_ssem(r.D, vol.inv_matrix);
                o.rD = nearest_rd(o.D, sv.x86);
                Dda s;
                if (!dda_setup(vol, sv.grids[vol.grid_id].n, o, s)) {
                    walk = false;
                    ++k.nearest;
                    pr.H[pr.at(p)] = make_float4(kBig, 0.f, 0.f, 0.f);
                    pr.HM[pr.at(p)] = kNone;  // vox -2, not inside glass
                }
            }
        }
    }
    uint32_t total;
    const uint32_t at = block_scan(walk ? 1u : 0u, total, sh);  // (its barrier orders the LDS writes)
    if (walk) lst[at] = p;
    __syncthreads();
    if (threadIdx.x < total) {
        const uint32_t q = lst[threadIdx.x];
        if (ONE) {
            nearest_record_1v<kSkipwNearest, kMincNearest, RUN>(sv, pr, q, k);
        } else {
            const float4 o = pr.O[pr.at(q)], d = pr.D[pr.at(q)];
            Ray r;
            r.O = mk(o.x, o.y, o.z);
            r.D = mk(d.x, d.y, d.z);
            r.inside = false;
            nearest_record(sv, pr, q, r, k);
        }
    }
    flush_counters(k, prim, ctr, VPX_STAGE_PRIMARY);
    if (SHADE) {  // level 0's material switch for this thread's own path (k_primary_shade)
        __syncthreads();  // the tile's hit records, written by the compacted walkers
        Counters ks{0u, 0u, 0u};
        bool defer = false;
        if (DEFER && p < w.P) {
            const float4 d = pr.D[pr.at(p)];
            if (__float_as_uint(d.w) & kActive) {
                const float4 o = pr.O[pr.at(p)], h = pr.H[pr.at(p)];
                defer = meets_later_volume(sv, mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), h.x);
                if (defer) {  // the instance pass reads the ray and the world's hit record
                    w.O[p] = o;
                    w.D[p] = d;
                    w.H[p] = h;
                    w.HM[p] = pr.HM[pr.at(p)];
                }
            }
        }
        if (DEFER) put_amask(w, p, defer);
        const bool cont = defer ? false : shade_path<true>(sv, f, w, pr, p, 0, ks);
        if (!DEFER && f.max_bounces > 0) put_amask(w, p, cont);
        flush_counters(ks, 0u, ctr, VPX_STAGE_SHADE);
    }
}

template <bool ONE, bool SHADE = false, bool X86 = false, bool DEFER = false>
__global__ __launch_bounds__(256) VPX_WPE(ONE ? VPX_WPE_NEAREST : VPX_WPE_MULTI_NEAREST) void k_primary(SceneView sv, FrameArgs f, WaveBufs w,
                                                 unsigned long long* __restrict__ ctr) {
    __shared__ HeadLds<SHADE> L;
    primary_tile<ONE, SHADE, kRunNearest, DEFER>(arith_view<X86>(sv), f, w, L, ctr);
}

// Level l + 1's live list from level l's shade bits: 256 mask words (16 k list positions) per
// workgroup, the words' counts scanned in the workgroup, one atomic per workgroup for its
// place in the list, then each wave writes its words' entries 64 at a time (coalesced).  The
// list order is whatever the workgroups' atomics give; each path's work is independent of its
// place, so results and counts are too.
__global__ __launch_bounds__(256) void k_compact(WaveBufs w, int level) {
    __shared__ uint32_t sh[4];
    __shared__ uint32_t base_s;
    const uint32_t n = live_count(w, level), words = (n + 63u) >> 6;
    if (blockIdx.x * 256u >= words) return;
    const uint32_t wi = blockIdx.x * 256u + threadIdx.x;
    uint64_t m = wi < words ? w.amask[wi] : 0ull;
    if (wi == words - 1u && (n & 63u)) m &= (1ull << (n & 63u)) - 1ull;  // positions past the list
    uint32_t total;
    const uint32_t off = block_scan((uint32_t)__popcll(m), total, sh);
    if (threadIdx.x == 0) base_s = atomicAdd(&w.pool[kPoolLive + level + 1], total);
    __syncthreads();
    const uint32_t base = base_s;
    const uint32_t lane = threadIdx.x & 63u, w0 = blockIdx.x * 256u + (threadIdx.x & ~63u);
    const uint32_t* L = live_list(w, level);
    uint32_t* out = ((level + 1) & 1) ? w.live1 : w.live0;
    for (uint32_t j = 0; j < 64u; ++j) {
        const uint64_t mj = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)m, (int)j) |
                            (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(m >> 32), (int)j) << 32;
        if (!mj) continue;
        const uint32_t oj = (uint32_t)__builtin_amdgcn_readlane((int)off, (int)j);
        if ((mj >> lane) & 1ull) {
            const uint32_t i = (w0 + j) * 64u + lane;
            out[base + oj + lane_rank(mj)] = level ? L[i] : i;
        }
    }
}

// The instance walks (FindNearest in the instance grids, k_instances) take the heads' words:
// skip minimum 1 / 3, two passes and skip weight 2 measured within noise of them (C4 42.31-42.87
// vs 42.39-42.44 ms, two interleaved runs each, round 5).

// Multi-volume primary rays in two launches: the world (volume 0, first in the reference's
// loop) walked by the lean single-volume head (k_primary<true, false>: 6 waves/SIMD, no
// spills) writing the hit records to HBM, then this instance pass: per tile, the paths whose
// ray can still meet a later volume or a shape — the TLAS root box within the ray's segment
// [0, world t], or every active path when there are shapes, instances outside the tree or no
// TLAS — compacted into the first waves, Renderer::FindNearest continued from volume 1
// (find_nearest_rest: the same candidates, order, bounds and counts as the one-launch loop),
// then level 0's shade for every path of the tile.  The one-launch kernel
// (k_primary<false, true>) carried the whole volume loop's state through the world walk (112
// VGPRs, 72 spilled SGPRs, 4 waves/SIMD), and every ray of the frame through the instance
// loop: C4's primary stage took 1.46 ms against 0.59 ms for the world alone (tools/c4_split.py).
// Round 5, rejected: the head shading the paths that cannot meet an instance from its LDS
// records and this pass walking and shading only a dense list of the others — C4 43.27-43.35
// vs 42.90-43.09 ms per step (three interleaved runs): most C4 rays are candidates, and the
// pass's HBM traffic is mostly the shade's three area-light slots per pixel (144 B), which the
// shadow pool reads back, not the rays it re-reads.
__global__ __launch_bounds__(256) VPX_WPE(VPX_WPE_MULTI_NEAREST) void k_instances(SceneView sv_, FrameArgs f, WaveBufs w,
                                                                                unsigned long long* __restrict__ ctr) {
    __shared__ uint32_t sh[4];
    __shared__ uint32_t lst[256];
    extern __shared__ uint32_t x86_lds[];  // the rcp table in reference arithmetic (x86_stage_lds)
    SceneView sv = sv_;
    sv.x86 = x86_stage_lds(sv_.x86, x86_lds);
    const uint32_t tb = tile_block() * 256u;
    const uint32_t p = tb + threadIdx.x;
    const PathRay pr{w.O, w.D, w.H, w.HM, 0u};
    Counters k{0u, 0u, 0u};
    bool go = false;
    if (p < w.P && (__float_as_uint(w.D[p].w) & kActive)) {
        const float4 o = w.O[p], d = w.D[p];
        go = meets_later_volume(sv, mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), w.H[p].x);
    }
#ifdef VPX_DEBUG_NO_INST_WALK
    go = false;  // timing probe only (wrong images): the pass without its instance walks
#endif
    uint32_t total;
    const uint32_t at = block_scan(go ? 1u : 0u, total, sh);
    if (go) lst[at] = p;
    __syncthreads();
    if (threadIdx.x < total) {
        const uint32_t q = lst[threadIdx.x];
        const float4 o = w.O[q], d = w.D[q], h = w.H[q];
        const uint32_t hm = w.HM[q];
        Ray r;
        r.O = mk(o.x, o.y, o.z);
        r.D = mk(d.x, d.y, d.z);
        r.t = h.x;
        r.N = mk(h.y, h.z, h.w);
        r.mat = hm & 0xffu;
        r.inside = (hm & 0x80000000u) != 0u;
        int32_t vox = (int32_t)((hm >> 8) & 0xffffu) - 2;
        if (find_nearest_rest(sv, r, k, &vox)) {
            w.H[q] = make_float4(r.t, r.N.x, r.N.y, r.N.z);
            w.HM[q] = r.mat | ((uint32_t)(vox + 2) << 8) | (r.inside ? 0x80000000u : 0u);
        }
    }
    flush_counters(k, 0u, ctr, VPX_STAGE_INSTANCES);
    __syncthreads();  // the tile's hit records, as the compacted lanes left them
    Counters ks{0u, 0u, 0u};
    const bool cont = shade_path<true>(sv, f, w, pr, p, 0, ks);
    if (f.max_bounces > 0) put_amask(w, p, cont);
    flush_counters(ks, 0u, ctr, VPX_STAGE_SHADE);
}

// The deferred instance pass (depth 0, after k_primary<.., DEFER>): the head's amask bits
// turned into live list 1 by k_compact (at Trace depth 0 the level lists are otherwise unused),
// one list entry per lane — FindNearest continued from volume 1, then the path's level-0 shade
// by the same lane, no tile barrier.  The same per-path operations as k_instances.  Per tile
// instead (the deferred ~15 % of a tile's paths in its first wave, the shade after a tile
// barrier): C4 29.77-29.91 vs 28.59-28.65 ms per step (three interleaved runs).
// 4 waves/SIMD (128 VGPRs, 6 spilled): 28.62-28.69 vs 28.91-29.03 ms at 3 (134, none).
#ifndef VPX_WPE_INST_LIST
#define VPX_WPE_INST_LIST VPX_WPE_MULTI_NEAREST
#endif
__global__ __launch_bounds__(256) VPX_WPE(VPX_WPE_INST_LIST) void k_instances_list(SceneView sv_, FrameArgs f, WaveBufs w,
                                                                                     unsigned long long* __restrict__ ctr) {
    extern __shared__ uint32_t x86_lds[];
    const uint32_t n = live_count(w, 1);
    if (blockIdx.x * 256u >= n) return;  // (workgroup-uniform: before the staging barrier; the
                                         // launch is sized for every path)
    SceneView sv = sv_;
    sv.x86 = x86_stage_lds(sv_.x86, x86_lds);
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const PathRay pr{w.O, w.D, w.H, w.HM, 0u};
    Counters k{0u, 0u, 0u}, ks{0u, 0u, 0u};
    if (i < n) {
        const uint32_t q = live_list(w, 1)[i];
        {
            const float4 o = w.O[q], d = w.D[q], h = w.H[q];
            const uint32_t hm = w.HM[q];
            Ray r;
            r.O = mk(o.x, o.y, o.z);
            r.D = mk(d.x, d.y, d.z);
            r.t = h.x;
            r.N = mk(h.y, h.z, h.w);
            r.mat = hm & 0xffu;
            r.inside = (hm & 0x80000000u) != 0u;
            int32_t vox = (int32_t)((hm >> 8) & 0xffffu) - 2;
            if (find_nearest_rest(sv, r, k, &vox)) {
                w.H[q] = make_float4(r.t, r.N.x, r.N.y, r.N.z);
                w.HM[q] = r.mat | ((uint32_t)(vox + 2) << 8) | (r.inside ? 0x80000000u : 0u);
            }
        }
        shade_path<true>(sv, f, w, pr, q, 0, ks);
    }
    flush_counters(k, 0u, ctr, VPX_STAGE_INSTANCES);
    flush_counters(ks, 0u, ctr, VPX_STAGE_SHADE);
}

// Renderer::FindNearest for the active paths of a tile (bounce levels).  Rejected (DESIGN.md
// §4): grouping a tile's walks by direction octant (C2 4.88 vs 4.82 ms), gathering 2 / 4 / 8
// tiles per workgroup (C1 2.87 / 3.22 / 4.36 vs 2.70 ms: walk lengths are heavy-tailed, a
// wave costs its longest ray), continuing a tile's unfinished walks in repacked waves after a
// step budget (C2 4.23-4.37 vs 4.28 ms), and walking the whole frame's bounce rays in the
// order of a counting sort by (direction octant, Morton index of the origin's 16^3-cell
// region): the sorted walker took 553 vs 541 us per level on C2 and the sort 350 us more —
// coherent starts do not shorten the walks, whose cost is their length and step latency.
// Multi-volume / shape scenes (the single-volume scenes walk their bounces in the pool below):
// the next level's live list in chunks of 64 entries (persistent waves, no barriers), so
// every wave is full — a tile's compaction left a deep level's few rays spread
// one or two per wave over the frame's 8100 tiles (Z1: 14 levels, 2 M paths at level 1, 4 k at
// level 14, each launch scanning all 2 M).  `level` is the shade level whose rays it walks.
__global__ __launch_bounds__(256) VPX_WPE(VPX_WPE_MULTI_NEAREST) void k_nearest_tile(SceneView sv_, WaveBufs w, int level,
                                                                                    unsigned long long* __restrict__ ctr) {
    extern __shared__ uint32_t x86_lds[];
    SceneView sv = sv_;
    sv.x86 = x86_stage_lds(sv_.x86, x86_lds);
    Counters k{0u, 0u, 0u};
    const uint32_t n = live_count(w, level + 1);
    const uint32_t lane = threadIdx.x & 63u;
    // one chunk per wave, the launch sized for the longest list (waves past its end return at
    // once): the hardware deals the workgroups as slots free up.  Dynamic grabs from one shared
    // counter serialised (Z1's bounce stage 0.134 -> 0.183 ms); chunks dealt statically to
    // persistent waves balanced the heavy-tailed walks worse (Z1 serial 3.64 vs 3.41 ms).
    {
        const uint32_t g = blockIdx.x * 4u + (threadIdx.x >> 6);
        if (g * 64u >= n) return;
        const uint32_t i = g * 64u + lane;
        if (i < n) {
            const uint32_t q = live_path(w, level + 1, i);
            const float4 o = w.O[q], d = w.D[q];
            Ray r;
            r.O = mk(o.x, o.y, o.z);
            r.D = mk(d.x, d.y, d.z);
            r.inside = (__float_as_uint(d.w) & kInside) != 0u;
            nearest_record<kSkipwBounce, kMincBounce, kRunBounce>(sv, PathRay{w.O, w.D, w.H, w.HM, 0u}, q, r, k);
        }
    }
    flush_counters(k, 0u, ctr, VPX_STAGE_BOUNCE);
}

// The bounce pool (single-volume scenes): Renderer::FindNearest for the level's traced rays,
// walked by persistent waves that refill their finished lanes.  A tile's bounce walks are
// heavy-tailed (C2: of a walk iteration's 64 lanes 16 step, 9 wait to skip and 39 are already
// done), and a tile's ~90 bounce rays leave its second wave mostly empty; here each wave takes
// the next kPoolChunk entries of the level's live list at a time (one global atomic; every
// entry traces a ray — until round 4 a grab was 4 words of a per-path trace mask, ~90 traced
// rays of 256 paths), and hands them to its lanes as lanes free up:
// the walk returns once kPoolLeave lanes have finished, their hit records are written, and new
// rays start in their place while the others keep their walk state.  Every ray is walked by
// exactly the per-lane sequence of nearest_record_1v (same cells, same counts, same records);
// only which lane and when differ.  Waves are independent (no barriers; four per workgroup).
// Measured (C2, ms per step, three interleaved runs each): tile kernel 3.03 / 3.01 / 3.03,
// pool 2.72 / 2.68 / 2.70; 64-thread workgroups 2.83 / 2.82 / 2.77; leave at 8 finished lanes
// 2.75 / 2.73 / 2.74, at 32 2.71 / 2.72 / 2.65; grabs of 2 words 2.84 / 2.77 / 2.82, of 8
// 2.79 / 2.79 / 2.71.
#ifndef VPX_POOL_CHUNK
#define VPX_POOL_CHUNK 128
#endif
#ifndef VPX_POOL_LEAVE
#define VPX_POOL_LEAVE 16
#endif
#ifndef VPX_POOL_WG
#define VPX_POOL_WG 256
#endif
constexpr uint32_t kPoolChunk = VPX_POOL_CHUNK;  // list entries (traced rays) per grab
constexpr uint32_t kPoolLeave = VPX_POOL_LEAVE;  // finished lanes that end a walk while rays are left
constexpr uint32_t kPoolWg = VPX_POOL_WG;        // threads per workgroup (its waves are independent)
template <bool X86>
__global__ __launch_bounds__(kPoolWg) VPX_WPE(VPX_WPE_BOUNCE) void k_nearest_pool(SceneView sv_, WaveBufs w, int level,
                                                                               unsigned long long* __restrict__ ctr) {
    const SceneView sv = arith_view<X86>(sv_);
        const uint32_t n = live_count(w, level + 1);  // the rays level `level`'s shade traced
    const uint32_t* L = live_list(w, level + 1);
    const PathRay pr{w.O, w.D, w.H, w.HM, 0u};
    const skip::GridView gv = grid_view(sv.grids[uni_ptr(&sv.volumes[0])->grid_id]);
    Counters k{0u, 0u, 0u};
    skip::Walk wk;
    uint32_t q = ~0u;     // the path this lane walks (~0u: none)
    int mode = kWalkMiss;
    uint32_t avail = 0u, cur = 0u;  // grabbed list entries not yet handed out, and where they start
    bool more = true;               // entries may be left in the list
    uint32_t line = pool_line0();
    for (;;) {
        if (q != ~0u && mode >= kWalkMiss) {  // finished: its hit record
            nearest_end_1v(sv, pr, q, wk, mode == kWalkHit);
            q = ~0u;
        }
        while (more) {
            const uint64_t idle = __ballot(q == ~0u);
            if (!idle) break;
            if (avail == 0u) {  // the next chunk of the list (every entry traces a ray)
                const uint32_t g = pool_grab(w.pool + kPoolBounce + level * kGrabBlock, (n + kPoolChunk - 1u) / kPoolChunk, line);
                if (g == ~0u) {
                    more = false;
                    break;
                }
                cur = g * kPoolChunk;
                avail = min(kPoolChunk, n - cur);
                continue;
            }
            const uint32_t take = min((uint32_t)__popcll(idle), avail);
            const uint32_t r = lane_rank(idle);
            if (q == ~0u && r < take) {
                q = L[cur + r];
                mode = nearest_begin_1v(sv, pr, q, k, wk) ? kWalkStep : kWalkMiss;
            }
            cur += take;
            avail -= take;
        }
        if (!__ballot(q != ~0u)) break;  // the list is done and every lane is done
        walk_wave<0, kSkipwBounce, kMincBounce, kRunBounce, true>(gv, wk, kBig, k.cells, &mode,
                                                                   more ? kPoolLeave : 65u);
    }
    flush_counters(k, 0u, ctr, VPX_STAGE_BOUNCE);
}

// Renderer::IsOccluded for the shadow slots of a tile (entry = slot << 27 | path).  The
// tile's slots are counting-sorted by the light they go to (LDS histogram, one wave's prefix
// sum, the scatter), so a wave's lanes walk toward the same light and read the same
// distance-field words (C3, 4 area lights x 3 samples: 6.69 -> 6.24 ms/frame).
// An occluded slot: its bit in the tile's LDS bitmap (fused tails), else kSlotOcc in its SD word.
constexpr uint32_t kOccWords = 15u * 256u / 32u;  // area_samples <= 15 slots per path
__device__ __forceinline__ void mark_occluded(const WaveBufs& w, uint64_t slot, uint32_t e, uint32_t* occ) {
    if (occ) {
        const uint32_t b = (e >> 27) * 256u + (e & 255u);
        atomicOr(&occ[b >> 5], 1u << (b & 31u));
    } else {
        w.SD[slot].w = __uint_as_float(__float_as_uint(w.SD[slot].w) | 4u /* kSlotOcc */);
    }
}

// occ: the fused tails' LDS bitmap of occluded slots (one tile per workgroup), else nullptr.
// RUN: the shadow walks' RUN word (vpx_trace.hpp kRun*).  k_frame0's shadow walks (80 VGPRs)
// keep kRunShadow: the two-compare step (5 spilled VGPRs instead of 3) measured C1
// 0.5824-0.5839 vs 0.5833-0.5859 ms and runs of 4 cells 0.5843-0.5873 (round 3, three
// interleaved runs each: noise / slower).
// p: this thread's path (the tile's, or a live-list entry; >= w.P: none).
// l16 (k_frame0: one slot per path, the tile's own paths): the list as 16-bit offsets into the
// tile in the caller's LDS instead of 32-bit entries in the dynamic LDS.
template <bool ONE, uint32_t RUN = kRunShadow>
__device__ __forceinline__ void shadow_tile(const SceneView& sv, const WaveBufs& w, unsigned long long* __restrict__ ctr,
                                            uint32_t* occ, uint32_t p, uint16_t* l16 = nullptr) {
    __shared__ uint32_t sh[4];
    if (occ)
        for (uint32_t i = threadIdx.x; i < w.S * 8u; i += 256u) occ[i] = 0u;  // published by the barriers below
    extern __shared__ uint32_t lst_dyn[];  // [S * 256]
    Counters k{0u, 0u, 0u};
    // counting sort of the tile's slots by light key: LDS histogram (the order inside a
    // bucket is whatever the atomics give — it only orders independent walks), bucket
    // offsets from one wave's prefix sum, then the scatter
    __shared__ uint32_t hist[kLightKeys];
    if (threadIdx.x < kLightKeys) hist[threadIdx.x] = 0u;
    __syncthreads();
    const uint32_t sm = p < w.P ? w.smask[p] : 0u;
    const uint32_t m = sm & kSlotBits, key = sm >> 16;
    const uint32_t pos = m ? atomicAdd(&hist[key], (uint32_t)__popc(m)) : 0u;
    __syncthreads();
    uint32_t total = 0;
    if (threadIdx.x < 64) {
        const uint32_t v = threadIdx.x < kLightKeys ? hist[threadIdx.x] : 0u;
        uint32_t t;
        const uint32_t ex = wave_prefix(v, t);
        if (threadIdx.x < kLightKeys) hist[threadIdx.x] = ex;
        if (threadIdx.x == 0) sh[0] = t;
    }
    __syncthreads();
    total = __builtin_amdgcn_readfirstlane(sh[0]);  // wave-uniform: a scalar register
    const uint32_t tb = tile_block() * 256u;
    {
        uint32_t at = m ? hist[key] + pos : 0u;
        if (l16) {
            if (m) l16[at] = (uint16_t)(p - tb);  // slot 0
        } else {
            for (uint32_t b = m; b; b &= b - 1u) lst_dyn[at++] = ((uint32_t)__ffs(b) - 1u) << 27 | p;
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < total; i += 256u) {
        const uint32_t e = l16 ? tb + l16[i] : lst_dyn[i];
        const uint64_t slot = (uint64_t)(e >> 27) * w.P + (e & 0x07ffffffu);
        if (ONE) {
            // Renderer::IsOccluded in the single volume with only the walk state live
            // across the walk (the slot flags are read back afterwards)
            const vpx_volume* vol = uni_ptr(&sv.volumes[0]);
            const DevGrid g = sv.grids[vol->grid_id];
            ++k.shadow;
            bool hit = false;
            {
                const float4 so = w.SO[slot], sd = w.SD[slot];
                ORay o;
                o.O = xform_pos(mk(so.x, so.y, so.z), vol->inv_matrix);
                o.D = xform_vec(mk(sd.x, sd.y, sd.z), vol->inv_matrix);
                o.rD = mk(__fdiv_rn(1.0f, o.D.x), __fdiv_rn(1.0f, o.D.y), __fdiv_rn(1.0f, o.D.z));
                Dda s;
                if (dda_setup(*vol, g.n, o, s)) {
                    skip::Walk wk = to_walk(s);
                    hit = walk_wave<16, kSkipwShadow, kMincShadow, RUN>(grid_view(g), wk, so.w, k.cells);
                }
            }
            asm volatile("" ::: "memory");
            if (hit) mark_occluded(w, slot, e, occ);
            continue;
        }
        const float4 so = w.SO[slot], sd = w.SD[slot];
        Ray r;
        r.O = mk(so.x, so.y, so.z);
        r.D = mk(sd.x, sd.y, sd.z);
        r.t = so.w;
        if (shadow(sv, r, k)) mark_occluded(w, slot, e, occ);
    }
    flush_counters(k, 0u, ctr, VPX_STAGE_SHADOW);
}

template <bool ONE>
__global__ __launch_bounds__(256) VPX_WPE(ONE ? VPX_WPE_SHADOW : VPX_WPE_MULTI_SHADOW) void k_shadow_tile(SceneView sv, WaveBufs w, unsigned long long* __restrict__ ctr) {
    shadow_tile<ONE>(sv, w, ctr, nullptr, tile_block() * 256u + threadIdx.x);
}

// Level l >= 1's shadow walks over its live list: a workgroup takes 256 entries and walks
// those paths' slots as shadow_tile walks a tile's (counting-sorted by light).
template <bool ONE>
__global__ __launch_bounds__(256) VPX_WPE(ONE ? VPX_WPE_SHADOW : VPX_WPE_MULTI_SHADOW) void k_shadow_list(SceneView sv, WaveBufs w, int level,
                                                                                                       unsigned long long* __restrict__ ctr) {
    const uint32_t n = live_count(w, level);
    if (blockIdx.x * 256u >= n) return;  // one chunk per workgroup (k_nearest_tile)
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    shadow_tile<ONE>(sv, w, ctr, nullptr, i < n ? live_path(w, level, i) : ~0u);
}

// The shadow pool (single-volume scenes): Renderer::IsOccluded for a level's shadow slots,
// walked by persistent waves that refill their finished lanes, as the bounce pool does for
// FindNearest.  A grab is `grab` mask words of paths (64 each, at most kShadowList slots);
// their slots are listed in the wave's LDS grouped by light key (the tile kernels' bucketing:
// a wave's lanes head for the same light), entry = slot << 27 | path.  Each slot's result goes
// to occb (1 = occluded) for k_resolve / k_resolve_finish; a slot is walked by exactly
// shadow_tile's per-lane sequence, so counts and occlusion are the same.
constexpr uint32_t kShadowList = 1024;  // listed slots per wave (LDS: 4 KiB)
// At 7 waves/SIMD (72 VGPRs) it spilled 29 VGPRs, 21 scratch accesses inside the skip phase;
// at 5 (96 VGPRs) one.  Measured C3 (ms, two runs each): 7 -> 4.85 / 4.81, 6 -> 3.83 / 3.80,
// 5 -> 3.72 / 3.71, against 4.96 / 4.94 for the tile kernels.
#ifndef VPX_WPE_SPOOL
#define VPX_WPE_SPOOL 5
#endif
template <bool MULTI>  // multi-volume / shape scenes: the pool walks the world and lists the rest (slist)
__global__ __launch_bounds__(kPoolWg) VPX_WPE(VPX_WPE_SPOOL) void k_shadow_pool(SceneView sv, WaveBufs w, int level,
                                                                              uint32_t grab,
                                                                              unsigned long long* __restrict__ ctr) {
    __shared__ uint32_t lst_wg[kPoolWg / 64][kShadowList];
    __shared__ uint32_t hist_wg[kPoolWg / 64][kLightKeys];
    uint32_t* lst = lst_wg[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)];
    uint32_t* hist = hist_wg[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t n = live_count(w, level);  // level 0: every path; later: the level's live list
    const uint32_t grabs = (n + 64u * grab - 1u) / (64u * grab);
    const vpx_volume* vol = uni_ptr(&sv.volumes[0]);
    const DevGrid g = sv.grids[vol->grid_id];
    const skip::GridView gv = grid_view(g);
    Counters k{0u, 0u, 0u};
    skip::Walk wk;
    uint32_t e = ~0u;  // the slot entry this lane walks (~0u: none)
    uint32_t walked = 0u;
    float bound = 0.f;
    int mode = kWalkMiss;
    uint32_t avail = 0u, cur = 0u;
    bool more = true;
    uint32_t line = pool_line0();
    // multi-volume / shape scenes: the pool walks the world (volume 0); a slot it leaves
    // unoccluded whose segment may meet a later volume goes to the level's slot list for
    // k_shadow_slots (one atomic per wave and batch of finished lanes)
    for (;;) {
        if constexpr (!MULTI) {  // (single volume: the result only)
            if (e != ~0u && mode >= kWalkMiss) {
                w.occb[(uint64_t)(e >> 27) * w.P + (e & 0x07ffffffu)] = mode == kWalkHit ? 1u : 0u;
                e = ~0u;
            }
        } else {
            const bool fin = e != ~0u && mode >= kWalkMiss;
            bool app = false;
            if (fin) {
                const uint64_t slot = (uint64_t)(e >> 27) * w.P + (e & 0x07ffffffu);
                w.occb[slot] = mode == kWalkHit ? 1u : 0u;
                if (mode != kWalkHit) {
                    const float4 so = w.SO[slot], sd = w.SD[slot];
                    app = meets_later_volume(sv, mk(so.x, so.y, so.z), mk(sd.x, sd.y, sd.z), so.w);
                }
            }
            const uint64_t b = __ballot(app);
            if (b) {
                uint32_t base = 0u;
                if (lane == (uint32_t)__ffsll((unsigned long long)b) - 1u)
                    base = atomicAdd(&w.pool[kPoolSlots + level * kLineWords], (uint32_t)__popcll(b));
                base = (uint32_t)__builtin_amdgcn_readlane((int)base, __ffsll((unsigned long long)b) - 1);
                if (app) slot_list(w)[base + lane_rank(b)] = e;
            }
            if (fin) e = ~0u;
        }
        while (more) {
            const uint64_t idle = __ballot(e == ~0u);
            if (!idle) break;
            if (avail == 0u) {
                const uint32_t gi = pool_grab(w.pool + kPoolShadow + level * kGrabBlock, grabs, line);
                if (gi == ~0u) {
                    more = false;
                    break;
                }
                wave_sync();
                // the grab's slots, grouped by light key: a counting sort over the wave (LDS
                // histogram with atomics, the buckets' prefix sum, the scatter)
                if (lane < kLightKeys) hist[lane] = 0u;
                wave_sync();
                uint32_t smv[4], pos[4];
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    const uint32_t i = (gi * grab + j) * 64u + lane;
                    smv[j] = (j < grab && i < n) ? w.smask[live_path(w, level, i)] : 0u;
                    const uint32_t m = smv[j] & kSlotBits;
                    pos[j] = m ? atomicAdd(&hist[smv[j] >> 16], (uint32_t)__popc(m)) : 0u;
                }
                wave_sync();
                uint32_t n;
                const uint32_t ex = wave_prefix(lane < kLightKeys ? hist[lane] : 0u, n);
                wave_sync();
                if (lane < kLightKeys) hist[lane] = ex;
                wave_sync();
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    const uint32_t m = smv[j] & kSlotBits;
                    if (m) {
                        const uint32_t p = live_path(w, level, (gi * grab + j) * 64u + lane);
                        uint32_t at = hist[smv[j] >> 16] + pos[j];
                        for (uint32_t b = m; b; b &= b - 1u) lst[at++] = ((uint32_t)__ffs(b) - 1u) << 27 | p;
                    }
                }
                wave_sync();
                avail = n;
                cur = 0u;
                continue;
            }
            const uint32_t take = min((uint32_t)__popcll(idle), avail);
            const uint32_t r = lane_rank(idle);
            if (e == ~0u && r < take) {
                e = lst[cur + r];
                const uint64_t slot = (uint64_t)(e >> 27) * w.P + (e & 0x07ffffffu);
                const float4 so = w.SO[slot], sd = w.SD[slot];
                ORay o;
                o.O = xform_pos(mk(so.x, so.y, so.z), vol->inv_matrix);
                o.D = xform_vec(mk(sd.x, sd.y, sd.z), vol->inv_matrix);
                o.rD = mk(__fdiv_rn(1.0f, o.D.x), __fdiv_rn(1.0f, o.D.y), __fdiv_rn(1.0f, o.D.z));
                Dda s;
                bound = so.w;
                mode = kWalkMiss;
                if (dda_setup(*vol, g.n, o, s)) {
                    wk = to_walk(s);
                    mode = kWalkStep;
                }
            }
            cur += take;
            avail -= take;
            walked += take;  // IsOccluded calls (a scalar: no register across the walks)
        }
        if (!__ballot(e != ~0u)) break;
        walk_wave<16, kSkipwShadowPool, kMincShadowPool, kRunShadowPool, true>(gv, wk, bound, k.cells, &mode,
                                                                   more ? kPoolLeave : 65u);
    }
    k.shadow = lane == 0u ? walked : 0u;
    flush_counters(k, 0u, ctr, VPX_STAGE_SHADOW);
}

// Multi-volume / shape scenes with area lights: the rest of Renderer::IsOccluded for the slots
// the world left unoccluded (k_shadow_pool walked volume 0, the first in the reference's loop,
// renderer.cpp:209-243): volumes 1.. in order, then the shapes; an occluder sets the slot's
// occb byte.  The slots' IsOccluded calls were counted by the pool.
// The instances' boxes (up to 64: volumes 1..64, bit k = volume k + 1) are tested against the
// slot's segment first, all of them, from a copy in LDS — a branch-free loop of independent tests — and the
// walks then visit the candidates in increasing index order (wave-uniform: one grid per walk),
// each lane stopping at its first occluder: the reference's loop (renderer.cpp:209-243)
// restricted to the volumes whose Setup3DDDA can succeed (misses_volume), so the same
// occlusion and cell counts.  The linear loop read each volume's sphere with a dependent
// vector load per iteration.
#ifndef VPX_INST_MASK
#define VPX_INST_MASK 1
#endif

#ifndef VPX_INST_CULL
#define VPX_INST_CULL 1
#endif
// The instance grids' shadow walks take the shadow words with skip minimum 2 (cubes of one
// brick stepped through): C4 42.43-42.51 vs 42.71-42.96 ms (five interleaved runs, all won; 3:
// 42.82-42.90, 4: 43.05-43.26; two passes per iteration 43.1-43.3, the two-compare step 42.7-42.8).
constexpr uint32_t kMincInstShadow = 2u;
__device__ __forceinline__ bool occluded_instances(const SceneView& sv, const float4* vb, const Ray& r, Counters& k) {
    const uint32_t nv = sv.num_volumes;
    uint64_t cand = 0ull;
#ifdef VPX_DEBUG_PROBE_INST_SHADOW
    if (VPX_DEBUG_PROBE_INST_SHADOW < 2)
#endif
    const f3 inv = world_inv(r.D);
    for (uint32_t i = 1; i < nv; ++i)
        cand |= (misses_volume(vb, i, r.O, inv, r.t) ? 0ull : 1ull) << (i - 1u);
    bool occ = false;
    if (sv.inst_grid >= 0 && VPX_LANE_VOLUMES) {  // each lane its own next candidate (lane_volumes)
        const DevGrid g = ldu(sv.grids, (uint32_t)sv.inst_grid);
        uint64_t rest = cand;
        auto next = [&](skip::Walk& wk, uint32_t& vi) {
            while (rest) {
                const uint32_t i = (uint32_t)__ffsll((unsigned long long)rest);  // bit i - 1 = volume i
                rest &= rest - 1ull;
                const vpx_volume& vol = sv.volumes[i];
                ORay o;
                o.O = xform_pos(r.O, vol.inv_matrix);
                o.D = xform_vec(r.D, vol.inv_matrix);
                o.rD = mk(__fdiv_rn(1.0f, o.D.x), __fdiv_rn(1.0f, o.D.y), __fdiv_rn(1.0f, o.D.z));
                Dda s;
                if (!dda_setup(vol, g.n, o, s)) continue;
                wk = to_walk(s);
                vi = i;
                return true;
            }
            return false;
        };
        auto done = [&](skip::Walk& wk, uint32_t) {
            if (walk_wave<16, kSkipwShadow, kMincInstShadow, kRunShadow>(grid_view(g), wk, r.t, k.cells)) {
                occ = true;
                rest = 0ull;  // the reference returns at the first occluder
            }
        };
        lane_volumes(grid_view(g), next, done);
        if (occ) return true;
        for (uint32_t i = 0; i < sv.num_spheres; ++i)
            if (sphere_is_hit(sv.spheres[i], r)) return true;
        for (uint32_t i = 0; i < sv.num_triangles; ++i)
            if (tri_is_hit(sv.triangles[i], r)) return true;
        return false;
    }

    // the volumes in increasing index order, wave-uniform (a walk needs one grid per wave); a
    // volume no lane of the wave can reach costs one ballot
    for (uint32_t i = 1; i < nv; ++i) {
        const bool want = !occ && ((cand >> (i - 1u)) & 1ull);
#ifdef VPX_DEBUG_PROBE_INST_SHADOW
        // timing probe only (wrong images): 1 = no instance walks, 2 = no sphere tests either
        if (VPX_DEBUG_PROBE_INST_SHADOW >= 1) continue;
#endif
        if (!__ballot(want)) continue;
#ifdef VPX_PHASE_PROF  // instance shadow visits: waves, lanes walking
        if ((threadIdx.x & 63u) == (uint32_t)__ffsll((unsigned long long)__ballot(true)) - 1u)
            atomicAdd(&g_phase[25], 1ull), atomicAdd(&g_phase[26], (unsigned long long)__popcll(__ballot(want)));
#endif
        if (!want) continue;
        const vpx_volume vol = ldu(sv.volumes, i);  // i is wave-uniform
        ORay o;
        o.O = xform_pos(r.O, vol.inv_matrix);
        o.D = xform_vec(r.D, vol.inv_matrix);
        o.rD = mk(__fdiv_rn(1.0f, o.D.x), __fdiv_rn(1.0f, o.D.y), __fdiv_rn(1.0f, o.D.z));
        const DevGrid g = ldu(sv.grids, vol.grid_id);
        Dda s;
        if (!dda_setup(vol, g.n, o, s)) continue;
        skip::Walk wk = to_walk(s);
        occ = walk_wave<16, kSkipwShadow, kMincInstShadow, kRunShadow>(grid_view(g), wk, r.t, k.cells);
    }
    if (occ) return true;
    for (uint32_t i = 0; i < sv.num_spheres; ++i)
        if (sphere_is_hit(sv.spheres[i], r)) return true;
    for (uint32_t i = 0; i < sv.num_triangles; ++i)
        if (tri_is_hit(sv.triangles[i], r)) return true;
    return false;
}

// The rest of Renderer::IsOccluded (volumes 1.., then the shapes) for the shadow pool's slot
// list (slots the world left unoccluded whose segment may meet a later volume): the same
// per-slot loop k_shadow_inst ran (round 5) over every slot of every tile, now over a dense
// list — C4's ~16 k candidate slots per frame had cost a scan of all 25 M slots' flags and rays
// (with lane_volumes: C4 32.5 -> 30.2 ms per step).
// Persistent workgroups striding over the list (its length is on the device).
// 4 waves/SIMD (106 VGPRs, no spills): C4 29.82-29.83 ms per step vs 29.66-29.81 at 5 (5 spilled
// VGPRs) and 30.25-30.36 at 6 (42 spilled, 96 B of scratch per lane).
#ifndef VPX_WPE_SHADOW_SLOTS
#define VPX_WPE_SHADOW_SLOTS 4
#endif
__global__ __launch_bounds__(256) VPX_WPE(VPX_WPE_SHADOW_SLOTS) void k_shadow_slots(SceneView sv, WaveBufs w, int level,
                                                                                   unsigned long long* __restrict__ ctr) {
    __shared__ float4 vb[2 * kTlasMaxVolumes];
    if (VPX_INST_MASK && threadIdx.x < 2u * sv.num_volumes && threadIdx.x < 2u * kTlasMaxVolumes)
        vb[threadIdx.x] = sv.vbounds[threadIdx.x];
    __syncthreads();
    Counters k{0u, 0u, 0u};
    const uint32_t n = __builtin_amdgcn_readfirstlane(w.pool[kPoolSlots + level * kLineWords]);
    for (uint32_t base = blockIdx.x * 256u; base < n; base += gridDim.x * 256u) {
        const uint32_t i = base + threadIdx.x;
        if (i >= n) continue;
        const uint32_t e = slot_list(w)[i];
        const uint64_t slot = (uint64_t)(e >> 27) * w.P + (e & 0x07ffffffu);
        const float4 so = w.SO[slot], sd = w.SD[slot];
        Ray r;
        r.O = mk(so.x, so.y, so.z);
        r.D = mk(sd.x, sd.y, sd.z);
        r.t = so.w;
        const bool occ = (VPX_INST_MASK && sv.num_volumes <= kTlasMaxVolumes) ? occluded_instances(sv, vb, r, k)
                                                                              : is_occluded(sv, r, k, 1u);
        if (occ) w.occb[slot] = 1u;
    }
    flush_counters(k, 0u, ctr, VPX_STAGE_SHADOW);
}

// ------------------------------------------------------------------- stage 4
// GetLuminance / ApplyReinhardJodie / RGBF32_to_RGB8 (renderer.cpp:2222-2240,
// template/precomp.h:372-388).
__device__ __forceinline__ uint32_t tonemap_pack(float4 a) {
    const f3 c = mk(a.x, a.y, a.z);
    const float lum = dot(c, mk(0.2126f, 0.7152f, 0.0722f));
    const f3 rh = c / mk(1.0f + c.x, 1.0f + c.y, 1.0f + c.z);
    const f3 la = c / (1.0f + lum);
    const float o0 = la.x + rh.x * (rh.x - la.x);
    const float o1 = la.y + rh.y * (rh.y - la.y);
    const float o2 = la.z + rh.z * (rh.z - la.z);
    const uint32_t r = (uint32_t)(int64_t)(255.0f * smin(1.0f, o0));
    const uint32_t gg = (uint32_t)(int64_t)(255.0f * smin(1.0f, o1));
    const uint32_t b = (uint32_t)(int64_t)(255.0f * smin(1.0f, o2));
    return (r << 16) + (gg << 8) + b;
}

// Running-average blend of the AVX path: fma(1-w, acc, px*w) (renderer.cpp:1797-1828).
__device__ __forceinline__ float4 blend(float4 acc, f3 px, float w, float iw) {
    return make_float4(fmaf(iw, acc.x, px.x * w), fmaf(iw, acc.y, px.y * w), fmaf(iw, acc.z, px.z * w),
                       fmaf(iw, acc.w, 0.0f * w));
}

// k_finish output modes: the image accumulator + screen (one GPU), the raw sample per packed
// slot (rank-0 composite), or a rank's own packed accumulator + packed RGB8 (the
// accumulator sharded with the tiles; only the RGB8 travels).
enum FinishMode : int { kFinishImage = 0, kFinishPackedSample = 1, kFinishPackedAccum = 2 };

// A path's value: the level records folded bottom-up (the recursion's rounding order); ls: the
// last level's light sum when the launch resolved it (fused tails).
__device__ __forceinline__ f3 path_value(const WaveBufs& w, uint32_t p, const LightSum* ls) {
    f3 v = mk(0.f, 0.f, 0.f);
    const uint32_t forms = w.forms[p];
    if (forms & kLeafBit) {
        const float4 lf = w.leaf[p];
        v = mk(lf.x, lf.y, lf.z);
    }
    for (int i = (int)forms_count(forms) - 1; i >= 0; --i) {
        const uint32_t form = (forms >> (2 * i)) & 3u;
        const uint64_t li = (uint64_t)i * w.P + p;
        const float4 a4 = w.LA[li];
        const f3 a = mk(a4.x, a4.y, a4.z);
        if (form == kFormMulAdd || form == kFormAddMul) {
            f3 b;
            if (ls && ls->lvl == (uint32_t)i) {
                b = ls->inc;  // this launch's resolve (fused tail)
            } else {
                const float4 b4 = w.LB[li];
                b = mk(b4.x, b4.y, b4.z);
            }
            v = form == kFormMulAdd ? b + v * a : (v + b) * a;
        } else if (form == kFormMul) {
            v = v * a;
        }
    }
    return v;
}

// Fold the level records (path_value), then write per MODE.
template <int MODE>
__device__ __forceinline__ void finish_path(const FrameArgs& f, const WaveBufs& w, uint32_t p, float4* __restrict__ accum,
                                            uint32_t* __restrict__ rgb8, float4* __restrict__ packed,
                                            const LightSum* ls = nullptr) {
    if (p >= w.P) return;
    uint32_t x, y;
    // window chains finish into packed samples only
    const bool valid = MODE == kFinishPackedSample ? path_pixel(f, p, x, y) : path_pixel_single(f, p, x, y);
    const f3 v = valid ? path_value(w, p, ls) : mk(0.f, 0.f, 0.f);
    if (MODE == kFinishPackedSample) {
        packed[p] = make_float4(v.x, v.y, v.z, 0.0f);
    } else if (MODE == kFinishPackedAccum) {  // accum / rgb8 are this rank's packed buffers
        if (valid) {
            const float4 a = blend(accum[p], v, f.weight, f.inv_weight);
            accum[p] = a;
            rgb8[p] = tonemap_pack(a);
        } else {
            accum[p] = make_float4(0.f, 0.f, 0.f, 0.f);
            rgb8[p] = 0u;
        }
    } else if (valid) {
        const uint64_t px = (uint64_t)y * f.width + x;
        if (f.flags & VPX_FLAG_NO_TONEMAP) {
            accum[px] = make_float4(v.x, v.y, v.z, 0.0f);
        } else {
            const float4 a = blend(accum[px], v, f.weight, f.inv_weight);
            accum[px] = a;
            if (rgb8) rgb8[px] = tonemap_pack(a);
        }
    }
}

template <int MODE>
__global__ __launch_bounds__(256) void k_finish(FrameArgs f, WaveBufs w, float4* __restrict__ accum,
                                                uint32_t* __restrict__ rgb8, float4* __restrict__ packed) {
    finish_path<MODE>(f, w, blockIdx.x * 256u + threadIdx.x, accum, rgb8, packed);
}

// The last level's resolve and the finish after the shadow pool (occb): k_shadow_finish's
// per-path tail as its own launch.
template <int MODE>
__global__ __launch_bounds__(256) void k_resolve_finish(SceneView sv, FrameArgs f, WaveBufs w, float4* __restrict__ accum,
                                                        uint32_t* __restrict__ rgb8, float4* __restrict__ packed) {
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;
    LightSum ls;
    resolve_path(sv, w, p, nullptr, &ls);
    finish_path<MODE>(f, w, p, accum, rgb8, packed, &ls);
}

// An accumulation window's frame weights (renderer.cpp:1651's 1/(n+1), computed on the host as
// frame_of does, so every blend uses the per-frame path's exact weights).
constexpr uint32_t kMaxWindow = 64;
struct WindowWeights {
    float w[kMaxWindow], iw[kMaxWindow];
};
struct WindowTail {
    uint32_t B;  // frames in the chain (frame b: tile blocks [b*batch_tiles, (b+1)*batch_tiles))
    int image;   // accum / rgb8 indexed by pixel (one GPU), else a rank's packed buffers
    WindowWeights ww;
};

// A window chain's tail on its lane (vpx_render_window, frames whose tail is a launch of its
// own): one thread per pixel of the chain resolves (RESOLVE: k_resolve_finish's last-level light
// sum) and folds each of its B frames' paths and blends them into the accumulator in frame
// order — the B per-frame blends of the same values, with no samples written or re-read.
template <bool RESOLVE>
__global__ __launch_bounds__(256) void k_finish_window(SceneView sv, FrameArgs f, WaveBufs w, WindowTail wt,
                                                       float4* __restrict__ accum, uint32_t* __restrict__ rgb8) {
    const uint32_t p0 = blockIdx.x * 256u + threadIdx.x;
    uint32_t x, y;
    const bool valid = path_pixel(f, p0, x, y);
    if (wt.image && !valid) return;
    const uint64_t at = wt.image ? (uint64_t)y * f.width + x : p0;
    if (!valid) {
        accum[at] = make_float4(0.f, 0.f, 0.f, 0.f);
        rgb8[at] = 0u;
        return;
    }
    float4 a = accum[at];
    const uint32_t stride = f.batch_tiles * 256u;
    for (uint32_t b = 0; b < wt.B; ++b) {
        const uint32_t p = p0 + b * stride;
        f3 v;
        if (RESOLVE) {
            LightSum ls;
            resolve_path(sv, w, p, nullptr, &ls);
            v = path_value(w, p, &ls);
        } else {
            v = path_value(w, p, nullptr);
        }
        a = blend(a, v, wt.ww.w[b], wt.ww.iw[b]);
    }
    accum[at] = a;
    if (rgb8) rgb8[at] = tonemap_pack(a);
}

// The deep levels in one launch (k_tail): from level `level` on, each lane carries one path of
// the level's live list through every remaining level — its FindNearest, the material switch,
// IsOccluded for the level's shadow slots, the light sum — until the path ends; k_finish then
// folds every path.  The same per-path operations as the level kernels (nearest_record,
// shade_path, shadow, resolve_path), so the same values, RNG order and counts; the levels stop
// costing a launch, a compaction and the longest walk of each level.  Deep levels hold few
// paths (Z1 at 1920x1080: 192 k at level 5, 3.7 k at level 14), so the kernel's registers (the
// whole chain inlined) and low occupancy cost little, while each of those levels cost ~0.2 ms
// of launches and latency chains in the per-level kernels.
// Its occupancy (round 6, Z1 ms per step, two interleaved runs): 2 waves/SIMD (172 VGPRs, SGPR
// spills only, to VGPR lanes) 1.488 / 1.495, 3 (168, 10 spilled VGPRs) 1.491 / 1.507, 4 (128, 80
// spilled, 212 B of scratch) 1.521 / 1.531 — the deep levels hold too few paths for a third wave
// per SIMD to find work, so the kernel costs its longest path's chain either way.
#ifndef VPX_WPE_TAIL
#define VPX_WPE_TAIL 2
#endif
__global__ __launch_bounds__(256) VPX_WPE(VPX_WPE_TAIL) void k_tail(SceneView sv_, FrameArgs f, WaveBufs w, int level,
                                                      unsigned long long* __restrict__ ctr) {
    Counters kn{0u, 0u, 0u}, ks{0u, 0u, 0u}, kh{0u, 0u, 0u};
    const uint32_t n = live_count(w, level);
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (blockIdx.x * 256u >= n) return;  // (workgroup-uniform: before the staging barrier)
    extern __shared__ uint32_t x86_lds[];
    SceneView sv = sv_;
    sv.x86 = x86_stage_lds(sv_.x86, x86_lds);
    const uint32_t p = i < n ? live_path(w, level, i) : ~0u;
    const PathRay pr{w.O, w.D, w.H, w.HM, 0u};
    for (int l = level; p != ~0u; ++l) {
        {  // Renderer::FindNearest for the ray the previous level's shade traced
            const float4 o = w.O[p], d = w.D[p];
            Ray r;
            r.O = mk(o.x, o.y, o.z);
            r.D = mk(d.x, d.y, d.z);
            r.inside = (__float_as_uint(d.w) & kInside) != 0u;
            nearest_record<kSkipwBounce, kMincBounce, kRunBounce>(sv, pr, p, r, kn);
        }
        const bool cont = shade_path(sv, f, w, pr, p, l, kh);
        const uint32_t slots = w.smask[p] & kSlotBits;
        for (uint32_t b = slots; b; b &= b - 1u) {  // IsOccluded of each of the level's shadow rays
            const uint64_t slot = (uint64_t)((uint32_t)__ffs(b) - 1u) * w.P + p;
            const float4 so = w.SO[slot], sd = w.SD[slot];
            Ray r;
            r.O = mk(so.x, so.y, so.z);
            r.D = mk(sd.x, sd.y, sd.z);
            r.t = so.w;
            if (shadow(sv, r, ks)) w.SD[slot].w = __uint_as_float(__float_as_uint(sd.w) | 4u /* kSlotOcc */);
        }
        resolve_path(sv, w, p);  // the level's light sum into LB (the slots' SD flags)
        if (!cont || l >= f.max_bounces) break;
    }
    flush_counters(kn, 0u, ctr, VPX_STAGE_BOUNCE);
    flush_counters(ks, 0u, ctr, VPX_STAGE_SHADOW);
    flush_counters(kh, 0u, ctr, VPX_STAGE_SHADE);
}

// The last level's tail in one launch: IsOccluded for the tile's shadow slots, then (after
// the workgroup barrier, which makes the slots' occluded flags visible to the whole tile)
// each thread resolves and finishes its own path.  The same per-path operations as
// k_shadow_tile -> k_resolve -> k_finish, so the same values; the light/accumulate work of
// a finished tile overlaps the walks of the others instead of running as two more
// bandwidth-bound launches after the slowest walk.
template <bool ONE, int MODE>
__global__ __launch_bounds__(256) VPX_WPE(ONE ? VPX_WPE_SHADOW : VPX_WPE_MULTI_SHADOW) void k_shadow_finish(
    SceneView sv, FrameArgs f, WaveBufs w, unsigned long long* __restrict__ ctr, float4* __restrict__ accum,
    uint32_t* __restrict__ rgb8, float4* __restrict__ packed) {
    __shared__ uint32_t occ[kOccWords];
    shadow_tile<ONE>(sv, w, ctr, occ, tile_block() * 256u + threadIdx.x);
    __syncthreads();
    uint32_t p = tile_block() * 256u + threadIdx.x;  // re-derived after the walks, not kept live across them
    asm volatile("" : "+v"(p));
    LightSum ls;
    resolve_path(sv, w, p, occ, &ls);
    finish_path<MODE>(f, w, p, accum, rgb8, packed, &ls);
}

// The other levels' tail is NOT fused the same way (IsOccluded walks + barrier + resolve as
// one launch measured 4.32-4.34 vs 4.30-4.31 ms on C2: the barrier holds the tile's finished
// waves longer than the separate 14-us resolve costs).
//
// A Trace-depth-0 frame in one launch (k_frame0): the fused head (primary walk + level-0
// shade) and the fused tail (the tile's shadow walks, resolve, finish) of the same tile, one
// barrier apart — the shade's slots are read back by the workgroup that wrote them (as
// k_shadow_finish reads its own occluded flags), and a tile's shadow walks overlap other
// tiles' primary walks instead of waiting for the slowest primary wave of the frame.
// Used for single-volume launches of at most kFuseFrameTiles tiles, where the walkers'
// drain tails dominate (one MI355X, ms, two launches -> one, VPX_WPE_FRAME 5: C1 0.723 ->
// 0.713; rank 0's share of C1 at 8 ranks 0.297 -> 0.228; C1 at 64x64 0.234 -> 0.198).  On
// the big launches the two kernels stay apart (C3 5.84 vs 6.14; C4, 65 volumes, 59.3 vs
// 64.5): there the separate kernels' 6 waves/SIMD pay more than the shared drain.  Running
// each wave's pixels through the whole frame with wave-local compaction and no
// workgroup barrier measured C1 0.725 vs 0.711 ms (the tile's barriers are not what sets the
// small-launch floor; its longest walk chains are).
#ifndef VPX_FUSE_FRAME_TILES
#define VPX_FUSE_FRAME_TILES 12288
#endif
constexpr uint32_t kFuseFrameTiles = VPX_FUSE_FRAME_TILES;
// k_frame0 occupancy: with the path state in LDS (round 3) 6 waves/SIMD spill 22 VGPRs
// (round 2: 272) and measured 1.5 % faster than 5 (no spills) with frames in flight
// (profiles/r03_frame_occupancy_ab.txt).  Round 5: the occluded bitmap sized for its one slot
// per path and the shadow list as 16-bit tile offsets in static LDS (23168 instead of
// 24128 bytes per workgroup) let 7 workgroups share a CU's 160 KiB; at 7 (72 VGPRs, 14-19
// spilled) C1 measured 0.5440-0.5509 vs 0.5478-0.5580 ms at 6 (seven interleaved runs, five
// won).
#ifndef VPX_WPE_FRAME
#define VPX_WPE_FRAME 7
#endif
// The depth-0 frame's path state never leaves the workgroup: a path is shaded, its light
// resolved and its pixel finished by the same thread, and its shadow slots are walked by the
// same tile, so the shade's records (LA / leaf, SM, forms, smask) and — one slot per path: the
// kernel runs scenes without area lights only — the slots themselves (SO, SD, SL) live in LDS.
// With area lights (several slots per path) the split frame with the shadow pool is faster
// (C3's rank-0 share at 4 ranks, 8100 tiles: 1.31 ms through k_frame0 with its slots in HBM,
// 2.6 x the 2-rank share).  They reuse the
// head's regions once the head is done with them: the slots take the tile's ray records
// (O / D / H: each thread reads its own path's before it writes its own slot), smask the hit
// records, forms the walker list (dead after the walks' barrier).  The tile's WaveBufs view
// points those arrays at LDS, shifted by the tile's first path so that path p indexes them
// as p (level 0 and slot 0 only: every index is p).  HBM sees the accumulator / screen.
template <bool ONE, int MODE, bool X86 = false>
__global__ __launch_bounds__(256) VPX_WPE(ONE ? VPX_WPE_FRAME : VPX_WPE_MULTI_NEAREST) void k_frame0(
    SceneView sv_, FrameArgs f_, WaveBufs w, unsigned long long* __restrict__ ctr, float4* __restrict__ accum,
    uint32_t* __restrict__ rgb8, float4* __restrict__ packed) {
    const SceneView sv = arith_view<X86>(sv_);
    FrameArgs f = f_;
    f.batch_tiles = 0;  // window chains do not take this launch (launch_render)
    __shared__ HeadLds<true> L;
    __shared__ float4 s_val[256];  // LA (a) or leaf of the path's one level
    __shared__ float4 s_sm[256];   // SM: the pending light
    __shared__ uint32_t occ[8];      // one slot per path (S == 1, checked at launch)
    __shared__ uint16_t l16[256];    // the shadow walks' list (shadow_tile)
    const uint32_t tb = tile_block() * 256u;
    const uint32_t p = tb + threadIdx.x;
    WaveBufs wl = w;
    wl.LA = s_val - tb;
    wl.leaf = s_val - tb;  // a path has a leaf (sky / emissive) or a level, never both
    wl.SM = s_sm - tb;
    wl.smask = L.hm - tb;
    wl.forms = L.lst - tb;
    wl.SO = L.ray - tb;
    wl.SD = L.ray + 256 - tb;
    wl.SL = L.ray + 512 - tb;
    primary_tile<ONE, true, kRunFrameNearest>(sv, f, wl, L, ctr);
    __syncthreads();
#ifdef VPX_FRAME_P_TILE
    shadow_tile<ONE, kRunFrameShadow>(sv, wl, ctr, occ, tile_block() * 256u + threadIdx.x, l16);
#else
    uint32_t ps = p;  // re-derived, not kept live across the head (as pt below)
    asm volatile("" : "+v"(ps));
    shadow_tile<ONE, kRunFrameShadow>(sv, wl, ctr, occ, ps, l16);
#endif
    __syncthreads();
    // the tail's own copy of p: the shade's per-lane LDS addresses are re-derived here
    // instead of being kept live (spilled) across the shadow walks
    uint32_t pt = p;
    asm volatile("" : "+v"(pt));
    LightSum ls;
    resolve_path(sv, wl, pt, occ, &ls);
    finish_path<MODE>(f, wl, pt, accum, rgb8, packed, &ls);
}

// ------------------------------------------------------ static-camera reprojection
// Renderer::Tick's static branch (renderer.cpp:1996-2101): TraceReproject per pixel
// (albedo and illumination kept apart at the top level), then per pixel: reproject the
// level-0 intersection into the previous camera, test it against the scene from the
// previous camera position, sample the illumination history bilinearly, clamp it to the
// YCoCg neighbourhood box of the new samples, blend by material, tonemap.

struct PrevCam {  // vpx_prev_camera
    f3 pos, left, right, top, bottom;
};

// Top level of TraceReproject from the path's records: (albedo, illumination).
__global__ __launch_bounds__(256) void k_finish_reproject(FrameArgs f, WaveBufs w, float4* __restrict__ alb,
                                                          float4* __restrict__ ill) {
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;
    if (p >= w.P) return;
    uint32_t x, y;
    if (!path_pixel_single(f, p, x, y)) return;
    const uint64_t px = (uint64_t)y * f.width + x;
    f3 A = mk(0.f, 0.f, 0.f), I = mk(0.f, 0.f, 0.f);  // TraceReproject(ray, depth < 0) = {0, 0}
    if (f.max_bounces < 0) {
        // the ray never reaches FindNearest: GetRayInfo sees t = 1e34, NONE (renderer.cpp:2020)
        const float4 o = w.O[p], d = w.D[p];
        const f3 ip = mk(o.x, o.y, o.z) + mk(d.x, d.y, d.z) * kBig;
        w.RD[px] = make_float4(ip.x, ip.y, ip.z, __uint_as_float(kNone));
    } else {
        const uint32_t forms = w.forms[p];
        f3 v = mk(0.f, 0.f, 0.f);
        if (forms & kLeafBit) {
            const float4 lf = w.leaf[p];
            v = mk(lf.x, lf.y, lf.z);
        }
        const int nl = (int)forms_count(forms);
        if (nl == 0) {  // sky / emissive at the top: {colour, 1} (renderer.cpp:1333, 2330-2333)
            A = v;
            I = mk(1.f, 1.f, 1.f);
        } else {
            for (int i = nl - 1; i >= 1; --i) {  // children's GetColor() bottom-up
                const uint32_t form = (forms >> (2 * i)) & 3u;
                const uint64_t li = (uint64_t)i * w.P + p;
                const float4 a4 = w.LA[li];
                const f3 a = mk(a4.x, a4.y, a4.z);
                if (form == kFormAddMul) {
                    const float4 b4 = w.LB[li];
                    v = (v + mk(b4.x, b4.y, b4.z)) * a;
                } else {
                    v = v * a;
                }
            }
            const float4 a4 = w.LA[p];
            A = mk(a4.x, a4.y, a4.z);
            if ((forms & 3u) == kFormAddMul) {
                const float4 b4 = w.LB[p];
                I = v + mk(b4.x, b4.y, b4.z);
            } else {
                I = v;
            }
        }
    }
    alb[px] = make_float4(A.x, A.y, A.z, 0.f);
    ill[px] = make_float4(I.x, I.y, I.z, 0.f);
}

// Camera::PointToUV (camera.h:33-49) + the half-pixel offset; IsValid (renderer.cpp:1635-1638);
// IsOccludedPrevFrame's ray (renderer.cpp:767-774) into shadow slot 0.
__global__ __launch_bounds__(256) void k_reproject_setup(FrameArgs f, WaveBufs w, PrevCam pc) {
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;
    if (p >= w.P) return;
    uint32_t x, y;
    uint32_t slots = 0;
    w.SM[p] = make_float4(0.f, 0.f, 0.f, __uint_as_float(0u));
    if (path_pixel_single(f, p, x, y)) {
        const float4 rd = w.RD[(uint64_t)y * f.width + x];
        const f3 P = mk(rd.x, rd.y, rd.z);
        const f3 delta = P - pc.pos;
        const float ld = dot(pc.left, delta), rdist = dot(pc.right, delta);
        const float td = dot(pc.top, delta), bd = dot(pc.bottom, delta);
        const float u = ld / (ld + rdist), v = td / (td + bd);
        const float hw = (1.0f / (float)f.width) / 2.0f, hh = (1.0f / (float)f.height) / 2.0f;
        const float uu = u + hw, vv = v + hh;
        const bool valid = uu >= 0.0f && uu < 1.0f && vv >= 0.0f && vv < 1.0f;
        w.SM[p] = make_float4(uu, vv, 0.f, __uint_as_float(valid ? 1u : 0u));
        if (valid) {
            const f3 dn = normalize(P - pc.pos);
            const f3 pos = offset_ray(P, -dn);
            const Ray occ = make_ray(pc.pos, dn);  // Ray{camPos, dir, length(pos - camPos)}
            put_slot(w, 0, p, occ.O, occ.D, length(pos - pc.pos), mk(0.f, 0.f, 0.f), kSlotValid);
            slots = 1u;
        }
    }
    w.smask[p] = slots;
}

__device__ __forceinline__ f3 ld4(const float4* a, uint64_t i) {
    const float4 v = a[i];
    return mk(v.x, v.y, v.z);
}
__device__ __forceinline__ f3 ycocg(f3 c) {  // RGBToYCoCg (renderer.cpp:833-839)
    const float k = (0.5f * 256.0f) / 255.0f;
    return mk(dot(c, mk(1.f, 2.f, 1.f)) * 0.25f, dot(c, mk(2.f, 0.f, -2.f)) * 0.25f + k,
              dot(c, mk(-1.f, 2.f, -1.f)) * 0.25f + k);
}
__device__ __forceinline__ f3 ycocg_rgb(f3 c) {  // YCoCgToRGB (renderer.cpp:842-851)
    const float k = (0.5f * 256.0f) / 255.0f;
    const float co = c.y - k, cg = c.z - k;
    return mk((c.x + co) - cg, c.x + cg, (c.x - co) - cg);
}
__device__ __forceinline__ float clampf_ref(float v, float a, float b) { return fmaxf(a, fminf(v, b)); }
__device__ __forceinline__ bool on_screen(int x, int y, const FrameArgs& f) {  // IsValidScreen
    return (float)x >= 0.0f && (float)x < (float)f.width && (float)y >= 0.0f && (float)y < (float)f.height;
}

// SampleHistory (renderer.cpp:777-830), ClampHistory (:856-910), the material weight and
// lerp (renderer.cpp:2048-2090), ApplyReinhardJodie + RGBF32_to_RGB8.
__global__ __launch_bounds__(256) void k_reproject_resolve(FrameArgs f, WaveBufs w, const float4* __restrict__ alb,
                                                           const float4* __restrict__ ill,
                                                           const float4* __restrict__ hist, float4* __restrict__ temp,
                                                           uint32_t* __restrict__ rgb8) {
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;
    if (p >= w.P) return;
    uint32_t x, y;
    if (!path_pixel_single(f, p, x, y)) return;
    const uint64_t px = (uint64_t)y * f.width + x;
    const f3 ns = ld4(ill, px);
    f3 fin = ns;
    const float4 uvv = w.SM[p];
    const bool occluded = (__float_as_uint(w.SD[p].w) & 4u) != 0u;
    if ((__float_as_uint(uvv.w) & 1u) && !occluded) {
        // bilinear history
        const float ux = uvv.x - (1.0f / (float)f.width) / 2.0f, uy = uvv.y - (1.0f / (float)f.height) / 2.0f;
        const float ptx = ux * (float)f.width, pty = uy * (float)f.height;
        const int tlx = trunc_i32(ptx), tly = trunc_i32(pty);
        const float fx = ptx - (float)tlx, fy = pty - (float)tly;
        const float gx = 1.0f - fx, gy = 1.0f - fy;
        const bool v1 = on_screen(tlx, tly, f), v2 = on_screen(tlx + 1, tly, f), v3 = on_screen(tlx, tly + 1, f),
                   v4 = on_screen(tlx + 1, tly + 1, f);
        float w1 = v1 ? gx * gy : 0.0f, w2 = v2 ? fx * gy : 0.0f, w3 = v3 ? gx * fy : 0.0f, w4 = v4 ? fx * fy : 0.0f;
        const float tw = ((w1 + w2) + w3) + w4;
        const float rtw = 1.0f / tw;
        w1 = w1 * rtw, w2 = w2 * rtw, w3 = w3 * rtw, w4 = w4 * rtw;
        f3 hs = mk(0.f, 0.f, 0.f);
        if (v1) hs = hs + ld4(hist, (uint64_t)tly * f.width + tlx) * w1;
        if (v2) hs = hs + ld4(hist, (uint64_t)tly * f.width + (tlx + 1)) * w2;
        if (v3) hs = hs + ld4(hist, (uint64_t)(tly + 1) * f.width + tlx) * w3;
        if (v4) hs = hs + ld4(hist, (uint64_t)(tly + 1) * f.width + (tlx + 1)) * w4;
        // neighbourhood clamp in YCoCg
        const f3 nsy = ycocg(ns);
        f3 hy = ycocg(hs);
        uint32_t nvalid = 1;
        f3 avg = nsy, var = nsy * nsy;
        const int ox[8] = {-1, 0, 1, -1, 1, -1, 0, 1}, oy[8] = {-1, -1, -1, 0, 0, 1, 1, 1};
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int qx = (int)x + ox[i], qy = (int)y + oy[i];
            if (on_screen(qx, qy, f)) {
                const f3 fe = ycocg(ld4(ill, (uint64_t)qx + (uint64_t)qy * f.width));
                avg = avg + fe;
                var = var + fe * fe;
                ++nvalid;
            }
        }
        const float inv = 1.0f / (float)nvalid;
        avg = avg * inv;
        var = var * inv;
        const f3 sg = mk(sqrtf(smax(0.0f, var.x - avg.x * avg.x)), sqrtf(smax(0.0f, var.y - avg.y * avg.y)),
                         sqrtf(smax(0.0f, var.z - avg.z * avg.z)));
        const f3 lo = avg - sg * 0.75f, hi = avg + sg * 0.75f;
        hy = mk(clampf_ref(hy.x, lo.x, hi.x), clampf_ref(hy.y, lo.y, hi.y), clampf_ref(hy.z, lo.z, hi.z));
        f3 hr = ycocg_rgb(hy);
        hr = mk(fmaxf(hr.x, 0.0f), fmaxf(hr.y, 0.0f), fmaxf(hr.z, 0.0f));
        const uint32_t mat = __float_as_uint(w.RD[px].w);
        float wt = 0.9f;
        if (mat <= VPX_MAT_NON_METAL_PINK) wt = 0.8f;
        else if (mat <= VPX_MAT_METAL_LOW) wt = 0.5f;
        else if (mat == VPX_MAT_GLASS) wt = 0.5f;
        else if (mat == VPX_MAT_EMISSIVE) wt = 0.0f;
        fin = ns + (hr - ns) * wt;  // lerp(a, b, t) = a + t * (b - a)
    }
    temp[px] = make_float4(fin.x, fin.y, fin.z, 0.f);
    if (rgb8) {  // ApplyReinhardJodie(albedo * final) into a float4 with w = 0, RGBF32_to_RGB8
        const f3 c = ld4(alb, px) * fin;
        rgb8[px] = tonemap_pack(make_float4(c.x, c.y, c.z, 0.f));
    }
}

}  // namespace vpx
