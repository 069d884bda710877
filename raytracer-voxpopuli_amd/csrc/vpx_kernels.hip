// vpx_kernels.hip — gfx950 kernels and the C-ABI of libvpx_hip.so (include/vpx.h).
//
// Kernels:
//   render_tiles<LEVELS, PACKED>  one lane per pixel, 16x16-pixel tiles per 256-thread
//                                 workgroup (four 16x4 wave strips), XCD-grouped tile order;
//                                 primary ray -> Trace -> accumulate -> tonemap -> RGB8 in one
//                                 pass (PACKED=false) or the raw sample into a rank's packed
//                                 tile buffer (PACKED=true, multi-GPU).
//   composite_tiles               rank-0 unpack + accumulate + tonemap of gathered tiles.
//   find_nearest_k / is_occluded_k / trace_k   per-ray unit entries.
//   tiled_world_k / checksum_k    world generator and grid checksum.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "vpx_trace.hpp"

using namespace vpx;

namespace {

constexpr int kTile = 16;  // 16x16 pixels per workgroup
constexpr int kThreads = 256;

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
};

// --------------------------------------------------------------- primary rays
// Camera::GetPrimaryRayNoDOF (camera.h:103-110) / GetPrimaryRay + thin lens (:68-83);
// AA jitter as the AVX path: fma(rand, aa, x) (renderer.cpp:1699-1708).
__device__ __forceinline__ Ray primary_ray(const FrameArgs& f, uint32_t x, uint32_t y, Rng& g) {
    float fx = (float)x, fy = (float)y;
    if (f.flags & VPX_FLAG_AA) {
        const float rx = g.next(), ry = g.next();
        fx = fmaf(rx, f.aa, fx);
        fy = fmaf(ry, f.aa, fy);
    }
    const float u = fx * __fdiv_rn(1.0f, (float)f.width);
    const float v = fy * __fdiv_rn(1.0f, (float)f.height);
    const f3 tl = ld3(f.cam.top_left), tr = ld3(f.cam.top_right), bl = ld3(f.cam.bottom_left);
    const f3 P = (tl + (tr - tl) * u) + (bl - tl) * v;
    const f3 cp = ld3(f.cam.cam_pos);
    if (f.flags & VPX_FLAG_DOF) {
        const float rr = sqrtf(g.next());
        const float theta = g.next() * (2.0f * kPi);
        const float cx = cr_cos(theta) * rr, cy = cr_sin(theta) * rr;
        const float jx = __fdiv_rn(cx * f.cam.defocus_jitter, (float)f.width);
        const float jy = __fdiv_rn(cy * f.cam.defocus_jitter, (float)f.width);
        const f3 focal = cp + normalize(P - cp) * f.cam.focal_distance;
        const f3 o = (cp + ld3(f.cam.right) * jx) + ld3(f.cam.up) * jy;
        return make_ray(o, focal - o);
    }
    return make_ray(cp, P - cp);
}

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

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// One 64-bit atomic per counter per wave: [0] shadow rays, [1] FindNearest calls,
// [2] DDA cells, [3] primary rays.
__device__ __forceinline__ void flush_counters(Counters k, uint32_t primary, unsigned long long* ctr) {
    const uint32_t sh = wave_sum(k.shadow), ne = wave_sum(k.nearest), ce = wave_sum(k.cells);
    const uint32_t pr = wave_sum(primary);
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&ctr[0], (unsigned long long)sh);
        atomicAdd(&ctr[1], (unsigned long long)ne);
        atomicAdd(&ctr[2], (unsigned long long)ce);
        atomicAdd(&ctr[3], (unsigned long long)pr);
    }
}

// XCD-grouped workgroup order: hardware deals consecutive workgroups round-robin over the
// 8 XCDs; hand each XCD a contiguous run of tiles so neighbouring tiles (which walk the
// same voxels) share that XCD's L2.  Speed only — any mapping is correct.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t nb) {
    const uint32_t full = nb & ~7u;
    if (b >= full) return b;
    const uint32_t per = full >> 3;
    return (b & 7u) * per + (b >> 3);
}

template <int LEVELS, bool PACKED>
__global__ __launch_bounds__(kThreads) void render_tiles(SceneView sv, FrameArgs f, float4* __restrict__ accum,
                                                         uint32_t* __restrict__ rgb8, float4* __restrict__ packed,
                                                         unsigned long long* __restrict__ ctr) {
    const uint32_t nb = gridDim.x;
    const uint32_t j = xcd_remap(blockIdx.x, nb);  // this rank's j-th tile
    const uint32_t tile = PACKED ? f.rank + j * f.n_ranks : j;
    Counters k{0u, 0u, 0u};
    // wave w of the workgroup takes rows 4w..4w+3 of the 16x16 tile (16x4 strip)
    const uint32_t lx = threadIdx.x & 15u, ly = threadIdx.x >> 4;
    const uint32_t x = (tile % f.tiles_x) * kTile + lx;
    const uint32_t y = (tile / f.tiles_x) * kTile + ly;
    const bool valid = tile < f.num_tiles && x < f.width && y < f.height;
    f3 v = mk(0.f, 0.f, 0.f);
    if (valid) {
        Rng g{pixel_seed(f.seed_base, f.frame_index, f.width, f.height, x, y)};
        const Ray r = primary_ray(f, x, y, g);
        v = trace_path<LEVELS>(sv, r, f.max_bounces, g, k);
    }
    if (PACKED) {
        if (j < f.tiles_per_rank)
            packed[(uint64_t)j * (kTile * kTile) + threadIdx.x] = make_float4(v.x, v.y, v.z, 0.0f);
    } else if (valid) {
        const uint64_t p = (uint64_t)y * f.width + x;
        if (f.flags & VPX_FLAG_NO_TONEMAP) {
            accum[p] = make_float4(v.x, v.y, v.z, 0.0f);
        } else {
            const float4 a = blend(accum[p], v, f.weight, f.inv_weight);
            accum[p] = a;
            if (rgb8) rgb8[p] = tonemap_pack(a);
        }
    }
    flush_counters(k, valid ? 1u : 0u, ctr);
}

__global__ __launch_bounds__(kThreads) void composite_tiles(FrameArgs f, const float4* __restrict__ gathered,
                                                            float4* __restrict__ accum, uint32_t* __restrict__ rgb8) {
    const uint32_t tile = blockIdx.x;
    const uint32_t lx = threadIdx.x & 15u, ly = threadIdx.x >> 4;
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

template <int LEVELS>
__global__ void trace_k(SceneView sv, const vpx_ray* rays, const uint32_t* seeds, uint32_t n, int32_t depth,
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
        const WalkResult w = dda_walk<kNearest>(g, s, r.t, cells);
        if (w.hit) r.t = w.t;
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
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    struct GridBuf {
        uint8_t* ptr = nullptr;
        uint32_t n = 0;
    };
    std::vector<GridBuf> grids;
    DevGrid* d_grids = nullptr;
    uint32_t d_grids_cap = 0;
    std::vector<vpx_volume> volumes;
    vpx_volume* d_volumes = nullptr;
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
    unsigned long long* d_ctr = nullptr;  // [0] shadow, [1] nearest calls, [2] cells, [3] primary
    unsigned long long* d_sum = nullptr;
    void* d_scratch = nullptr;
    size_t scratch_bytes = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
};

namespace {

int fail(vpx_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

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
    for (uint32_t i = 0; i < n; ++i) h[i] = DevGrid{c->grids[i].ptr, c->grids[i].n, 0};
    if (n) VPX_HIP(c, hipMemcpy(c->d_grids, h.data(), sizeof(DevGrid) * n, hipMemcpyHostToDevice));
    return VPX_OK;
}

SceneView view_of(const vpx_ctx* c, const float sky[3], int32_t area_samples) {
    SceneView sv;
    sv.grids = c->d_grids;
    sv.volumes = c->d_volumes;
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
    return f;
}

int validate_frame(vpx_ctx* c, const vpx_frame_params* p) {
    if (!p) return fail(c, VPX_E_INVALID, "null frame params");
    if (p->width == 0 || p->height == 0 || p->width > 32768 || p->height > 32768)
        return fail(c, VPX_E_INVALID, "frame size out of range");
    if (p->max_bounces < -1 || p->max_bounces > kMaxLevels - 2)
        return fail(c, VPX_E_INVALID, "max_bounces must be in [-1, 14]");
    if (p->area_samples < 0 || p->area_samples > 1024) return fail(c, VPX_E_INVALID, "area_samples out of range");
    if (!c->have_camera) return fail(c, VPX_E_STATE, "no camera set (vpx_set_camera)");
    return check_ready(c);
}

template <bool PACKED>
void launch_render(vpx_ctx* c, const SceneView& sv, const FrameArgs& f, uint32_t blocks, float4* accum,
                   uint32_t* rgb8, float4* packed) {
    const dim3 grid(blocks), block(kThreads);
    if (f.max_bounces <= 0)
        hipLaunchKernelGGL((render_tiles<1, PACKED>), grid, block, 0, c->stream, sv, f, accum, rgb8, packed, c->d_ctr);
    else if (f.max_bounces <= 4)
        hipLaunchKernelGGL((render_tiles<5, PACKED>), grid, block, 0, c->stream, sv, f, accum, rgb8, packed, c->d_ctr);
    else
        hipLaunchKernelGGL((render_tiles<kMaxLevels, PACKED>), grid, block, 0, c->stream, sv, f, accum, rgb8, packed,
                           c->d_ctr);
}

int snapshot_counters(vpx_ctx* c, unsigned long long out[4]) {
    VPX_HIP(c, hipMemcpyAsync(out, c->d_ctr, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
    VPX_HIP(c, hipStreamSynchronize(c->stream));
    return VPX_OK;
}

void fill_stats(vpx_stats* s, const unsigned long long a[4], const unsigned long long b[4]) {
    s->shadow_rays = b[0] - a[0];
    s->primary_rays = b[3] - a[3];
    s->bounce_rays = (b[1] - a[1]) - s->primary_rays;
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
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&c->d_ctr, 4 * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&c->d_sum, sizeof(unsigned long long)) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipEventCreate(&c->ev2) != hipSuccess) {
        vpx_destroy(c);
        return VPX_E_DEVICE;
    }
    c->stream = c->own_stream;
    (void)hipMemset(c->d_ctr, 0, 4 * sizeof(unsigned long long));
    *out = c;
    return VPX_OK;
}

int vpx_destroy(vpx_ctx* c) {
    if (!c) return VPX_E_INVALID;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (auto& g : c->grids)
        if (g.ptr) (void)hipFree(g.ptr);
    void* ptrs[] = {c->d_grids, c->d_volumes, c->d_materials, c->d_points, c->d_spots, c->d_areas,
                    c->d_spheres, c->d_triangles, c->d_ctr, c->d_sum, c->d_scratch};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
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
    c->stream = s ? (hipStream_t)s : c->own_stream;
    return VPX_OK;
}

int vpx_synchronize(vpx_ctx* c) {
    if (!c) return VPX_E_INVALID;
    VPX_HIP(c, hipStreamSynchronize(c->stream));
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
        VPX_HIP(c, hipStreamSynchronize(c->stream));
        (void)hipFree(g.ptr);
        g.ptr = nullptr;
    }
    if (!g.ptr) VPX_HIP(c, hipMalloc(&g.ptr, bytes));
    g.n = n;
    return sync_grids(c);
}

int vpx_upload_grid(vpx_ctx* c, uint32_t id, const uint8_t* cells, uint32_t n) {
    if (!c || !cells) return fail(c, VPX_E_INVALID, "null argument");
    int rc = alloc_grid(c, id, n);
    if (rc) return rc;
    VPX_HIP(c, hipMemcpy(c->grids[id].ptr, cells, (size_t)n * n * n, hipMemcpyHostToDevice));
    return VPX_OK;
}

int vpx_generate_tiled_grid(vpx_ctx* c, uint32_t id, uint32_t n, const uint8_t* model, uint32_t mx, uint32_t my,
                            uint32_t mz, uint32_t px, uint32_t py, uint32_t pz, uint32_t ground) {
    if (!c || !model) return fail(c, VPX_E_INVALID, "null argument");
    if (!mx || !my || !mz || !px || !py || !pz) return fail(c, VPX_E_INVALID, "zero model size or period");
    int rc = alloc_grid(c, id, n);
    if (rc) return rc;
    const size_t mbytes = (size_t)mx * my * mz;
    uint8_t* dm = nullptr;
    VPX_HIP(c, hipMalloc(&dm, mbytes));
    VPX_HIP(c, hipMemcpy(dm, model, mbytes, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(tiled_world_k, dim3(4096), dim3(256), 0, c->stream, c->grids[id].ptr, n, dm, mx, my, mz, px,
                       py, pz, ground);
    VPX_HIP(c, hipGetLastError());
    VPX_HIP(c, hipStreamSynchronize(c->stream));
    (void)hipFree(dm);
    return VPX_OK;
}

int vpx_grid_checksum(vpx_ctx* c, uint32_t id, uint64_t* out) {
    if (!c || !out) return fail(c, VPX_E_INVALID, "null argument");
    if (id >= c->grids.size() || !c->grids[id].ptr) return fail(c, VPX_E_INVALID, "unknown grid");
    const uint64_t count = (uint64_t)c->grids[id].n * c->grids[id].n * c->grids[id].n;
    VPX_HIP(c, hipMemsetAsync(c->d_sum, 0, sizeof(unsigned long long), c->stream));
    hipLaunchKernelGGL(checksum_k, dim3(2048), dim3(256), 0, c->stream, c->grids[id].ptr, count, c->d_sum);
    VPX_HIP(c, hipGetLastError());
    unsigned long long h = 0;
    VPX_HIP(c, hipMemcpyAsync(&h, c->d_sum, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    VPX_HIP(c, hipStreamSynchronize(c->stream));
    *out = (uint64_t)h;
    return VPX_OK;
}

int vpx_set_volumes(vpx_ctx* c, const vpx_volume* v, uint32_t count) {
    if (!c || (!v && count)) return fail(c, VPX_E_INVALID, "null argument");
    if (count > 65536) return fail(c, VPX_E_INVALID, "too many volumes");
    VPX_HIP(c, hipStreamSynchronize(c->stream));
    if (count > c->d_volumes_cap) {
        if (c->d_volumes) (void)hipFree(c->d_volumes);
        c->d_volumes = nullptr;
        VPX_HIP(c, hipMalloc(&c->d_volumes, sizeof(vpx_volume) * count));
        c->d_volumes_cap = count;
    }
    c->volumes.assign(v, v + count);
    if (count) VPX_HIP(c, hipMemcpy(c->d_volumes, v, sizeof(vpx_volume) * count, hipMemcpyHostToDevice));
    return VPX_OK;
}

int vpx_set_materials(vpx_ctx* c, const vpx_material* m, uint32_t count) {
    if (!c || !m) return fail(c, VPX_E_INVALID, "null argument");
    if (count == 0 || count > VPX_NUM_MATERIALS) return fail(c, VPX_E_INVALID, "material count must be 1..256");
    vpx_material full[VPX_NUM_MATERIALS];
    // entries past `count` behave like MaterialSetUp's padding: white, roughness 1
    for (auto& e : full) e = vpx_material{{1, 1, 1}, 1.0f, 0.0f, 1.5f, {0, 0}};
    std::memcpy(full, m, sizeof(vpx_material) * count);
    VPX_HIP(c, hipStreamSynchronize(c->stream));
    int rc = upload_table(c, c->d_materials, full, VPX_NUM_MATERIALS);
    if (rc) return rc;
    VPX_HIP(c, hipStreamSynchronize(c->stream));
    c->have_materials = true;
    return VPX_OK;
}

int vpx_set_lights(vpx_ctx* c, const vpx_point_light* p, uint32_t np, const vpx_spot_light* s, uint32_t ns,
                   const vpx_area_light* a, uint32_t na, const vpx_dir_light* d) {
    if (!c) return VPX_E_INVALID;
    VPX_HIP(c, hipStreamSynchronize(c->stream));
    int rc;
    if ((rc = upload_table(c, c->d_points, p, np))) return rc;
    if ((rc = upload_table(c, c->d_spots, s, ns))) return rc;
    if ((rc = upload_table(c, c->d_areas, a, na))) return rc;
    VPX_HIP(c, hipStreamSynchronize(c->stream));
    c->n_points = np, c->n_spots = ns, c->n_areas = na;
    if (d) c->dir = *d;
    return VPX_OK;
}

int vpx_set_shapes(vpx_ctx* c, const vpx_sphere* s, uint32_t ns, const vpx_triangle* t, uint32_t nt) {
    if (!c) return VPX_E_INVALID;
    VPX_HIP(c, hipStreamSynchronize(c->stream));
    int rc;
    if ((rc = upload_table(c, c->d_spheres, s, ns))) return rc;
    if ((rc = upload_table(c, c->d_triangles, t, nt))) return rc;
    VPX_HIP(c, hipStreamSynchronize(c->stream));
    c->n_spheres = ns, c->n_triangles = nt;
    return VPX_OK;
}

int vpx_set_camera(vpx_ctx* c, const vpx_camera* cam) {
    if (!c || !cam) return fail(c, VPX_E_INVALID, "null argument");
    c->cam = *cam;
    c->have_camera = true;
    return VPX_OK;
}

int vpx_render(vpx_ctx* c, const vpx_frame_params* p, float* accum, uint32_t* rgb8, vpx_stats* stats) {
    if (!c) return VPX_E_INVALID;
    int rc = validate_frame(c, p);
    if (rc) return rc;
    if (!accum) return fail(c, VPX_E_INVALID, "accum (device float4[W*H]) is required");
    VPX_HIP(c, hipSetDevice(c->device));
    unsigned long long before[4] = {0, 0, 0, 0};
    if (stats && (rc = snapshot_counters(c, before))) return rc;
    const SceneView sv = view_of(c, p->sky, p->area_samples);
    const FrameArgs f = frame_of(c, p, 0, 1);
    if (stats) VPX_HIP(c, hipEventRecord(c->ev0, c->stream));
    launch_render<false>(c, sv, f, f.num_tiles, reinterpret_cast<float4*>(accum), rgb8, nullptr);
    VPX_HIP(c, hipGetLastError());
    if (stats) {
        VPX_HIP(c, hipEventRecord(c->ev1, c->stream));
        unsigned long long after[4];
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

int vpx_render_tiles(vpx_ctx* c, const vpx_frame_params* p, uint32_t tile_w, uint32_t tile_h, uint32_t rank,
                     uint32_t n_ranks, float* packed, vpx_stats* stats) {
    if (!c) return VPX_E_INVALID;
    int rc = validate_frame(c, p);
    if (rc) return rc;
    if (tile_w != kTile || tile_h != kTile) return fail(c, VPX_E_INVALID, "tiles must be 16x16");
    if (n_ranks == 0 || rank >= n_ranks || !packed) return fail(c, VPX_E_INVALID, "bad rank / packed buffer");
    VPX_HIP(c, hipSetDevice(c->device));
    unsigned long long before[4] = {0, 0, 0, 0};
    if (stats && (rc = snapshot_counters(c, before))) return rc;
    const SceneView sv = view_of(c, p->sky, p->area_samples);
    const FrameArgs f = frame_of(c, p, rank, n_ranks);
    if (stats) VPX_HIP(c, hipEventRecord(c->ev0, c->stream));
    launch_render<true>(c, sv, f, f.tiles_per_rank, nullptr, nullptr, reinterpret_cast<float4*>(packed));
    VPX_HIP(c, hipGetLastError());
    if (stats) {
        VPX_HIP(c, hipEventRecord(c->ev1, c->stream));
        unsigned long long after[4];
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

int vpx_composite_tiles(vpx_ctx* c, const vpx_frame_params* p, uint32_t tile_w, uint32_t tile_h, uint32_t n_ranks,
                        const float* gathered, float* accum, uint32_t* rgb8) {
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
    unsigned long long now[4];
    int rc = snapshot_counters(c, now);
    if (rc) return rc;
    const unsigned long long zero[4] = {0, 0, 0, 0};
    std::memset(out, 0, sizeof(*out));
    fill_stats(out, zero, now);
    if (reset) {
        VPX_HIP(c, hipMemsetAsync(c->d_ctr, 0, 4 * sizeof(unsigned long long), c->stream));
        VPX_HIP(c, hipStreamSynchronize(c->stream));
    }
    return VPX_OK;
}

int vpx_find_nearest(vpx_ctx* c, const vpx_ray* rays, uint32_t n, vpx_hit* hits) {
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
    VPX_HIP(c, hipStreamSynchronize(c->stream));
    return VPX_OK;
}

int vpx_is_occluded(vpx_ctx* c, const vpx_ray* rays, uint32_t n, uint8_t* occ) {
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
    VPX_HIP(c, hipStreamSynchronize(c->stream));
    return VPX_OK;
}

int vpx_trace(vpx_ctx* c, const vpx_ray* rays, const uint32_t* seeds, uint32_t n, int32_t depth, const float sky[3],
              int32_t area_samples, float* radiance) {
    if (!c || (n && (!rays || !seeds || !radiance)) || !sky) return fail(c, VPX_E_INVALID, "null argument");
    if (depth < -1 || depth > kMaxLevels - 2) return fail(c, VPX_E_INVALID, "depth must be in [-1, 14]");
    int rc = check_ready(c);
    if (rc) return rc;
    if (n == 0) return VPX_OK;
    const size_t rb = sizeof(vpx_ray) * n, sb = 4ull * n, ob = 12ull * n;
    if ((rc = ensure_scratch(c, rb + sb + ob))) return rc;
    vpx_ray* dr = (vpx_ray*)c->d_scratch;
    uint32_t* ds = (uint32_t*)((char*)c->d_scratch + rb);
    float* dout = (float*)((char*)c->d_scratch + rb + sb);
    VPX_HIP(c, hipMemcpyAsync(dr, rays, rb, hipMemcpyHostToDevice, c->stream));
    VPX_HIP(c, hipMemcpyAsync(ds, seeds, sb, hipMemcpyHostToDevice, c->stream));
    const SceneView sv = view_of(c, sky, area_samples);
    const dim3 g((n + 255) / 256), b(256);
    if (depth <= 0)
        hipLaunchKernelGGL(trace_k<1>, g, b, 0, c->stream, sv, dr, ds, n, depth, dout);
    else if (depth <= 4)
        hipLaunchKernelGGL(trace_k<5>, g, b, 0, c->stream, sv, dr, ds, n, depth, dout);
    else
        hipLaunchKernelGGL(trace_k<kMaxLevels>, g, b, 0, c->stream, sv, dr, ds, n, depth, dout);
    VPX_HIP(c, hipGetLastError());
    VPX_HIP(c, hipMemcpyAsync(radiance, dout, ob, hipMemcpyDeviceToHost, c->stream));
    VPX_HIP(c, hipStreamSynchronize(c->stream));
    return VPX_OK;
}

int vpx_focus_distance(vpx_ctx* c, uint32_t width, uint32_t height, float* fd) {
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
    VPX_HIP(c, hipStreamSynchronize(c->stream));
    return VPX_OK;
}

uint32_t vpx_pixel_seed(uint32_t base, uint32_t frame, uint32_t w, uint32_t h, uint32_t x, uint32_t y) {
    return pixel_seed(base, frame, w, h, x, y);
}

}  // extern "C"
