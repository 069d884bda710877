/*
 * vpx_oracle.h — CPU restatement of the reference per-pixel ray-trace path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the checker for libvpx_hip.so: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The product
 * path never links, calls or falls back to it.
 *
 * Parity status: UNPINNED for the trace path.  The reference (Windows/MSVC C++) cannot
 * be compiled in this image without stand-ins for <windows.h>, <io.h>, <intrin.h> and
 * SVML, which the build rules forbid, and the reference ships no tests, fixtures or
 * golden vectors for this path.  The restatement follows the reference
 * source expression by expression (file:line cited per function); see DESIGN.md §3 for
 * the parity-hazard decisions (exact 1/x instead of rcpps, left-to-right argument
 * order, correctly rounded transcendentals, FTZ/DAZ).  The .vox decode feeding the
 * worlds IS pinned: tests/golden/<model>.npz are produced by the reference's own vendored
 * ogt_vox v0.997 (lib/ogt_vox.h) compiled where it lies (oracle/Makefile, _ref/).
 */
#ifndef VPX_ORACLE_H_
#define VPX_ORACLE_H_

#include "../include/vpx.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_grid {
    const uint8_t* cells;
    uint32_t n;
} oracle_grid;

typedef struct oracle_scene {
    const oracle_grid* grids;
    uint32_t num_grids;
    const vpx_volume* volumes;
    uint32_t num_volumes;
    const vpx_material* materials;  /* 256 entries */
    const vpx_point_light* points;
    uint32_t num_points;
    const vpx_spot_light* spots;
    uint32_t num_spots;
    const vpx_area_light* areas;
    uint32_t num_areas;
    vpx_dir_light dir;
    const vpx_sphere* spheres;
    uint32_t num_spheres;
    const vpx_triangle* triangles;
    uint32_t num_triangles;
    vpx_camera camera;
    /* sky dome (vpx_set_sky): RGB float texels, NULL = none */
    const float* sky_pixels;
    uint32_t sky_w, sky_h;
    float sky_hdr;
} oracle_scene;

/* Renderer::FindNearest per ray (renderer.cpp:946-1018). */
int oracle_find_nearest(const oracle_scene* sc, const vpx_ray* rays, uint32_t n, vpx_hit* hits);
/* Renderer::IsOccluded per ray (renderer.cpp:209-243). cells may be NULL. */
int oracle_is_occluded(const oracle_scene* sc, const vpx_ray* rays, uint32_t n,
                       uint8_t* occluded, uint32_t* cells);
/* Renderer::Trace(ray, depth) per ray with an explicit xorshift32 state; sky NULL =
   the scene's sky texture (activateSky). */
int oracle_trace(const oracle_scene* sc, const vpx_ray* rays, const uint32_t* seeds, uint32_t n,
                 int32_t depth, const float sky[3], int32_t area_samples, float* radiance,
                 vpx_stats* stats);
/* New per-pixel sample (float4, w = 0) for the listed pixel ids (y*W + x), as vpx_render
   computes it before accumulation.  threads <= 0: all hardware threads. */
int oracle_render_pixels(const oracle_scene* sc, const vpx_frame_params* p,
                         const uint32_t* pixel_ids, uint32_t n, float* sample4,
                         vpx_stats* stats, int threads);
/* Whole frame: sample + accumulate + tonemap (Renderer::Update, renderer.cpp:1646-1891).
   accum float4[W*H] in/out, rgb8 uint32[W*H] out. */
int oracle_render(const oracle_scene* sc, const vpx_frame_params* p, float* accum,
                  uint32_t* rgb8, vpx_stats* stats, int threads);
/* Rank-0 epilogue on one pixel sample (accumulate + Reinhard-Jodie + RGB8). */
void oracle_accumulate_tonemap(const float* sample4, uint32_t frame_index, float* acc4,
                               uint32_t* rgb8);
/* Focus ray of Renderer::Tick (renderer.cpp:1987-1991). */
float oracle_focus_distance(const oracle_scene* sc, uint32_t width, uint32_t height);

/* ---- worlds ---------------------------------------------------------------------- */
/* Scene::LoadModel placement (template/scene.cpp:449-529) of an ogt-decoded model
   (voxel_data index x + y*sx + z*sx*sy, 0 = empty) into an N^3 grid (out: N^3 bytes,
   reset to NONE first).  scale_model = Scene::scaleModel on entry (normally 1,1,1). */
void oracle_load_model(const uint8_t* voxels, uint32_t sx, uint32_t sy, uint32_t sz,
                       uint32_t n, const float scale_model[3], uint8_t* out);
/* Grid-orient an ogt model (x, y, z) -> (x, z, y) as LoadModel does, no scaling. */
void oracle_orient_model(const uint8_t* voxels, uint32_t sx, uint32_t sy, uint32_t sz,
                         uint8_t* out /* sx*sz*sy, index x + y*sx + z*sx*sz */);
/* Build-defined tiled world; same contract as vpx_generate_tiled_grid. */
void oracle_tiled_world(const uint8_t* model, uint32_t mx, uint32_t my, uint32_t mz,
                        uint32_t px, uint32_t py, uint32_t pz, uint32_t ground, uint32_t n,
                        uint8_t* out);
uint64_t oracle_grid_checksum(const uint8_t* cells, uint64_t count);

/* ---- math pieces exposed for known-answer tests --------------------------------- */
uint32_t oracle_wang_hash(uint32_t s);
uint32_t oracle_xorshift32(uint32_t* state);
float oracle_random_float(uint32_t* state);
uint32_t oracle_pixel_seed(uint32_t seed_base, uint32_t frame_index, uint32_t width,
                           uint32_t height, uint32_t x, uint32_t y);
void oracle_offset_ray(const float p[3], const float n[3], float out[3]);
float oracle_cube_intersect(const float b0[3], const float b1[3], const float o[3],
                            const float d[3], const float rd[3]);

/* Static-camera path: one frame of Renderer::Tick's static branch
   (renderer.cpp:1996-2101) — TraceReproject per pixel, reprojection into `prev`, history
   blend.  history: float4[W*H] in/out (illuminationHistoryBuffer); rgb8 may be NULL. */
int oracle_render_reproject(const oracle_scene* sc, const vpx_frame_params* p, const vpx_prev_camera* prev,
                            float* history, uint32_t* rgb8, vpx_stats* stats, int threads);

/* World edits: Scene::LoadModelPartial / CreateEmmisiveSphere. */
void oracle_load_model_partial(const uint8_t* vox, uint32_t sx, uint32_t sy, uint32_t sz, uint32_t n,
                               const float scale_model[3], uint32_t columns, uint32_t thickness, uint8_t* out);
void oracle_emissive_sphere(uint8_t* grid, uint32_t n, uint8_t mat, float radius);

/* BasicBVH (src/BVH/BasicBVH.{h,cpp}): the constructor's random triangle
   set (returns the RNG state after), BuildBVH (returns nodes used; nodes: 2n-1 entries,
   tri_idx: n) and IntersectBVH(ray, 0) per ray (t_out = ray.t afterwards; rays built as
   oracle_find_nearest builds them).  nodes == NULL: no BVH, t_out = tmax. */
uint32_t oracle_bvh_random_tris(uint32_t seed, vpx_bvh_tri* out);
uint32_t oracle_bvh_build(const vpx_bvh_tri* tris, uint32_t n, vpx_bvh_node* nodes, uint32_t* tri_idx);
int oracle_bvh_intersect(const vpx_bvh_node* nodes, const vpx_bvh_tri* tris, const uint32_t* tri_idx,
                         const vpx_ray* rays, uint32_t n, float* t_out);

/* The reference's x86 approximations on/off (FastReciprocal in FindNearest, rsqrtps in the
   primary normalize); off by default.  Process-global; -1 on a non-x86 host. */
int oracle_set_x86_approx(int on);
/* Known-answer hooks (tests/test_kat_reference.py): GetNormalVoxel of the ray (o, d) at t;
   one light evaluator at a hit; Schlick / SchlickNonMetal / Refract / Absorption / Reflect. */
int oracle_kat_normal(const float o[3], const float d[3], float t, uint32_t n, const float m[16], float out[3]);
int oracle_kat_light(const oracle_scene* sc, int kind, uint32_t index, const float o[3], const float d[3], float t,
                     const float nrm[3], uint32_t mat, int32_t area_samples, uint32_t* rng, float out[3]);
int oracle_kat_shading(int fn, const float* in, float* out);
/* sinf/cosf/expf/powf(x,5) as the restatement evaluates them (fn 0..3), for the pin test. */
void oracle_dm_eval(int fn, const float* x, float* out, uint32_t n);

#ifdef __cplusplus
}
#endif
#endif
