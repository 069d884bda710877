/*
 * vpx.h — C-ABI of the MI355X (gfx950) voxel ray-trace library `libvpx_hip.so`.
 *
 * This is the drop-in boundary behind `Renderer::Tick(deltaTime)` of
 * Tycro-Games/Raytracer-VoxPopuli.  The host keeps its tmpl8 template, window,
 * UI and game logic; inside `Renderer::Update()` it calls `vpx_render` instead
 * of the per-pixel `Trace` loop (reference renderer.cpp:1646-1891), and the
 * library owns persistent device copies of the voxel grids, the volume
 * transforms and the material / light tables.
 *
 * Every function returns VPX_OK (0) or a negative VPX_E_* status; nothing
 * throws across the ABI and nothing aborts.  `vpx_last_error(ctx)` returns a
 * human-readable message for the last failure on that context.
 *
 * All structs are plain-old-data with fixed layout (asserted in vpx_api.cpp);
 * matrices are tmpl8 `mat4::cell` order (row-major, translation in cells 3/7/11).
 *
 * Reference interfaces replaced (file:line in the reference tree):
 *   vpx_create[_multi]    Renderer::Init (device side) renderer.cpp:688-736
 *   vpx_render            Renderer::Update            renderer.cpp:1646-1891
 *                         (+ Renderer::Trace           renderer.cpp:1076-1328)
 *   vpx_find_nearest      Renderer::FindNearest       renderer.cpp:946-1018
 *                         Scene::FindNearest          template/scene.cpp:751-811
 *   vpx_is_occluded       Renderer::IsOccluded        renderer.cpp:209-243
 *                         Scene::IsOccluded           template/scene.cpp:1009-1047
 *   vpx_trace             Renderer::Trace(Ray&, int)  renderer.cpp:1076
 *   vpx_focus_distance    focus ray in Renderer::Tick renderer.cpp:1987-1991
 *   vpx_upload_grid       Scene::grid (owned by host) template/scene.h:258
 *   vpx_set_volumes       Renderer::voxelVolumes      renderer.h:211
 *   vpx_set_materials     Renderer::materials         renderer.h:190, MaterialSetUp renderer.cpp:357-443
 *   vpx_set_lights        point/spot/area/dirLight    renderer.h:193-197
 *   vpx_set_shapes        Renderer::spheres/triangles renderer.h:207-208
 *   vpx_set_camera        Renderer::camera            renderer.h:181, template/camera.h:14-192
 *   vpx_set_sky           Renderer::skyPixels (+ SampleSky) renderer.cpp:691, 2308-2326
 *   vpx_bvh_set           Renderer::bvh (BasicBVH)    renderer.h:220, src/BVH/BasicBVH.cpp:72-136
 *   vpx_bvh_intersect     BasicBVH::IntersectBVH      src/BVH/BasicBVH.cpp:19-70
 * Host-side helpers that restate reference host code (no GPU needed):
 *   vpx_camera_look_at       Camera::HandleInput basis   template/camera.h:113-181
 *   vpx_volume_set_transform Scene::SetTransform         template/scene.cpp:373-405
 *   vpx_default_materials    Renderer::MaterialSetUp     renderer.cpp:357-443
 *   vpx_bvh_build_host       BasicBVH::BuildBVH          src/BVH/BasicBVH.cpp:72-136
 *   vpx_bvh_random_tris      BasicBVH::BasicBVH()        src/BVH/BasicBVH.cpp:4-16
 *   vpx_bvh_depth            (recursion depth of IntersectBVH, src/BVH/BasicBVH.cpp:47-61)
 *   vpx_vox_decode           ogt_vox_read_scene ->models[0], ->palette, template/scene.cpp:474-475
 */
#ifndef VPX_H_
#define VPX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VPX_ABI_VERSION 2  /* 1 -> 2: vpx_profile grew to 160 bytes (stage_busy_ms); packed tiles hold 8x8 quadrants */

/* ---- status codes ---------------------------------------------------------------- */
#define VPX_OK 0
#define VPX_E_INVALID (-1)   /* bad argument (null pointer, size, id)           */
#define VPX_E_DEVICE (-2)    /* HIP runtime error                              */
#define VPX_E_NOMEM (-3)     /* device allocation failed                       */
#define VPX_E_STATE (-4)     /* call order (e.g. render before any volume)     */

/* ---- material indices (MaterialType::MatType, template/scene.h:36-58) ------------- */
#define VPX_MAT_NON_METAL_WHITE 0
#define VPX_MAT_NON_METAL_PINK 4
#define VPX_MAT_METAL_HIGH 5
#define VPX_MAT_METAL_LOW 7
#define VPX_MAT_GLASS 8
#define VPX_MAT_SMOKE_LOW_DENSITY 9
#define VPX_MAT_SMOKE_PLAYER 14
#define VPX_MAT_EMISSIVE 15
#define VPX_MAT_NONE 255
#define VPX_NUM_MATERIALS 256

/* ---- frame flags -------------------------------------------------------------------- */
#define VPX_FLAG_AA 0x1u        /* sub-pixel jitter x+RandomFloat()*aa (renderer.cpp:1682-1708)   */
#define VPX_FLAG_DOF 0x2u       /* thin-lens jitter (template/camera.h:68-83)                    */
#define VPX_FLAG_NO_TONEMAP 0x4u /* skip accumulate/tonemap: write raw radiance to accum (tests) */
#define VPX_FLAG_SKY 0x8u       /* activateSky: misses sample the vpx_set_sky texture (renderer.cpp:2308-2326) */

/* ---- POD scene description -------------------------------------------------------- */

/* One voxel volume (a `Scene` in the reference, template/scene.h:173-266). */
typedef struct vpx_volume {
    uint32_t grid_id;       /* grid uploaded with vpx_upload_grid; volumes may share a grid */
    uint32_t reserved;
    float matrix[16];       /* Scene::matrix    (object -> world)                */
    float inv_matrix[16];   /* Scene::invMatrix (world -> object) — used as-is    */
    float b0[3];            /* Scene::cube.b[0]                                  */
    float b1[3];            /* Scene::cube.b[1]                                  */
} vpx_volume;               /* 160 bytes */

/* Material (src/Materials/Material.h:3-12), indexed by voxel value. */
typedef struct vpx_material {
    float albedo[3];
    float roughness;
    float emissive;         /* emissiveStrength */
    float ior;              /* IOR */
    float pad[2];
} vpx_material;             /* 32 bytes */

typedef struct vpx_point_light {  /* PointLightData, src/Lighting/PointLight.h:3-7 */
    float position[3];
    float color[3];
} vpx_point_light;

typedef struct vpx_spot_light {   /* SpotLightData, src/Lighting/SpotLight.h:12-18 */
    float position[3];
    float direction[3];
    float color[3];
    float angle;                  /* cosine of the cone half-angle */
} vpx_spot_light;

typedef struct vpx_area_light {   /* SphereAreaLightData, src/Lighting/SphereAreaLight.h:2-9 */
    float position[3];
    float color[3];
    float color_multiplier;
    float radius;
} vpx_area_light;

typedef struct vpx_dir_light {    /* DirectionalLightData, src/Lighting/DirectionalLight.h:2-6 */
    float direction[3];
    float color[3];
} vpx_dir_light;

typedef struct vpx_sphere {       /* Sphere, src/BVH/Shapes.h:4-68 */
    float center[3];
    float radius;
    uint32_t material;
    uint32_t pad[3];
} vpx_sphere;

typedef struct vpx_triangle {     /* Triangle, src/BVH/Shapes.h:71-150 */
    float position[3];
    float v0[3], v1[3], v2[3];
    uint32_t material;
    uint32_t pad[3];
} vpx_triangle;

/* Camera state used by primary-ray generation (template/camera.h:68-110, 183-191). */
typedef struct vpx_camera {
    float cam_pos[3];
    float top_left[3];
    float top_right[3];
    float bottom_left[3];
    float right[3];
    float up[3];
    float focal_distance;
    float defocus_jitter;
} vpx_camera;

/* Per-frame parameters (the knobs of Renderer::Update / Trace). */
typedef struct vpx_frame_params {
    uint32_t width, height;       /* SCRWIDTH/SCRHEIGHT (compile-time in the reference);    */
                                  /* each <= 32768, 16x16-tile-padded W*H <= 2^27           */
    int32_t max_bounces;          /* depth handed to Trace (Renderer::maxBounces)           */
    uint32_t frame_index;         /* numRenderedFrames: weight 1/(n+1) and seed stream      */
    uint32_t seed_base;           /* added to the pixel key of the per-pixel seed           */
    uint32_t flags;               /* VPX_FLAG_*                                             */
    float aa_strength;            /* antiAliasingStrength                                   */
    int32_t area_samples;         /* numCheckShadowsAreaLight                               */
    float sky[3];                 /* SampleSky colour when activateSky == false             */
    uint32_t reserved;
} vpx_frame_params;

/* Ray for the unit entries (a `Ray` built with Ray(origin, direction), scene.cpp:83-93). */
typedef struct vpx_ray {
    float origin[3];
    float direction[3];           /* normalised by the library exactly like the Ray ctor   */
    float tmax;                   /* Ray::t on entry (1e34 = unbounded)                     */
    uint32_t inside_glass;        /* Ray::isInsideGlass                                     */
} vpx_ray;

typedef struct vpx_hit {
    float t;                      /* Ray::t after the call                                  */
    float normal[3];              /* Ray::rayNormal                                         */
    int32_t vox_index;            /* Renderer::FindNearest return: -2 none, -1 analytic, i  */
    uint32_t material;            /* Ray::indexMaterial (255 = NONE)                        */
    uint32_t cells;               /* DDA cells read for this ray                            */
    uint32_t inside_glass;        /* Ray::isInsideGlass after the call                      */
} vpx_hit;

/* Work counters of one render call (always on; per-wave reduced on device). */
typedef struct vpx_stats {
    uint64_t primary_rays;        /* W*H                                                     */
    uint64_t shadow_rays;         /* IsOccluded calls actually made                          */
    uint64_t bounce_rays;         /* FindNearest calls beyond the primary                    */
    uint64_t dda_cells;           /* grid cells read by every DDA (nearest + shadow + exits) */
    float kernel_ms;              /* device time of the trace kernel (HIP events)            */
    float total_ms;               /* device time of the whole call                           */
} vpx_stats;

typedef struct vpx_ctx vpx_ctx;

/* ---- lifetime ------------------------------------------------------------------------ */
int vpx_create(int device, vpx_ctx** out);
/* A device set for a single-process host (the tmpl8 Renderer::Tick on a multi-GPU node):
   one member context per entry of devices[0..ndev) (the world and tables are uploaded to
   every member by the same calls as for one device).  vpx_render deals the 16x16 tiles
   round-robin to the members, renders them concurrently, gathers the packed results to
   devices[0] over RCCL (one communicator per device, ncclCommInitAll; device copies when
   the set repeats a device) and composites there: with accum != NULL the float4 samples
   travel and accum / rgb8 (devices[0] pointers) are bit-identical to vpx_render on one
   device; with accum == NULL each member keeps the running average of its own tiles and
   only RGB8 travels into rgb8.  vpx_set_stream sets devices[0]'s stream; unit entries,
   profiles, vpx_render_reproject and the rank-level entries (vpx_render_tiles*,
   vpx_composite_*) run on devices[0]; vpx_get_counters sums the members.  Every call on a
   set restores the caller's current HIP device before it returns; stats (vpx_render) read
   the members' counters outside the launches, so the members still overlap.
   Verification status: sets that repeat a device (the device-copy gather) are tested bit
   for bit on one GPU; the distinct-device RCCL gather has its test
   (test_device_set_equals_single_device[devices3]) but runs only on a node with >= 2 GPUs
   and has not yet executed on hardware. */
int vpx_create_multi(const int* devices, int ndev, vpx_ctx** out);
int vpx_destroy(vpx_ctx* ctx);
const char* vpx_last_error(const vpx_ctx* ctx);
int vpx_abi_version(void);
/* Use an external HIP stream (hipStream_t as void*); NULL = the context's own stream. */
int vpx_set_stream(vpx_ctx* ctx, void* hip_stream);
int vpx_synchronize(vpx_ctx* ctx);
/* Frames in flight (depth 2..4; 0 / 1 = off, the default).  With depth D, vpx_render and
   vpx_render_tiles_accum render each frame on the next of D library-owned streams ("lanes",
   each with its own path-state buffers and its own hardware queue — CU-mask streams, outside
   the GPU_MAX_HW_QUEUES pool the caller's streams share) into packed float4 samples, and queue only the
   frame's accumulate / tonemap / RGB8 pack (or the rank's packed running average) on the
   context's stream, after the previous frame's: frame f+1's walks run while frame f's last
   tiles drain.  Results are bit-identical (the same blend of the same sample, in frame order);
   accum / rgb8 are complete when the context's stream is.  Renders that take stats, the
   static-camera path, VPX_FLAG_NO_TONEMAP frames and vpx_render_tiles (samples into the
   caller's buffer) run on the stream as without lanes.
   World / table updates wait for the frames in flight.  No reference counterpart: the
   reference renders one frame per Tick (renderer.cpp:1646-1891).
   Queues and ordering: each lane takes a hardware queue of its own (D per context, and per
   member of a device set), up to 16 such lanes per process; lanes past that cap are plain
   non-blocking streams from the process's shared queue pool.  Frames with bounce levels also
   take one more such queue per path state (the context's own, and each lane's when at most two
   lanes run a single-volume scene): the level fork, a second stream that runs a level's
   bounce walks beside its shadow walks and joins back within the frame.  Dedicated-queue lanes are
   blocking streams: they synchronise with the legacy null stream (hipStreamLegacy / torch's
   default stream), so work the caller queues there serialises with the frames in flight —
   render on a created stream (vpx_set_stream) to keep them overlapped. */
int vpx_set_pipeline(vpx_ctx* ctx, uint32_t depth);

/* ---- world ----------------------------------------------------------------------------- */
/* Upload a dense N^3 grid of MatType bytes, index x + y*N + z*N*N (scene.h:241-248).
   Device memory per grid: N^3 bytes + the walkers' levels built from them, about N^3 / 4
   bytes (l1 cell masks N^3/8, distance-field octant planes N^3/8, l2 N^3/512): 1.25 GiB
   at N = 1024, 10 GiB at 2048, 80 GiB at 4096 (the maximum). */
int vpx_upload_grid(vpx_ctx* ctx, uint32_t grid_id, const uint8_t* cells, uint32_t n);
/* Build-defined world generator on device: a grid-oriented model
   (mx*my*mz bytes, index x + y*mx + z*mx*my) tiled with period (px,py,pz) above a
   NON_METAL_WHITE ground slab of `ground` cells.  Same result as oracle_tiled_world. */
int vpx_generate_tiled_grid(vpx_ctx* ctx, uint32_t grid_id, uint32_t n, const uint8_t* model,
                            uint32_t mx, uint32_t my, uint32_t mz,
                            uint32_t px, uint32_t py, uint32_t pz, uint32_t ground);
/* In-place world edits.  Each refreshes the occupancy levels
   of the touched bricks only.
   Scene::ResetGrid(type) (template/scene.cpp:356-359): every cell = value. */
int vpx_grid_fill(vpx_ctx* ctx, uint32_t grid_id, uint8_t value);
/* Dirty-region upload: a box of cells, host bytes x fastest (src[x + y*dx + z*dx*dy]),
   written at (x0, y0, z0) — what Scene::Set-based edits change (LoadModelPartial from
   ModifyingProp::Update, src/Game/ModifyingProp.cpp:11-21; zone changes). */
int vpx_grid_write_box(vpx_ctx* ctx, uint32_t grid_id, const uint8_t* src, uint32_t x0, uint32_t y0,
                       uint32_t z0, uint32_t dx, uint32_t dy, uint32_t dz);
/* Scene::CreateEmmisiveSphere(mat, radius) (template/scene.cpp:685-711) on the device:
   cells with length(worldsize/2 - (x,y,z)) < radius get `mat` (others unchanged). */
int vpx_grid_emissive_sphere(vpx_ctx* ctx, uint32_t grid_id, uint8_t mat, float radius);
/* FNV-1a-style 64-bit checksum of a device grid (for size-independent parity checks). */
int vpx_grid_checksum(vpx_ctx* ctx, uint32_t grid_id, uint64_t* out);
int vpx_set_volumes(vpx_ctx* ctx, const vpx_volume* volumes, uint32_t count);
int vpx_set_materials(vpx_ctx* ctx, const vpx_material* materials, uint32_t count);
int vpx_set_lights(vpx_ctx* ctx,
                   const vpx_point_light* points, uint32_t n_points,
                   const vpx_spot_light* spots, uint32_t n_spots,
                   const vpx_area_light* areas, uint32_t n_areas,
                   const vpx_dir_light* dir);
int vpx_set_shapes(vpx_ctx* ctx, const vpx_sphere* spheres, uint32_t n_spheres,
                   const vpx_triangle* triangles, uint32_t n_triangles);
int vpx_set_camera(vpx_ctx* ctx, const vpx_camera* camera);
/* Sky dome: Renderer::skyPixels / skyWidth / skyHeight (stbi_loadf RGB floats of the
   equirectangular HDR, renderer.cpp:691; renderer.h:224-226) and HDRLightContribution.
   Texel (u, v) at rgb[3*(u + v*width)].  Used by SampleSky (renderer.cpp:2308-2326) when a
   frame sets VPX_FLAG_SKY, and by vpx_trace when its sky argument is NULL.
   rgb == NULL (or a zero size) removes the texture. */
int vpx_set_sky(vpx_ctx* ctx, const float* rgb, uint32_t width, uint32_t height,
                float hdr_contribution);

/* ---- arithmetic mode ----------------------------------------------------------------
   VPX_ARITH_EXACT (the default): exact 1/x and 1/sqrtf where the reference uses x86
   approximations.  VPX_ARITH_X86_HOST: the reference's own arithmetic,
   bit for bit as THIS host's CPU computes it — FastReciprocal (rcpps + one Newton step,
   renderer.cpp:929-934) for every Renderer::FindNearest volume visit (:969), and
   normalize(__m128) = v * rsqrtps(dpps(v, v, 0x7F)) (template/tmpl8math.h:2356-2360) for the
   primary directions of Renderer::Update (:1735-1765).  rcpps / rsqrtps differ between CPU
   vendors, so the call captures the host's tables (vpx_x86_arith_tables) and uploads them;
   VPX_E_STATE when the host is not x86 or its instructions do not follow the table model.
   The static-camera path's primary rays (GetPrimaryRayNoDOF, the Ray constructor) stay exact,
   as in the reference. */
#define VPX_ARITH_EXACT 0u
#define VPX_ARITH_X86_HOST 1u
int vpx_set_arithmetic(vpx_ctx* ctx, uint32_t mode);
/* Host only (no device): capture this CPU's rcpss / rsqrtss tables under FTZ | DAZ and
   spot-check the model (vpx_x86.hpp) against the instructions.  info = {rcp key shift, rsqrt
   key shift, first rsqrt entry, entries}; out (may be NULL: sizes only) receives the entries
   (cap >= info[3]).  VPX_E_STATE: not x86, or the spot check failed. */
int vpx_x86_arith_tables(uint32_t* out, uint64_t cap, uint32_t info[4]);
/* Host only: the model against this CPU's rcpss and rsqrtss for every input bit pattern in
   [lo, hi] (0, 0xffffffff = all 2^32) on `threads` threads; mismatches[0] / [1] count rcp /
   rsqrt disagreements, first_bad[] the first input of each. */
int vpx_x86_arith_verify(uint32_t lo, uint32_t hi, uint32_t threads, uint64_t mismatches[2],
                         uint32_t first_bad[2]);

/* ---- display interop ---------------------------------------------
   Replaces the per-frame host upload of Surface::pixels in GLTexture::CopyFrom
   (template/opengl.cpp:144-149, called from template/template.cpp:305).  The host creates a
   GL_PIXEL_UNPACK_BUFFER of W*H*4 bytes once and registers it with its GL context current on
   the calling thread, on this context's GPU (device set: devices[0]); gl_buffer == 0
   unregisters (vpx_destroy does too).  Per frame: vpx_gl_map returns the buffer's device
   address (ordered on the context's stream), the host passes it as `rgb8` to vpx_render or
   vpx_render_reproject, vpx_gl_unmap hands it back to GL, and glTexSubImage2D with the
   buffer bound updates the texture — the frame never crosses PCIe.  `bytes` (may be NULL)
   receives the buffer size; the host checks it against W*H*4.  Errors: VPX_E_DEVICE when
   HIP cannot register the buffer (no current GL context, another GPU), VPX_E_STATE for
   map / unmap / register out of order.  Unmeasured on hardware: no GL display here. */
int vpx_gl_register_buffer(vpx_ctx* ctx, unsigned int gl_buffer);
int vpx_gl_map(vpx_ctx* ctx, uint32_t** rgb8, size_t* bytes);
int vpx_gl_unmap(vpx_ctx* ctx);

/* ---- the hot path -------------------------------------------------------------------- */
/* One frame: primary rays, Trace(ray, max_bounces) per pixel, running-average accumulate
   (w = 1/(frame_index+1)), Reinhard-Jodie tonemap, RGB8 pack.  `accum` (float4[W*H]) and
   `rgb8` (uint32[W*H]) are DEVICE pointers; accum is read-modify-write. Either may be NULL
   when VPX_FLAG_NO_TONEMAP is not set for rgb8.  `stats` (host) may be NULL.            */
int vpx_render(vpx_ctx* ctx, const vpx_frame_params* params, float* accum, uint32_t* rgb8,
               vpx_stats* stats);
/* Tile-sharded variant for multi-GPU: render the tiles t (tile_w x tile_h, row-major tile
   order) with t % n_ranks == rank into a packed float4 buffer (tile after tile; inside a
   16x16 tile entry i is pixel (8*((i>>6)&1) + (i&7), 8*(i>>7) + ((i>>3)&7)): the four 8x8
   quadrants in row-major order, row-major inside each; partial edge tiles padded with
   zeros).  DEVICE pointer.                                                               */
int vpx_render_tiles(vpx_ctx* ctx, const vpx_frame_params* params, uint32_t tile_w,
                     uint32_t tile_h, uint32_t rank, uint32_t n_ranks, float* packed,
                     vpx_stats* stats);
/* Number of float4 elements one rank's packed buffer holds (all ranks use the max). */
uint64_t vpx_tiles_packed_len(uint32_t width, uint32_t height, uint32_t tile_w,
                              uint32_t tile_h, uint32_t n_ranks);
/* Tile-sharded render with the accumulator sharded with the tiles: the rank keeps the
   running average of ITS tiles in `accum_packed` (float4[vpx_tiles_packed_len], DEVICE,
   persistent across frames, packed layout as vpx_render_tiles; blended with weight
   1/(frame_index+1) like vpx_render's accumulator, so start it finite, e.g. zeroed) and
   tonemaps them into `rgb8_packed` (uint32[len], DEVICE) — the only bytes rank 0 needs
   for the screen.  Bit-identical to vpx_render's accumulator / screen for those pixels. */
int vpx_render_tiles_accum(vpx_ctx* ctx, const vpx_frame_params* params, uint32_t tile_w,
                           uint32_t tile_h, uint32_t rank, uint32_t n_ranks, float* accum_packed,
                           uint32_t* rgb8_packed, vpx_stats* stats);
/* Accumulation windows: frames frame_index .. frame_index + n_frames - 1 of params (the
   reference's spp loop of Renderer::Tick calls, renderer.cpp:1646-1891, one per frame with
   w = 1/(n+1)), with the same results as n_frames calls of vpx_render /
   vpx_render_tiles_accum (bit-identical accumulator and RGB8).  When a frame's share is small
   (a rank's 1/n_ranks of the tiles), several frames render in ONE chain of launches — frame b
   in tile blocks [b*T, (b+1)*T) with its own seeds — and a single blend folds their samples
   into the accumulator in frame order; large frames render one chain each.  Lanes
   (vpx_set_pipeline) carry the chains as they carry frames.  VPX_FLAG_NO_TONEMAP frames and
   device sets (vpx_create_multi) render frame by frame. */
int vpx_render_window(vpx_ctx* ctx, const vpx_frame_params* params, uint32_t n_frames, float* accum,
                      uint32_t* rgb8);
int vpx_render_tiles_accum_window(vpx_ctx* ctx, const vpx_frame_params* params, uint32_t n_frames,
                                  uint32_t tile_w, uint32_t tile_h, uint32_t rank, uint32_t n_ranks,
                                  float* accum_packed, uint32_t* rgb8_packed);
/* Rank 0: scatter n_ranks gathered packed RGB8 buffers (back to back, DEVICE) into the
   screen rgb8 (uint32[W*H], DEVICE). */
int vpx_composite_rgb8(vpx_ctx* ctx, const vpx_frame_params* params, uint32_t tile_w,
                       uint32_t tile_h, uint32_t n_ranks, const uint32_t* gathered, uint32_t* rgb8);
/* Rank-0 composite: `gathered` = n_ranks packed buffers back to back (DEVICE); unpack,
   accumulate into accum and tonemap into rgb8 exactly like vpx_render's epilogue.      */
int vpx_composite_tiles(vpx_ctx* ctx, const vpx_frame_params* params, uint32_t tile_w,
                        uint32_t tile_h, uint32_t n_ranks, const float* gathered,
                        float* accum, uint32_t* rgb8);

/* ---- static-camera path ------------------------------------ */
/* Renderer::prevCamera as CopyToPrevCamera leaves it (renderer.cpp:1893-1902): position
   and the four frustum-plane normals of Camera::SetFrustumNormals (camera.h:53-66). */
typedef struct vpx_prev_camera {
    float cam_pos[3];
    float left_normal[3];
    float right_normal[3];
    float top_normal[3];
    float bottom_normal[3];
    float pad;
} vpx_prev_camera;  /* 64 bytes */
/* One frame of Renderer::Tick's static branch (renderer.cpp:1996-2101): TraceReproject
   (renderer.cpp:1330-1585) of Camera::GetPrimaryRayNoDOF per pixel (AA / DOF flags are
   ignored), then per pixel PointToUV into `prev`, IsOccludedPrevFrame, SampleHistory,
   ClampHistory, the material weight, lerp, ApplyReinhardJodie, RGB8.  `history`
   (float4[W*H], DEVICE) is illuminationHistoryBuffer: read, then replaced by this frame's
   illumination (tempIlluminationBuffer).  `rgb8` DEVICE uint32[W*H] (may be NULL). */
int vpx_render_reproject(vpx_ctx* ctx, const vpx_frame_params* params, const vpx_prev_camera* prev,
                         float* history, uint32_t* rgb8, vpx_stats* stats);

/* Work counters accumulated on device over every render call since the last reset
   (no per-frame synchronisation); kernel_ms/total_ms are not filled here.            */
int vpx_get_counters(vpx_ctx* ctx, vpx_stats* out, int reset);

/* ---- per-stage profile (measurement; off by default) ------------------------------ */
/* Stages of one vpx_render / vpx_render_tiles call. */
#define VPX_STAGE_PRIMARY 0  /* primary rays + Renderer::FindNearest                   */
#define VPX_STAGE_SHADE 1    /* Trace material switch (+ glass/smoke exit marches)      */
#define VPX_STAGE_SHADOW 2   /* Renderer::IsOccluded of the emitted shadow rays         */
#define VPX_STAGE_RESOLVE 3  /* light sums                                              */
#define VPX_STAGE_BOUNCE 4   /* Renderer::FindNearest of bounce rays                    */
#define VPX_STAGE_FINISH 5   /* fold + accumulate + tonemap (or tile pack)              */
#define VPX_STAGE_FRAME 6    /* a whole Trace-depth-0 frame in one launch (small launches,
                                single volume: stages 0, 1, 2, 3, 5 fused)    */
#define VPX_STAGE_INSTANCES 7 /* multi-volume scenes: the primary rays' Renderer::FindNearest
                                over the volumes after the world (volume 0, walked in stage 0)
                                and the analytic shapes, then level 0's shade */
#define VPX_NUM_STAGES 8
typedef struct vpx_profile {
    float stage_ms[8];            /* summed device time per stage (HIP events on the stream) */
    uint32_t stage_launches[8];   /* kernel launches timed per stage                         */
    uint64_t stage_cells[8];      /* DDA cells read per stage (all launches, incl. untimed)  */
    float stage_busy_ms[8];       /* union of the stage's launch intervals: launches that run
                                     at the same time (frames in flight, vpx_set_pipeline)
                                     count once; equals stage_ms when they do not overlap     */
} vpx_profile;
/* Time every stage launch of the next renders with HIP events on the library's stream
   (up to `max_launches` launches; 0 turns profiling off).  Adds no synchronisation. */
int vpx_profile_enable(vpx_ctx* ctx, uint32_t max_launches);
/* Time only the stages whose bit (1 << VPX_STAGE_*) is set in `stage_mask` (default: all).
   Each timed launch adds two event records to the stream: timing all five C1 stages
   slowed the frame by 4.3 %, so a benchmark times only the stage it reports. */
int vpx_profile_select(vpx_ctx* ctx, uint32_t stage_mask);
/* Synchronise, sum the recorded stage times and return them (reset: clear events and
   the per-stage cell counters). */
int vpx_profile_read(vpx_ctx* ctx, vpx_profile* out, int reset);
/* The busy-time rule vpx_profile_read applies (host only, no device): the length of the union
   of n intervals [se[2i], se[2i+1]) in ms, overlaps counted once.  Starts may be negative
   (a lane's launch that began before the first recorded event). */
float vpx_profile_busy_union(const float* se, uint32_t n);

/* ---- unit entries (host pointers; mirror the reference per-ray functions) ---------- */
int vpx_find_nearest(vpx_ctx* ctx, const vpx_ray* rays, uint32_t n, vpx_hit* hits);
int vpx_is_occluded(vpx_ctx* ctx, const vpx_ray* rays, uint32_t n, uint8_t* occluded);
/* Trace(ray, depth) with an explicit xorshift32 state per ray; radiance = float3[n].
   sky: the constant SampleSky colour (activateSky == false), or NULL for the texture. */
int vpx_trace(vpx_ctx* ctx, const vpx_ray* rays, const uint32_t* seeds, uint32_t n,
              int32_t depth, const float sky[3], int32_t area_samples, float* radiance);
/* Focus ray of Renderer::Tick (world-space ray against every Scene::FindNearest). */
int vpx_focus_distance(vpx_ctx* ctx, uint32_t width, uint32_t height, float* focal_distance);

/* ---- BasicBVH (src/BVH/BasicBVH.{h,cpp}) ----------------------- */
/* The reference's triangle BVH: midpoint split on the longest axis, leaves of <= 2
   triangles, recursive left-then-right traversal that only shortens Ray::t.  A Renderer
   member (renderer.h:220) that Renderer::Trace does not call; offered as the reference
   offers it.  The device traversal stages the whole BVH (nodes, triangles, indices) in
   LDS per workgroup, one ray per lane. */
#define VPX_BVH_MAX_TRIS 512
#define VPX_BVH_MAX_DEPTH 63   /* deepest tree the device traversal stack holds (root = 1) */
typedef struct vpx_bvh_tri {       /* Tri (BasicBVH.h:3-7) without the centroid */
    float v0[3], v1[3], v2[3];
} vpx_bvh_tri;                     /* 36 bytes */
typedef struct vpx_bvh_node {      /* BVHNode (BasicBVH.h:11-20) */
    float aabb_min[3], aabb_max[3];
    uint32_t left_first, tri_count;
} vpx_bvh_node;                    /* 32 bytes */
/* Build (vpx_bvh_build_host) and upload the BVH of n triangles (1..VPX_BVH_MAX_TRIS;
   n = 0 removes it).  The midpoint split has no depth cap (as the reference's recursion):
   a tree deeper than VPX_BVH_MAX_DEPTH (vpx_bvh_depth) is refused with VPX_E_INVALID. */
int vpx_bvh_set(vpx_ctx* ctx, const vpx_bvh_tri* tris, uint32_t n);
/* IntersectBVH(ray, 0) per ray: rays built as in vpx_find_nearest (Ray(O, D) normalises D,
   t = tmax); t_out[i] = ray.t afterwards (tmax when nothing closer is hit). */
int vpx_bvh_intersect(vpx_ctx* ctx, const vpx_ray* rays, uint32_t n, float* t_out);

/* ---- host-side helpers restating reference host code (no device work) -------------- */
/* Camera basis exactly as Camera::HandleInput(0) leaves it (camera.h:121-178). */
int vpx_camera_look_at(const float pos[3], const float target[3], uint32_t width,
                       uint32_t height, vpx_camera* out);
/* Scene::SetCubeBoundaries + Scene::SetTransform (scene.cpp:213-217, 373-405). */
int vpx_volume_set_transform(const float position[3], const float scale[3],
                             const float rotation[3], vpx_volume* out);
/* Camera::HandleInput(0) basis + SetFrustumNormals + CopyToPrevCamera
   (camera.h:53-66, 113-181; renderer.cpp:710-711, 1893-1902). */
int vpx_prev_camera_look_at(const float pos[3], const float target[3], uint32_t width, uint32_t height,
                            vpx_prev_camera* out);
/* Renderer::MaterialSetUp table, padded to 256 entries (renderer.cpp:357-443). */
int vpx_default_materials(vpx_material* out256);
/* Per-pixel xorshift32 state used by vpx_render: 0x12345678 + WangHash((k+1)*17),
   k = seed_base + frame_index*W*H + y*W + x  (InitSeed, template/tmpl8math.cpp:35-38). */
uint32_t vpx_pixel_seed(uint32_t seed_base, uint32_t frame_index, uint32_t width,
                        uint32_t height, uint32_t x, uint32_t y);
/* BasicBVH::BuildBVH (BasicBVH.cpp:72-136): nodes needs 2n-1 entries, tri_idx n; the
   number of nodes used is stored in *nodes_used. */
int vpx_bvh_build_host(const vpx_bvh_tri* tris, uint32_t n, vpx_bvh_node* nodes, uint32_t* tri_idx,
                       uint32_t* nodes_used);
/* MagicaVoxel .vox (versions 150 / 200) decoded as ogt_vox v0.997 hands it to
   Scene::LoadModel (template/scene.cpp:449-529: read_scene_with_flags(buf, n, 0)->models[0]
   and ->palette): size_out = (size_x, size_y, size_z); voxels (if not NULL, capacity
   voxels_cap >= sx*sy*sz) = voxel_data, index x + y*sx + z*sx*sy, palette index, 0 = empty,
   after the IMAP remap; palette_rgba (if not NULL) = 256 RGBA, voxel byte k's colour at
   4k.  voxels == palette_rgba == NULL only queries the size.  VPX_E_INVALID for a malformed
   file, VPX_E_STATE when a palette is asked of a file without an RGBA chunk (MagicaVoxel's
   built-in default palette is not carried). */
int vpx_vox_decode(const uint8_t* data, uint64_t len, uint32_t size_out[3], uint8_t* voxels,
                   uint64_t voxels_cap, uint8_t palette_rgba[1024]);
/* Depth of a tree built by vpx_bvh_build_host (a leaf root = 1; 0 when nodes_used == 0). */
uint32_t vpx_bvh_depth(const vpx_bvh_node* nodes, uint32_t nodes_used);
/* BasicBVH::BasicBVH() triangle set (BasicBVH.cpp:4-16): 64 triangles, vertex0 = r0*9-5,
   vertex1 = vertex0+r1, vertex2 = vertex0+r2, each r a float3 of RandomFloat() from the
   xorshift32 state *seed (advanced; the three draws of a float3 taken left to right —
   C++ leaves that order unspecified). */
int vpx_bvh_random_tris(uint32_t* seed, vpx_bvh_tri out[64]);
/* The world box the device culls a volume's walks with (no reference counterpart: the
   reference sets up every volume in Renderer::FindNearest / IsOccluded, renderer.cpp:209-243,
   946-1018): out = (lo x, y, z, hi x, y, z), the box of the cube b0..b1's corners mapped by the
   inverse of the affine part of inv_matrix (rows 0-2, as TransformPosition reads it), padded by
   0.1 % of the half-diagonal + 1e-3 of the scale and rounded outward; +-inf when the 3x3 part
   is singular (never culled).  A ray's segment [0, t] that misses the box reads no cell of the
   volume in the reference's loop. */
int vpx_volume_bounds(const vpx_volume* v, float out[6]);

#ifdef __cplusplus
}
#endif
#endif /* VPX_H_ */
