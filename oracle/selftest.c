/*
 * selftest.c — TEST INFRASTRUCTURE: drives every entry of the CPU restatement
 * (vpx_oracle.c) over a small synthetic world, for the AddressSanitizer /
 * UndefinedBehaviorSanitizer build of SURVEY.md §5 (`make -C oracle sanitize`, run by
 * tests/test_sanitizers.py).  Exit status 0 = every call returned VPX_OK and the
 * sanitizers stayed quiet (they abort on the first report: -fno-sanitize-recover).
 *
 * World: 48^3 cells — a white ground slab, pillars of default materials (16..19), a glass
 * block, a smoke block, an emissive cell row and the NONE index 255 scattered in; three
 * volumes (the grid, a rotated / scaled instance sharing it, an exact duplicate), a sphere
 * and a triangle, every light kind, a sky texture.  Frames at depths -1, 0, 3 and 14 with
 * AA + DOF, the static-camera path, the per-ray entries and BasicBVH.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "vpx_oracle.h"

#define N 48
#define W 40
#define H 28

static int fails = 0;
#define OK(x)                                                                   \
    do {                                                                        \
        const int rc_ = (x);                                                    \
        if (rc_ != 0) {                                                         \
            fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, rc_);   \
            ++fails;                                                            \
        }                                                                       \
    } while (0)

static void ident(float m[16]) {
    memset(m, 0, 16 * sizeof(float));
    m[0] = m[5] = m[10] = m[15] = 1.0f;
}

int main(void) {
    static uint8_t cells[N * N * N];
    for (int z = 0; z < N; ++z)
        for (int y = 0; y < N; ++y)
            for (int x = 0; x < N; ++x) {
                uint8_t v = VPX_MAT_NONE;
                if (y < 2) v = VPX_MAT_NON_METAL_WHITE;
                else if ((x & 7) < 3 && (z & 7) < 3 && y < 4 + ((x * 7 + z * 3) % 13)) v = (uint8_t)(16 + (x + z) % 4);
                else if (x > 30 && x < 36 && z > 30 && z < 36 && y < 12) v = VPX_MAT_GLASS;
                else if (x > 8 && x < 14 && z > 30 && z < 38 && y < 10) v = 10;  /* smoke */
                else if (y == 20 && z == 5) v = VPX_MAT_EMISSIVE;
                else if (y == 3 && (x * 31 + z * 17) % 29 == 0) v = (uint8_t)(5 + x % 3);  /* metals */
                cells[x + y * N + z * N * N] = v;
            }
    oracle_grid grid = {cells, N};

    vpx_volume vols[3];
    memset(vols, 0, sizeof(vols));
    ident(vols[0].matrix), ident(vols[0].inv_matrix);
    vols[0].b1[0] = vols[0].b1[1] = vols[0].b1[2] = 1.0f;
    vols[1] = vols[0];
    /* rotated about y by 0.5 rad, scaled 0.3, moved up: matrix and its inverse */
    const float c = cosf(0.5f), s = sinf(0.5f), k = 0.3f;
    const float m1[16] = {k * c, 0, k * s, 0.2f, 0, k, 0, 0.9f, -k * s, 0, k * c, 0.3f, 0, 0, 0, 1};
    const float i1[16] = {c / k, 0, -s / k, 0, 0, 1 / k, 0, 0, s / k, 0, c / k, 0, 0, 0, 0, 1};
    memcpy(vols[1].matrix, m1, sizeof(m1));
    memcpy(vols[1].inv_matrix, i1, sizeof(i1));
    for (int r = 0; r < 3; ++r) {  /* inv(M) translation part */
        float t = 0;
        for (int q = 0; q < 3; ++q) t -= i1[r * 4 + q] * m1[q * 4 + 3];
        vols[1].inv_matrix[r * 4 + 3] = t;
    }
    vols[2] = vols[0];

    static vpx_material mats[256];
    for (int i = 0; i < 256; ++i) {
        mats[i].albedo[0] = 0.2f + (float)(i % 7) * 0.1f, mats[i].albedo[1] = 0.5f, mats[i].albedo[2] = 0.8f;
        mats[i].roughness = (i % 3) * 0.3f;
        mats[i].emissive = (i >= 9 && i <= 14) ? 3.0f + (float)i : (i == 15 ? 5.0f : 0.0f);
        mats[i].ior = 1.45f;
    }
    const vpx_point_light pts[1] = {{{0.5f, 1.5f, 0.5f}, {1, 1, 1}}};
    const vpx_spot_light sps[1] = {{{0.2f, 1.2f, 0.2f}, {0.0f, -1.0f, 0.0f}, {1.5f, 1.5f, 1.5f}, 0.7f}};
    const vpx_area_light ars[2] = {{{0.5f, 2.0f, 0.5f}, {1, 1, 1}, 1.2f, 0.4f}, {{-0.5f, 1.5f, 0.5f}, {1, 0.8f, 0.6f}, 1.0f, 0.3f}};
    const vpx_sphere sph[1] = {{{0.6f, 0.5f, 0.2f}, 0.1f, VPX_MAT_GLASS, {0, 0, 0}}};
    const vpx_triangle tri[1] = {{{0.3f, 0.4f, 0.7f}, {-0.1f, 0, 0}, {0, 0.1f, 0}, {0.1f, 0, 0}, 20, {0, 0, 0}}};
    static float sky[16 * 8 * 3];
    for (int i = 0; i < 16 * 8 * 3; ++i) sky[i] = 0.1f * (float)(i % 11);

    oracle_scene sc;
    memset(&sc, 0, sizeof(sc));
    sc.grids = &grid, sc.num_grids = 1;
    sc.volumes = vols, sc.num_volumes = 3;
    sc.materials = mats;
    sc.points = pts, sc.num_points = 1;
    sc.spots = sps, sc.num_spots = 1;
    sc.areas = ars, sc.num_areas = 2;
    sc.dir = (vpx_dir_light){{-0.3f, -1.0f, -0.2f}, {1, 1, 1}};
    sc.spheres = sph, sc.num_spheres = 1;
    sc.triangles = tri, sc.num_triangles = 1;
    /* camera at (1.25, 0.9, -0.35) looking at (0.45, 0.15, 0.55): a hand-built basis */
    vpx_camera* cam = &sc.camera;
    const float P[3] = {1.25f, 0.9f, -0.35f};
    memcpy(cam->cam_pos, P, sizeof(P));
    const float tl[3] = {0.3f, 0.9f, 0.2f}, tr[3] = {1.3f, 0.9f, 0.8f}, bl[3] = {0.3f, 0.1f, 0.2f};
    memcpy(cam->top_left, tl, sizeof(tl)), memcpy(cam->top_right, tr, sizeof(tr)), memcpy(cam->bottom_left, bl, sizeof(bl));
    cam->right[0] = 1, cam->up[1] = 1, cam->focal_distance = 1.0f, cam->defocus_jitter = 2.0f;
    sc.sky_pixels = sky, sc.sky_w = 16, sc.sky_h = 8, sc.sky_hdr = 1.3f;

    static float accum[W * H * 4], hist[W * H * 4];
    static uint32_t rgb[W * H];
    vpx_stats st;
    const int depths[] = {-1, 0, 3, 14};
    for (int di = 0; di < 4; ++di) {
        for (uint32_t f = 0; f < 2; ++f) {
            vpx_frame_params p;
            memset(&p, 0, sizeof(p));
            p.width = W, p.height = H, p.max_bounces = depths[di], p.frame_index = f;
            p.flags = VPX_FLAG_AA | VPX_FLAG_DOF | (di == 2 ? VPX_FLAG_SKY : 0u);
            p.aa_strength = 1.0f, p.area_samples = 3;
            p.sky[0] = 0.392f, p.sky[1] = 0.584f, p.sky[2] = 0.829f;
            OK(oracle_render(&sc, &p, accum, rgb, &st, 2));
            vpx_prev_camera prev;
            memset(&prev, 0, sizeof(prev));
            memcpy(prev.cam_pos, P, sizeof(P));
            prev.left_normal[0] = 1, prev.right_normal[0] = -1, prev.top_normal[1] = -1, prev.bottom_normal[1] = 1;
            OK(oracle_render_reproject(&sc, &p, &prev, hist, rgb, &st, 2));
        }
    }
    enum { NR = 512 };
    static vpx_ray rays[NR];
    static vpx_hit hits[NR];
    static uint32_t seeds[NR], ccount[NR];
    static uint8_t occ[NR];
    static float rad[NR * 3], tout[NR];
    uint32_t g = 0x9E3779B9u;
    for (int i = 0; i < NR; ++i) {
        for (int a = 0; a < 3; ++a) {
            g ^= g << 13, g ^= g >> 17, g ^= g << 5;
            rays[i].origin[a] = -0.5f + 2.0f * (float)(g & 0xffff) / 65535.0f;
            g ^= g << 13, g ^= g >> 17, g ^= g << 5;
            rays[i].direction[a] = -1.0f + 2.0f * (float)(g & 0xffff) / 65535.0f;
        }
        if (i % 17 == 0) rays[i].direction[i % 3] = 0.0f;  /* axis-parallel: infinite rD */
        rays[i].tmax = (i % 3) ? 1e34f : 0.7f;
        rays[i].inside_glass = (uint32_t)(i % 5 == 0);
        seeds[i] = g | 1u;
    }
    OK(oracle_find_nearest(&sc, rays, NR, hits));
    OK(oracle_is_occluded(&sc, rays, NR, occ, ccount));
    const float skyc[3] = {0.392f, 0.584f, 0.829f};
    OK(oracle_trace(&sc, rays, seeds, NR, 14, skyc, 3, rad, &st));
    OK(oracle_trace(&sc, rays, seeds, NR, 4, NULL, 5, rad, &st));
    (void)oracle_focus_distance(&sc, W, H);

    vpx_bvh_tri tris[64];
    vpx_bvh_node nodes[127];
    uint32_t idx[64];
    (void)oracle_bvh_random_tris(0x12345678u, tris);
    const uint32_t used = oracle_bvh_build(tris, 64, nodes, idx);
    if (!used) ++fails;
    OK(oracle_bvh_intersect(nodes, tris, idx, rays, NR, tout));

    static uint8_t model[16 * 16 * 16], out[N * N * N];
    for (int i = 0; i < 16 * 16 * 16; ++i) model[i] = (uint8_t)((i * 7) % 9 == 0 ? 20 + i % 5 : 0);
    const float scale[3] = {1, 1, 1};
    oracle_load_model(model, 16, 16, 16, N, scale, out);
    oracle_load_model_partial(model, 16, 16, 16, N, scale, 8, 20, out);
    oracle_emissive_sphere(out, N, VPX_MAT_EMISSIVE, 5.5f);
    printf("selftest: %d failure(s); last frame primary %llu shadow %llu cells %llu\n", fails,
           (unsigned long long)st.primary_rays, (unsigned long long)st.shadow_rays,
           (unsigned long long)st.dda_cells);
    return fails ? 1 : 0;
}
