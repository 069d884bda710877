// ogt_ref_dump.cpp — TEST INFRASTRUCTURE: compiles the reference's vendored ogt_vox
// v0.997 (lib/ogt_vox.h, where it lies under /root/reference) and dumps model 0 of a
// .vox file exactly as Scene::LoadModel receives it (template/scene.cpp:474-475):
// size_x/y/z, voxel_data (x + y*sx + z*sx*sy, palette index, 0 = empty) and palette.
// Output (little endian): "VPXM" u32 sx u32 sy u32 sz, 256*4 palette RGBA, voxels.
#define OGT_VOX_IMPLEMENTATION
#include "ogt_vox.h"
#include <cstdio>
#include <cstdint>
#include <vector>

int main(int argc, char** argv)
{
    if (argc != 3) { std::fprintf(stderr, "usage: %s in.vox out.bin\n", argv[0]); return 2; }
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) { std::perror(argv[1]); return 1; }
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    std::vector<uint8_t> buf((size_t)n);
    if (std::fread(buf.data(), 1, (size_t)n, f) != (size_t)n) { std::fclose(f); return 1; }
    std::fclose(f);
    const ogt_vox_scene* scene = ogt_vox_read_scene_with_flags(buf.data(), (uint32_t)n, 0);
    if (!scene || scene->num_models < 1) return 1;
    const ogt_vox_model* m = scene->models[0];
    FILE* o = std::fopen(argv[2], "wb");
    if (!o) { std::perror(argv[2]); return 1; }
    const uint32_t hdr[3] = {m->size_x, m->size_y, m->size_z};
    std::fwrite("VPXM", 1, 4, o);
    std::fwrite(hdr, 4, 3, o);
    for (int i = 0; i < 256; i++) {
        const ogt_vox_rgba c = scene->palette.color[i];
        const uint8_t rgba[4] = {c.r, c.g, c.b, c.a};
        std::fwrite(rgba, 1, 4, o);
    }
    std::fwrite(m->voxel_data, 1, (size_t)m->size_x * m->size_y * m->size_z, o);
    std::fclose(o);
    ogt_vox_destroy_scene(scene);
    return 0;
}
