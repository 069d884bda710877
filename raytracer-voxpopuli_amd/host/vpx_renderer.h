// vpx_renderer.h — C++ host mirror of the reference Renderer's hot-path surface.
//
// The reference keeps its game loop in `Renderer::Tick(float deltaTime)` (renderer.cpp:1972,
// virtual in template/precomp.h:399) and renders with `Renderer::Update()`
// (renderer.cpp:1646-1891): a parallel loop over pixels calling `Trace(ray, maxBounces)`,
// a running-average accumulator and a Reinhard-Jodie tonemap into `Surface::pixels`.
// This class keeps that surface — same member names, same meaning — and replaces the loop
// by ONE call into libvpx_hip.so (include/vpx.h).  It talks to the library only through
// the C-ABI; HIP is used here just for the two HBM frame buffers and the D2H copy.
//
// Errors: every method returns the VPX_* status of the first failing call (0 = ok) and
// never throws; `LastError()` is the library's message.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/vpx.h"

namespace vpxhost {

class Renderer {
public:
    explicit Renderer(int device = 0);
    // A device set (vpx_create_multi): frames tile-sharded over `devices`, gathered over
    // RCCL to devices[0], where the accumulator and screen live.
    explicit Renderer(const std::vector<int>& devices);
    ~Renderer();
    Renderer(const Renderer&) = delete;
    Renderer& operator=(const Renderer&) = delete;

    // Renderer::Init minus window/asset/game setup (renderer.cpp:688-736): frame buffers.
    int Init(uint32_t width, uint32_t height);

    // --- world (the host owns Scene::grid; the library keeps the device copy) -----------
    int UploadGrid(uint32_t grid_id, const uint8_t* cells, uint32_t n);  // Scene::grid
    int SetVolumes(const std::vector<vpx_volume>& volumes);               // voxelVolumes
    int SetMaterials(const std::vector<vpx_material>& materials);         // materials
    int SetLights(const std::vector<vpx_point_light>& points, const std::vector<vpx_spot_light>& spots,
                  const std::vector<vpx_area_light>& areas, const vpx_dir_light& dir);
    int SetShapes(const std::vector<vpx_sphere>& spheres, const std::vector<vpx_triangle>& triangles);
    // Camera::camPos / camTarget + HandleInput(0) (template/camera.h:113-181).
    int LookAt(const float pos[3], const float target[3]);
    // skyPixels / skyWidth / skyHeight (stbi_loadf RGB floats, renderer.cpp:691) and
    // HDRLightContribution; sampled when activateSky is set.  rgb == nullptr removes it.
    int SetSky(const float* rgb, uint32_t width, uint32_t height, float hdr_contribution);
    // prevCamera = the current camera (CopyToPrevCamera, renderer.cpp:1893-1902).
    int CopyToPrevCamera();
    // The reference's own x86 arithmetic (FastReciprocal in FindNearest, rsqrtps for the
    // primary rays) as this host computes it: VPX_ARITH_X86_HOST; VPX_ARITH_EXACT (default).
    int SetArithmetic(uint32_t mode);

    // --- per frame -----------------------------------------------------------------------
    void ResetAccumulator() { numRenderedFrames = 0; }  // renderer.cpp:343-346
    int Update(vpx_stats* stats = nullptr);             // renderer.cpp:1646-1891
    // Tick: moving camera -> focus ray + Update; staticCamera -> the reprojection branch
    // (renderer.cpp:1996-2101) through vpx_render_reproject with the history in HBM.
    int Tick(float deltaTime, vpx_stats* stats = nullptr);
    // Surface::pixels (0x00RRGGBB, W*H) for display: device -> host copy of the frame.
    int CopyScreen(uint32_t* host_pixels) const;
    // Display interop in place of GLTexture::CopyFrom (template/opengl.cpp:144-149): with a
    // GL pixel-unpack buffer of W*H*4 bytes registered (its GL context current on this
    // thread), Update / Tick pack the frame straight into it (vpx_gl_map -> render ->
    // vpx_gl_unmap) and the window updates its texture from the buffer; CopyScreen then reads
    // the screen out of it.  pbo == 0 returns to the HBM screen.
    int UseGLBuffer(unsigned int pbo);
    int CopyAccumulator(float* host_rgba) const;
    int CopyHistory(float* host_rgba) const;  // illuminationHistoryBuffer (static branch)

    const char* LastError() const;
    vpx_ctx* Context() const { return ctx_; }

    // Members of the reference Renderer this path reads (renderer.h:175-205).
    int32_t maxBounces = 0;
    uint32_t numRenderedFrames = 0;
    float antiAliasingStrength = 1.0f;
    int32_t numCheckShadowsAreaLight = 3;
    bool staticCamera = false;  // renderer.h:229: Tick takes the reprojection branch
    bool activateSky = false;   // renderer.h:216 (needs SetSky; the reference's HDR is missing)
    uint32_t flags = 0;         // VPX_FLAG_AA / VPX_FLAG_DOF
    float sky[3] = {0.392f, 0.584f, 0.829f};  // SampleSky, activateSky == false (renderer.cpp:2310-2313)
    vpx_camera camera{};
    vpx_prev_camera prevCamera{};  // renderer.h:182

private:
    int UpdateStatic(vpx_stats* stats);
    int MapScreen(uint32_t** out) const;  // the frame's RGB8 target: the GL buffer or screen_
    int UnmapScreen(int rc) const;
    bool glBuffer_ = false;
    float camPos_[3] = {0, 0, 0}, camTarget_[3] = {0, 0, 1};
    bool havePrev_ = false;
    float* history_ = nullptr;      // illuminationHistoryBuffer float4[W*H] in HBM
    int status_ = VPX_OK;
    int device_ = 0;
    vpx_ctx* ctx_ = nullptr;
    uint32_t width_ = 0, height_ = 0;
    float* accumulator_ = nullptr;  // float4[W*H] in HBM
    uint32_t* screen_ = nullptr;    // uint32[W*H] in HBM
    std::string err_;
};

}  // namespace vpxhost
