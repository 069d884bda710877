// vpx_renderer.cpp — see vpx_renderer.h.
#include "vpx_renderer.h"

#include <hip/hip_runtime_api.h>

namespace vpxhost {

Renderer::Renderer(int device) : device_(device) { status_ = vpx_create(device, &ctx_); }

Renderer::Renderer(const std::vector<int>& devices) : device_(devices.empty() ? 0 : devices[0]) {
    status_ = devices.empty() ? VPX_E_INVALID : vpx_create_multi(devices.data(), (int)devices.size(), &ctx_);
}

Renderer::~Renderer() {
    if (accumulator_) (void)hipFree(accumulator_);
    if (screen_) (void)hipFree(screen_);
    if (history_) (void)hipFree(history_);
    if (ctx_) vpx_destroy(ctx_);
}

const char* Renderer::LastError() const {
    if (!err_.empty()) return err_.c_str();
    return ctx_ ? vpx_last_error(ctx_) : "vpx_create failed (no usable HIP device)";
}

int Renderer::Init(uint32_t width, uint32_t height) {
    if (status_) return status_;
    if (vpx_abi_version() != VPX_ABI_VERSION) {  // a stale libvpx_hip.so
        err_ = "libvpx_hip.so ABI version differs from include/vpx.h";
        return status_ = VPX_E_STATE;
    }
    if (!width || !height) return VPX_E_INVALID;
    if (hipSetDevice(device_) != hipSuccess ||
        hipMalloc(&accumulator_, sizeof(float) * 4 * width * height) != hipSuccess ||
        hipMalloc(&screen_, sizeof(uint32_t) * width * height) != hipSuccess ||
        hipMemset(accumulator_, 0, sizeof(float) * 4 * width * height) != hipSuccess ||
        hipMemset(screen_, 0, sizeof(uint32_t) * width * height) != hipSuccess) {
        err_ = "frame buffer allocation failed";
        return VPX_E_NOMEM;
    }
    width_ = width, height_ = height;
    numRenderedFrames = 0;
    return VPX_OK;
}

int Renderer::UploadGrid(uint32_t grid_id, const uint8_t* cells, uint32_t n) {
    return status_ ? status_ : vpx_upload_grid(ctx_, grid_id, cells, n);
}

int Renderer::SetVolumes(const std::vector<vpx_volume>& v) {
    return status_ ? status_ : vpx_set_volumes(ctx_, v.data(), (uint32_t)v.size());
}

int Renderer::SetMaterials(const std::vector<vpx_material>& m) {
    return status_ ? status_ : vpx_set_materials(ctx_, m.data(), (uint32_t)m.size());
}

int Renderer::SetLights(const std::vector<vpx_point_light>& p, const std::vector<vpx_spot_light>& s,
                        const std::vector<vpx_area_light>& a, const vpx_dir_light& d) {
    if (status_) return status_;
    return vpx_set_lights(ctx_, p.data(), (uint32_t)p.size(), s.data(), (uint32_t)s.size(), a.data(),
                          (uint32_t)a.size(), &d);
}

int Renderer::SetShapes(const std::vector<vpx_sphere>& s, const std::vector<vpx_triangle>& t) {
    if (status_) return status_;
    return vpx_set_shapes(ctx_, s.data(), (uint32_t)s.size(), t.data(), (uint32_t)t.size());
}

int Renderer::LookAt(const float pos[3], const float target[3]) {
    if (status_) return status_;
    const float keep_focal = camera.focal_distance, keep_jitter = camera.defocus_jitter;
    int rc = vpx_camera_look_at(pos, target, width_, height_, &camera);
    if (rc) return rc;
    for (int i = 0; i < 3; ++i) camPos_[i] = pos[i], camTarget_[i] = target[i];
    if (keep_focal > 0.0f) camera.focal_distance = keep_focal, camera.defocus_jitter = keep_jitter;
    return vpx_set_camera(ctx_, &camera);
}

int Renderer::Update(vpx_stats* stats) {
    if (status_) return status_;
    if (!accumulator_) return VPX_E_STATE;
    vpx_frame_params p{};
    p.width = width_, p.height = height_;
    p.max_bounces = maxBounces;
    p.frame_index = numRenderedFrames;
    p.seed_base = 0;
    p.flags = (flags & ~VPX_FLAG_SKY) | (activateSky ? VPX_FLAG_SKY : 0u);
    p.aa_strength = antiAliasingStrength;
    p.area_samples = numCheckShadowsAreaLight;
    p.sky[0] = sky[0], p.sky[1] = sky[1], p.sky[2] = sky[2];
    uint32_t* target = nullptr;
    int rc = MapScreen(&target);
    if (rc) return rc;
    rc = UnmapScreen(vpx_render(ctx_, &p, accumulator_, target, stats));
    if (rc == VPX_OK) ++numRenderedFrames;
    return rc;
}

int Renderer::SetSky(const float* rgb, uint32_t width, uint32_t height, float hdr_contribution) {
    return status_ ? status_ : vpx_set_sky(ctx_, rgb, width, height, hdr_contribution);
}

int Renderer::SetArithmetic(uint32_t mode) { return status_ ? status_ : vpx_set_arithmetic(ctx_, mode); }

int Renderer::CopyToPrevCamera() {
    if (status_) return status_;
    const int rc = vpx_prev_camera_look_at(camPos_, camTarget_, width_, height_, &prevCamera);
    if (rc == VPX_OK) havePrev_ = true;
    return rc;
}

// The static branch of Renderer::Tick (renderer.cpp:1996-2101): TraceReproject per pixel,
// reprojection into prevCamera, SampleHistory / ClampHistory, blend, tonemap, RGB8.
int Renderer::UpdateStatic(vpx_stats* stats) {
    if (!history_) {
        const size_t bytes = sizeof(float) * 4 * (size_t)width_ * height_;
        if (hipMalloc(&history_, bytes) != hipSuccess || hipMemset(history_, 0, bytes) != hipSuccess) {
            err_ = "history allocation failed";
            return VPX_E_NOMEM;
        }
    }
    if (!havePrev_) {
        const int rc = CopyToPrevCamera();
        if (rc) return rc;
    }
    vpx_frame_params p{};
    p.width = width_, p.height = height_;
    p.max_bounces = maxBounces;
    p.frame_index = numRenderedFrames;
    p.flags = activateSky ? VPX_FLAG_SKY : 0u;
    p.aa_strength = antiAliasingStrength;
    p.area_samples = numCheckShadowsAreaLight;
    p.sky[0] = sky[0], p.sky[1] = sky[1], p.sky[2] = sky[2];
    uint32_t* target = nullptr;
    int rc = MapScreen(&target);
    if (rc) return rc;
    rc = UnmapScreen(vpx_render_reproject(ctx_, &p, &prevCamera, history_, target, stats));
    if (rc == VPX_OK) ++numRenderedFrames;
    return rc;
}

int Renderer::CopyHistory(float* host_rgba) const {
    if (status_) return status_;
    if (!history_) return VPX_E_STATE;
    int rc = vpx_synchronize(ctx_);
    if (rc) return rc;
    return hipMemcpy(host_rgba, history_, sizeof(float) * 4 * width_ * height_, hipMemcpyDeviceToHost) == hipSuccess
               ? VPX_OK
               : VPX_E_DEVICE;
}

int Renderer::Tick(float /*deltaTime*/, vpx_stats* stats) {
    if (status_) return status_;
    if (staticCamera) return UpdateStatic(stats);
    if (flags & VPX_FLAG_DOF) {  // focus ray of Renderer::Tick (renderer.cpp:1987-1991)
        int rc = vpx_focus_distance(ctx_, width_, height_, &camera.focal_distance);
        if (rc) return rc;
        rc = vpx_set_camera(ctx_, &camera);
        if (rc) return rc;
    }
    return Update(stats);
}

int Renderer::UseGLBuffer(unsigned int pbo) {
    if (status_) return status_;
    const int rc = vpx_gl_register_buffer(ctx_, pbo);
    glBuffer_ = rc == VPX_OK && pbo != 0u;
    return rc;
}

int Renderer::MapScreen(uint32_t** out) const {
    if (!glBuffer_) {
        *out = screen_;
        return VPX_OK;
    }
    size_t bytes = 0;
    int rc = vpx_gl_map(ctx_, out, &bytes);
    if (rc) return rc;
    if (bytes < sizeof(uint32_t) * (size_t)width_ * height_) {
        (void)vpx_gl_unmap(ctx_);
        return VPX_E_INVALID;  // the GL buffer is smaller than the frame
    }
    return VPX_OK;
}

int Renderer::UnmapScreen(int rc) const {
    if (!glBuffer_) return rc;
    const int rc2 = vpx_gl_unmap(ctx_);
    return rc ? rc : rc2;
}

int Renderer::CopyScreen(uint32_t* host_pixels) const {
    if (status_) return status_;
    uint32_t* src = nullptr;
    int rc = MapScreen(&src);
    if (rc) return rc;
    rc = vpx_synchronize(ctx_);
    if (rc == VPX_OK && hipMemcpy(host_pixels, src, sizeof(uint32_t) * width_ * height_, hipMemcpyDeviceToHost) != hipSuccess)
        rc = VPX_E_DEVICE;
    return UnmapScreen(rc);
}

int Renderer::CopyAccumulator(float* host_rgba) const {
    if (status_) return status_;
    int rc = vpx_synchronize(ctx_);
    if (rc) return rc;
    return hipMemcpy(host_rgba, accumulator_, sizeof(float) * 4 * width_ * height_, hipMemcpyDeviceToHost) ==
                   hipSuccess
               ? VPX_OK
               : VPX_E_DEVICE;
}

}  // namespace vpxhost
