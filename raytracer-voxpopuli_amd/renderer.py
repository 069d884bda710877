"""Host mirror of the reference Renderer's hot-path surface (renderer.h:42-245).

`Renderer.Tick(deltaTime)` keeps the reference's contract (template/precomp.h:399,
renderer.cpp:1972-1995): optional focus ray, then `Update()`, which here is ONE call into
libvpx_hip.so (`vpx_render`) instead of the execution::par pixel loop
(renderer.cpp:1646-1891).  The accumulator (float4[W*H]) and the screen (uint32
0x00RRGGBB, template/surface.h) live in HBM as torch tensors; `screen_host()` copies the
8-bit frame out for display.  The C++ twin of this class is host/vpx_renderer.{h,cpp}.
"""
import torch

from . import abi
from .context import Context


class Renderer:
    def __init__(self, scene, device=0, ctx=None):
        self.scene = scene
        self.device = torch.device("cuda", device)
        self.ctx = ctx or Context(device)
        self.maxBounces = scene.max_bounces               # renderer.h:175
        self.numRenderedFrames = 0                        # renderer.h:204
        self.antiAliasingStrength = scene.aa_strength     # renderer.h:185
        self.numCheckShadowsAreaLight = scene.area_samples  # renderer.h:205
        self.staticCamera = False
        self.activateSky = bool(scene.flags & abi.VPX_FLAG_SKY)  # renderer.h:216
        self.HDRLightContribution = scene.sky_hdr               # renderer.h:224
        self.skyPixels = scene.sky_texture                      # renderer.h:226 (float32 (H, W, 3))
        self.prevCamera = None             # renderer.h:182 (vpx_prev_camera)
        self.illuminationHistory = None    # renderer.h:242, float4[W*H] in HBM
        self.accumulator = None
        self.screen = None
        self.last_stats = None

    def Init(self):
        """Renderer::Init minus window/asset/game setup (renderer.cpp:688-736)."""
        w, h = self.scene.width, self.scene.height
        self.accumulator = torch.zeros(w * h * 4, dtype=torch.float32, device=self.device)
        self.screen = torch.zeros(w * h, dtype=torch.int32, device=self.device)
        torch.cuda.synchronize(self.device)
        # the library launches on this torch stream (never the legacy NULL stream, whose
        # handle 0 would select the context's own stream instead)
        self.stream = torch.cuda.Stream(self.device)
        self.ctx.set_stream(self.stream.cuda_stream)
        self.ctx.load_scene(self.scene)
        self._sky_uploaded = (self.skyPixels, self.HDRLightContribution)
        return self

    def SetArithmetic(self, mode):
        """abi.VPX_ARITH_X86_HOST: the reference's FastReciprocal / rsqrtps as this host computes
        them (vpx_set_arithmetic); abi.VPX_ARITH_EXACT: exact 1/x, 1/sqrtf (default)."""
        self.ctx.set_arithmetic(mode)
        return self

    def _frame_params(self):
        p = self.scene.frame_params(frame_index=self.numRenderedFrames)
        p.max_bounces = self.maxBounces
        p.area_samples = self.numCheckShadowsAreaLight
        up_px, up_hdr = self._sky_uploaded
        if self.skyPixels is not up_px or self.HDRLightContribution != up_hdr:  # ImGui edits, renderer.cpp:2591
            self.ctx.set_sky(self.skyPixels, self.HDRLightContribution)
            self._sky_uploaded = (self.skyPixels, self.HDRLightContribution)
        p.flags = (p.flags & ~abi.VPX_FLAG_SKY) | (abi.VPX_FLAG_SKY if self.activateSky else 0)
        return p

    def ResetAccumulator(self):  # renderer.cpp:343-346
        self.numRenderedFrames = 0

    def Update(self, stats=False):
        p = self._frame_params()
        p.aa_strength = self.antiAliasingStrength
        self.last_stats = self.ctx.render(p, self.accumulator.data_ptr(), self.screen.data_ptr(), stats=stats)
        self.numRenderedFrames += 1
        return self.last_stats

    def CopyToPrevCamera(self):  # renderer.cpp:1893-1902
        from .scene import prev_camera
        self.prevCamera = prev_camera(self.scene._cam_pos, self.scene._cam_target, self.scene.width, self.scene.height)

    def Tick(self, deltaTime=0.0, stats=False):
        if not self.staticCamera:
            if self.scene.flags & abi.VPX_FLAG_DOF:  # focus ray, renderer.cpp:1987-1991
                self.scene.camera.focal_distance = self.ctx.focus_distance(self.scene.width, self.scene.height)
                self.ctx.set_camera(self.scene.camera)
            return self.Update(stats=stats)
        # static branch (renderer.cpp:1996-2101): TraceReproject + history reprojection
        if self.prevCamera is None:
            self.CopyToPrevCamera()
        if self.illuminationHistory is None:
            w, h = self.scene.width, self.scene.height
            self.illuminationHistory = torch.zeros(w * h * 4, dtype=torch.float32, device=self.device)
            torch.cuda.synchronize(self.device)  # allocated on torch's stream; the library uses its own
        p = self._frame_params()
        st = self.ctx.render_reproject(p, self.prevCamera, self.illuminationHistory.data_ptr(), self.screen.data_ptr(),
                                       stats=stats)
        self.numRenderedFrames += 1
        return st

    def history_host(self):
        self.synchronize()
        return self.illuminationHistory.cpu().numpy().reshape(self.scene.height, self.scene.width, 4)

    def synchronize(self):
        self.stream.synchronize()

    def screen_host(self):
        self.synchronize()
        return self.screen.cpu().numpy().view("uint32").reshape(self.scene.height, self.scene.width)

    def accumulator_host(self):
        self.synchronize()
        return self.accumulator.cpu().numpy().reshape(self.scene.height, self.scene.width, 4)
