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
        return self

    def ResetAccumulator(self):  # renderer.cpp:343-346
        self.numRenderedFrames = 0

    def Update(self, stats=False):
        p = self.scene.frame_params(frame_index=self.numRenderedFrames)
        p.max_bounces = self.maxBounces
        p.aa_strength = self.antiAliasingStrength
        p.area_samples = self.numCheckShadowsAreaLight
        self.last_stats = self.ctx.render(p, self.accumulator.data_ptr(), self.screen.data_ptr(), stats=stats)
        self.numRenderedFrames += 1
        return self.last_stats

    def Tick(self, deltaTime=0.0, stats=False):
        if not self.staticCamera:
            if self.scene.flags & abi.VPX_FLAG_DOF:  # focus ray, renderer.cpp:1987-1991
                self.scene.camera.focal_distance = self.ctx.focus_distance(self.scene.width, self.scene.height)
                self.ctx.set_camera(self.scene.camera)
            return self.Update(stats=stats)
        raise NotImplementedError("static-camera reprojection path is out of scope (SURVEY.md §8(f) rank 1)")

    def synchronize(self):
        self.stream.synchronize()

    def screen_host(self):
        self.synchronize()
        return self.screen.cpu().numpy().view("uint32").reshape(self.scene.height, self.scene.width)

    def accumulator_host(self):
        self.synchronize()
        return self.accumulator.cpu().numpy().reshape(self.scene.height, self.scene.width, 4)
