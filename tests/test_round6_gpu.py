"""Round-6 GPU parity: the instance paths the round added, each against the oracle bit for bit.

- Depth-0 frames of multi-volume scenes shade the paths that cannot meet an instance in the
  world head and defer the others (k_compact's list, k_instances_list); deeper frames keep the
  per-tile k_instances.
- The shadow pool lists the slots a later volume may occlude and k_shadow_slots walks only
  those (with shapes in the scene every unoccluded slot is listed).
- Instances that share one grid walk each lane's own next candidate in one walk (lane_volumes,
  SceneView::inst_grid); instances of different grids keep the wave's union of candidates.
Scenes: a world plus a lattice of rotated, scaled instances (C4's shape), their grids shared or
alternating between two, with area lights (several slots per path), with and without an
analytic sphere, at depths 0 and 2, serial and with frames in flight.
Also: the static-camera branch over the lattice, and the library loaded before torch in a
fresh process still finds the device.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from cases import bits  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def lattice_scene(pkg, grids, depth, sphere=False, n_inst=27):
    sc, abi = pkg.scene, pkg.abi
    desc = sc.model_scene("monu3", 64, 64, 48, depth, city_lights=True)
    size, vox, _ = sc.load_model("monu3")
    desc.grids.append(sc.GridSpec(n=32, dense=sc.load_model_grid(size, vox, 32)))
    if grids == 2:
        desc.grids.append(sc.GridSpec(n=16, dense=sc.load_model_grid(size, vox, 16)))
    rng = np.random.default_rng(7)
    vols = [sc.volume()]
    for k in range(n_inst):
        i, j, l = k % 3, (k // 3) % 3, k // 9
        pos = (0.3 * i - 0.2, 0.5 + 0.25 * j, 0.3 * l - 0.2)
        vols.append(sc.volume(pos, tuple(rng.uniform(0.08, 0.16, 3)), tuple(rng.uniform(-2, 2, 3)),
                              grid_id=1 + (k % grids)))
    desc.volumes = (abi.Volume * len(vols))(*vols)
    desc.areas = [sc.area_light((0.5, 2.2, 0.5), radius=0.5), sc.area_light((-0.8, 1.5, 0.2), radius=0.3)]
    desc.area_samples = 3
    if sphere:
        desc.spheres = [abi.Sphere(abi.vec3((0.35, 0.9, 0.3)), 0.12, 8)]
    desc.flags = abi.VPX_FLAG_AA
    return desc


def render(pkg, desc, frames, lanes=0):
    ctx = pkg.context.Context(0)
    s = torch.cuda.Stream()
    ctx.set_stream(s.cuda_stream)
    ctx.load_scene(desc)
    ctx.set_pipeline(lanes)
    W, H = desc.width, desc.height
    acc = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
    rgb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ctx.counters(reset=True)
    with torch.cuda.stream(s):
        for f in range(frames):
            ctx.render(desc.frame_params(f), acc.data_ptr(), rgb.data_ptr())
    ctx.synchronize()
    st = ctx.counters()
    out = (bits(acc.cpu().numpy().reshape(-1, 4)), rgb.cpu().numpy().view(np.uint32),
           tuple(int(getattr(st, k)) for k in ("primary_rays", "shadow_rays", "bounce_rays", "dda_cells")))
    ctx.close()
    return out


def oracle(orc, pkg, desc, frames):
    o = orc.Oracle(pkg.abi, desc)
    acc, tot = None, np.zeros(4, np.int64)
    for f in range(frames):
        acc, rgb, st = o.render(desc.frame_params(f), accum=acc)
        tot += [st.primary_rays, st.shadow_rays, st.bounce_rays, st.dda_cells]
    return bits(acc), rgb.view(np.uint32), tuple(int(x) for x in tot)


@pytest.mark.parametrize("grids", [1, 2])
@pytest.mark.parametrize("depth", [0, 2])
@pytest.mark.parametrize("sphere", [False, True])
def test_instance_paths_bit_exact(pkg, orc, grids, depth, sphere):
    desc = lattice_scene(pkg, grids, depth, sphere)
    frames = 2
    a_o, r_o, c_o = oracle(orc, pkg, desc, frames)
    for lanes in (0, 3):
        a_g, r_g, c_g = render(pkg, desc, frames, lanes)
        assert np.array_equal(a_g, a_o), f"accumulator differs ({lanes} lanes)"
        assert np.array_equal(r_g, r_o), f"RGB8 differs ({lanes} lanes)"
        assert c_g == c_o, (lanes, c_g, c_o)
    assert c_o[1] > 0 and c_o[3] > 0


def test_library_loaded_before_torch():
    """A fresh process that loads libvpx_hip.so before importing torch (the package imports
    torch first, abi.load_library) creates a context: one HIP runtime in the process."""
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import __graft_entry__ as e\n"
            "pkg = e.load_package(); pkg.abi.load_library()\n"
            "import torch\n"
            "c = pkg.context.Context(0); c.close(); print('ctx ok')\n") % REPO
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ctx ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.parametrize("depth", [0, 2])
def test_static_camera_reprojection_instances(pkg, orc, depth):
    """Renderer::Tick's static branch (TraceReproject, renderer.cpp:1996-2101) over the instance
    lattice: at depth 0 the deferred instance pass shades the paths a later volume may change,
    including the reprojection's level-0 record; 3 frames, the live camera nudged after the
    first, RGB8 and the illumination history bit-exact."""
    sc = pkg.scene
    desc = lattice_scene(pkg, 1, depth)
    desc.flags = 0
    r = pkg.renderer.Renderer(desc, 0)
    r.Init()
    r.staticCamera = True
    o = orc.Oracle(pkg.abi, desc)
    hist_o = np.zeros((desc.width * desc.height, 4), np.float32)
    prev = sc.prev_camera(desc._cam_pos, desc._cam_target, desc.width, desc.height)
    for f in range(3):
        if f > 0:
            pos = tuple(np.float32(v) + np.float32((0.0, 0.004, 0.04)[f]) for v in desc._cam_pos)
            desc.camera = sc.look_at(pos, desc._cam_target, desc.width, desc.height)
            r.ctx.set_camera(desc.camera)
            o.set_camera(desc.camera)
        st = r.Tick(0.0, stats=True)
        torch.cuda.synchronize()
        rgb_g = r.screen_host().reshape(-1).copy()
        hist_g = r.history_host().reshape(-1, 4).copy()
        rgb_o, ost = o.render_reproject(desc.frame_params(f), prev, hist_o)
        assert np.array_equal(bits(hist_g), bits(hist_o)), f"frame {f}: history"
        assert np.array_equal(rgb_g, rgb_o), f"frame {f}: rgb8"
        assert (st.shadow_rays, st.bounce_rays, st.dda_cells) == (ost.shadow_rays, ost.bounce_rays, ost.dda_cells)
    r.ctx.close()


def _window_image(pkg, desc, first, n, lanes, pre=0):
    """`pre` per-frame renders, then frames pre .. pre + n - 1 as one vpx_render_window."""
    ctx = pkg.context.Context(0)
    s = torch.cuda.Stream()
    ctx.set_stream(s.cuda_stream)
    ctx.load_scene(desc)
    ctx.set_pipeline(lanes)
    W, H = desc.width, desc.height
    acc = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
    rgb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ctx.counters(reset=True)
    with torch.cuda.stream(s):
        for f in range(pre):
            ctx.render(desc.frame_params(f), acc.data_ptr(), rgb.data_ptr())
        ctx.render_window(desc.frame_params(first), n, acc.data_ptr(), rgb.data_ptr())
    ctx.synchronize()
    st = ctx.counters()
    out = (bits(acc.cpu().numpy().reshape(-1, 4)), rgb.cpu().numpy().view(np.uint32),
           tuple(int(getattr(st, k)) for k in ("primary_rays", "shadow_rays", "bounce_rays", "dda_cells")))
    ctx.close()
    return out


@pytest.mark.parametrize("depth", [0, 2])
def test_window_image_bit_exact(pkg, orc, depth):
    """vpx_render_window over the instance lattice (64x48: 12 tiles, so the whole window is one
    chain of launches, each frame in its own tile blocks with its own seeds): accumulator, RGB8
    and ray / cell counts equal the oracle's frame-by-frame accumulation, with and without
    lanes, from frame 0 and continuing a running average from frame 1."""
    desc = lattice_scene(pkg, 1, depth, sphere=True)
    frames = 4
    a_o, r_o, c_o = oracle(orc, pkg, desc, frames)
    for lanes in (0, 3):
        for pre in (0, 1):
            a_g, r_g, c_g = _window_image(pkg, desc, pre, frames - pre, lanes, pre)
            assert np.array_equal(a_g, a_o), f"accumulator differs (lanes {lanes}, pre {pre})"
            assert np.array_equal(r_g, r_o), f"RGB8 differs (lanes {lanes}, pre {pre})"
            assert c_g == c_o, (lanes, pre, c_g, c_o)


def _tiles_accum(pkg, desc, R, frames, lanes, window):
    ctx = pkg.context.Context(0)
    s = torch.cuda.Stream()
    ctx.set_stream(s.cuda_stream)
    ctx.load_scene(desc)
    ctx.set_pipeline(lanes)
    L = ctx.packed_len(desc.width, desc.height, R)
    out = []
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        for r in range(R):
            acc = torch.zeros(L * 4, dtype=torch.float32, device="cuda")
            rgb = torch.zeros(L, dtype=torch.int32, device="cuda")
            if window:
                ctx.render_tiles_accum_window(desc.frame_params(0), frames, r, R, acc.data_ptr(), rgb.data_ptr())
            else:
                for f in range(frames):
                    ctx.render_tiles_accum(desc.frame_params(f), r, R, acc.data_ptr(), rgb.data_ptr())
            out.append((acc, rgb))
    ctx.synchronize()
    res = [(bits(a.cpu().numpy().reshape(-1, 4)), g.cpu().numpy().view(np.uint32)) for a, g in out]
    ctx.close()
    return res


@pytest.mark.parametrize("depth", [0, 2])
def test_window_tiles_accum_matches_per_frame(pkg, depth):
    """vpx_render_tiles_accum_window against frame-by-frame vpx_render_tiles_accum (itself
    checked against the oracle in test_gpu_parity): 512x512 at 3 ranks (342 tiles a rank: the
    40 frames in one chain) and at one rank (1024 tiles: chains of 32 frames, so the window
    splits 32 + 8); lanes 0 and 3; every rank's packed accumulator and RGB8 bit-exact."""
    desc = lattice_scene(pkg, 2, depth).with_size(512, 512)
    desc.area_samples = 2
    for R in (3, 1):
        ref = _tiles_accum(pkg, desc, R, 40, 0, False)
        for lanes in (0, 3):
            got = _tiles_accum(pkg, desc, R, 40, lanes, True)
            for r in range(R):
                assert np.array_equal(got[r][0], ref[r][0]), f"R={R} rank {r} lanes {lanes}: accumulator"
                assert np.array_equal(got[r][1], ref[r][1]), f"R={R} rank {r} lanes {lanes}: RGB8"


@pytest.mark.parametrize("size", [(64, 40), (2048, 2048)])
@pytest.mark.parametrize("pipe", [3, 4])
def test_window_deep_area_lights_matches_per_frame(pkg, pipe, size):
    """Window chains with area lights (several slots per path) at depth 14 (the frames run
    k_tail) and depth 2 over the lattice.  At 2048x2048 (16384 tiles, VPX_WINDOW_FUSED) each
    chain blends in its own tail after the caller's event (k_finish_window, with the resolve at
    depth 2, without it after k_tail); small frames blend on the caller's stream.  Against
    frame-by-frame vpx_render on the stream (itself checked against the oracle): 6 frames,
    accumulator and RGB8 bit-exact."""
    sc = pkg.scene
    W, H = size
    for desc in (sc.city_scene("roomGlass", 128, W, H, 14, areas=sc.C3_AREAS[:2]), lattice_scene(pkg, 1, 2).with_size(W, H)):
        desc.area_samples = 3
        desc.flags = pkg.abi.VPX_FLAG_AA
        a_r, r_r, _ = render(pkg, desc, 6, 0)
        a_w, r_w, _ = _window_image(pkg, desc, 0, 6, pipe)
        assert np.array_equal(a_w, a_r), f"accumulator differs (depth {desc.max_bounces}, {pipe} lanes)"
        assert np.array_equal(r_w, r_r), f"RGB8 differs (depth {desc.max_bounces}, {pipe} lanes)"
