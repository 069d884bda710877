"""GPU parity: libvpx_hip.so (through the C-ABI) against the CPU restatement (oracle/).

The bar is bit-exactness: t, normals, materials, occlusion, cells visited and every float
of the radiance / accumulator, and every RGB8 byte.  The oracle itself is "parity
unpinned" against the reference; these tests pin the GPU to the oracle.
"""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)


from cases import SCENES, bits, random_rays  # noqa: E402


def make_ctx(pkg, desc):
    ctx = pkg.context.Context(0)
    ctx.load_scene(desc)
    return ctx


def cmp_hits(pkg, gh, oh, n):
    g = pkg.context.hits_to_numpy(gh, n)
    o = pkg.context.hits_to_numpy(oh, n)
    for f in ("vox_index", "material", "cells", "inside_glass"):
        assert np.array_equal(g[f], o[f]), f
    assert np.array_equal(bits(g["t"]), bits(o["t"]))
    assert np.array_equal(bits(g["normal"]), bits(o["normal"]))
    return g


@pytest.mark.parametrize("name", sorted(SCENES))
def test_find_nearest_and_occlusion(pkg, orc, name):
    desc = SCENES[name](pkg.scene)
    ctx = make_ctx(pkg, desc)
    o = orc.Oracle(pkg.abi, desc)
    org, dirs = random_rays(4096, 7)
    rays = pkg.context.make_rays(org, dirs)
    g = cmp_hits(pkg, ctx.find_nearest(rays), o.find_nearest(rays), len(rays))
    assert (g["vox_index"] >= 0).mean() > 0.1  # the test hits something
    srays = pkg.context.make_rays(org, dirs, tmax=np.random.default_rng(3).uniform(0.05, 3.0, len(org)))
    occ_g = ctx.is_occluded(srays)
    occ_o, _ = o.is_occluded(srays)
    assert np.array_equal(occ_g, occ_o)
    ctx.close()


@pytest.mark.parametrize("name", sorted(SCENES))
@pytest.mark.parametrize("depth", [0, 4, 14])
def test_trace_rays(pkg, orc, name, depth):
    desc = SCENES[name](pkg.scene)
    ctx = make_ctx(pkg, desc)
    o = orc.Oracle(pkg.abi, desc)
    org, dirs = random_rays(2048, 11 + depth)
    rays = pkg.context.make_rays(org, dirs, inside=(np.arange(len(org)) % 5 == 0).astype(np.uint32))
    seeds = np.random.default_rng(depth).integers(1, 2**32 - 1, len(org), dtype=np.uint64).astype(np.uint32)
    rg = ctx.trace(rays, seeds, depth, desc.sky, desc.area_samples)
    ro, _ = o.trace(rays, seeds, depth, desc.sky, desc.area_samples)
    assert np.array_equal(bits(rg), bits(ro))
    ctx.close()


def render_gpu(pkg, desc, frames=1, flags=None):
    r = pkg.renderer.Renderer(desc, 0)
    if flags is not None:
        desc.flags = flags
    r.Init()
    stats = []
    for _ in range(frames):
        stats.append(r.Tick(0.0, stats=True))
    torch.cuda.synchronize()
    acc, rgb = r.accumulator_host().reshape(-1, 4).copy(), r.screen_host().reshape(-1).copy()
    r.ctx.close()
    return acc, rgb, stats


@pytest.mark.parametrize("name", sorted(SCENES))
def test_render_frame_bit_exact(pkg, orc, name):
    desc = SCENES[name](pkg.scene)
    acc_g, rgb_g, st = render_gpu(pkg, desc)
    o = orc.Oracle(pkg.abi, desc)
    acc_o, rgb_o, ost = o.render(desc.frame_params(0))
    assert np.array_equal(bits(acc_g), bits(acc_o))
    assert np.array_equal(rgb_g, rgb_o)
    s = st[0]
    assert (s.primary_rays, s.shadow_rays, s.bounce_rays, s.dda_cells) == (
        ost.primary_rays, ost.shadow_rays, ost.bounce_rays, ost.dda_cells)


@pytest.mark.parametrize("depth", [-1, 0, 1, 3])
@pytest.mark.parametrize("lights", ["points", "areas"])
def test_depth_sweep_fused_head_tail(pkg, orc, depth, lights):
    """The fused kernels' edges: level 0 shaded inside k_primary, the last level's IsOccluded
    + light resolve + finish in k_shadow_finish (several area-light slots per path), and
    Trace(ray, -1) (no level runs: the plain finish folds the zero leaf).  Two frames, so the
    running average goes through the fused finish twice."""
    sc = pkg.scene
    areas = sc.C3_AREAS[:2] if lights == "areas" else None
    desc = sc.city_scene("roomGlass", 128, 48, 40, depth, areas=areas)
    desc.area_samples = 3
    acc_g, rgb_g, st = render_gpu(pkg, desc, frames=2)
    o = orc.Oracle(pkg.abi, desc)
    acc = None
    ost = None
    for f in range(2):
        acc, rgb, ost = o.render(desc.frame_params(f), accum=acc)
    assert np.array_equal(bits(acc_g), bits(acc))
    assert np.array_equal(rgb_g, rgb)
    s = st[-1]
    assert (s.primary_rays, s.shadow_rays, s.bounce_rays, s.dda_cells) == (
        ost.primary_rays, ost.shadow_rays, ost.bounce_rays, ost.dda_cells)
    if depth >= 0:
        assert s.shadow_rays > 0
    else:
        assert s.bounce_rays == 0 and s.dda_cells == 0


@pytest.mark.parametrize("samples,wh,depth", [(2, (16, 16), 0), (15, (40, 24), 2), (7, (96, 64), 1)])
def test_pools_slot_counts(pkg, orc, samples, wh, depth):
    """The pools: bounce walks of every level and the area-light shadow walks
    by persistent waves that refill finished lanes.  Edges: one tile (a single grab), 15 slots
    per path (a grab of one mask word, up to 960 listed slots per wave), 2 slots per path; the
    shadow results go through occb to k_resolve (depth > 0) and k_resolve_finish."""
    sc = pkg.scene
    desc = sc.city_scene("roomGlass", 128, wh[0], wh[1], depth, areas=sc.C3_AREAS)
    desc.area_samples = samples
    acc_g, rgb_g, st = render_gpu(pkg, desc, frames=2)
    o = orc.Oracle(pkg.abi, desc)
    acc = None
    ost = None
    for f in range(2):
        acc, rgb, ost = o.render(desc.frame_params(f), accum=acc)
    assert np.array_equal(bits(acc_g), bits(acc))
    assert np.array_equal(rgb_g, rgb)
    s = st[-1]
    assert (s.primary_rays, s.shadow_rays, s.bounce_rays, s.dda_cells) == (
        ost.primary_rays, ost.shadow_rays, ost.bounce_rays, ost.dda_cells)
    assert s.shadow_rays > 0


@pytest.mark.parametrize("depth", [13, 14])
def test_deepest_levels(pkg, orc, depth):
    """Renderer::maxBounces = 14 (renderer.h:175), the API's maximum: 15 levels of records
    in the per-path forms word (2 bits a level + the sentinel that marks the count).  The
    tiled glass rooms keep paths alive to the last level (checked: depth d casts more bounce
    rays than depth d - 1); two frames, every float and byte equal to the oracle."""
    sc = pkg.scene
    desc = sc.city_scene("roomGlass", 128, 64, 48, depth)
    acc_g, rgb_g, st = render_gpu(pkg, desc, frames=2)
    o = orc.Oracle(pkg.abi, desc)
    acc = None
    for f in range(2):
        acc, rgb, ost = o.render(desc.frame_params(f), accum=acc)
    assert np.array_equal(bits(acc_g), bits(acc))
    assert np.array_equal(rgb_g, rgb)
    s = st[-1]
    assert (s.primary_rays, s.shadow_rays, s.bounce_rays, s.dda_cells) == (
        ost.primary_rays, ost.shadow_rays, ost.bounce_rays, ost.dda_cells)
    desc.max_bounces = depth - 1
    _, _, shallower = o.render(desc.frame_params(1))
    assert ost.bounce_rays > shallower.bounce_rays  # some paths reach level `depth`


def test_progressive_accumulation_aa(pkg, orc):
    """4 frames with AA jitter: running average w = 1/(n+1), seeds advance per frame."""
    desc = pkg.scene.model_scene("monu3", 128, 80, 48, 1, city_lights=True)
    desc.flags = pkg.abi.VPX_FLAG_AA
    acc_g, rgb_g, _ = render_gpu(pkg, desc, frames=4)
    o = orc.Oracle(pkg.abi, desc)
    acc = None
    for f in range(4):
        acc, rgb, _ = o.render(desc.frame_params(f), accum=acc)
    assert np.array_equal(bits(acc_g), bits(acc))
    assert np.array_equal(rgb_g, rgb)


def test_dof_focus(pkg, orc):
    desc = pkg.scene.model_scene("monu3", 128, 64, 40, 0, city_lights=True)
    desc.flags = pkg.abi.VPX_FLAG_AA | pkg.abi.VPX_FLAG_DOF
    ctx = make_ctx(pkg, desc)
    o = orc.Oracle(pkg.abi, desc)
    fd = ctx.focus_distance(desc.width, desc.height)
    assert np.float32(fd).view(np.uint32) == np.float32(o.focus_distance(desc.width, desc.height)).view(np.uint32)
    ctx.close()
    desc.camera.focal_distance = fd
    acc_g, rgb_g, _ = render_gpu(pkg, desc)
    o.set_camera(desc.camera)
    acc_o, rgb_o, _ = o.render(desc.frame_params(0))
    assert np.array_equal(bits(acc_g), bits(acc_o))


@pytest.mark.parametrize("wh", [(1, 1), (17, 5), (33, 31)])
def test_odd_frame_sizes(pkg, orc, wh):
    desc = pkg.scene.model_scene("monu3", 128, wh[0], wh[1], 2, city_lights=True)
    acc_g, rgb_g, _ = render_gpu(pkg, desc)
    acc_o, rgb_o, _ = orc.Oracle(pkg.abi, desc).render(desc.frame_params(0))
    assert np.array_equal(bits(acc_g), bits(acc_o)) and np.array_equal(rgb_g, rgb_o)


def test_tiles_composite_equals_monolithic(pkg, orc):
    """Multi-GPU layout on one device: R ranks' packed tiles -> composite == vpx_render."""
    desc = pkg.scene.city_scene("monu3", 128, 100, 70, 0)
    acc_ref, rgb_ref, _ = render_gpu(pkg, desc)
    ctx = make_ctx(pkg, desc)
    R = 3
    L = ctx.packed_len(desc.width, desc.height, R)
    gathered = torch.zeros(R * L * 4, dtype=torch.float32, device="cuda")
    p = desc.frame_params(0)
    for rank in range(R):
        ctx.render_tiles(p, rank, R, gathered.data_ptr() + rank * L * 16)
    acc = torch.zeros(desc.width * desc.height * 4, dtype=torch.float32, device="cuda")
    rgb = torch.zeros(desc.width * desc.height, dtype=torch.int32, device="cuda")
    ctx.composite_tiles(p, R, gathered.data_ptr(), acc.data_ptr(), rgb.data_ptr())
    ctx.synchronize()
    assert np.array_equal(bits(acc.cpu().numpy().reshape(-1, 4)), bits(acc_ref))
    assert np.array_equal(rgb.cpu().numpy().view(np.uint32), rgb_ref)
    ctx.close()


def test_sharded_accumulator_equals_monolithic(pkg, orc):
    """The bench's multi-GPU flow on one device: R ranks accumulate their own tiles
    (vpx_render_tiles_accum) over 3 AA frames, rank 0 scatters the RGB8 (vpx_composite_rgb8);
    screen and every rank's packed accumulator equal vpx_render's frames bit for bit."""
    desc = pkg.scene.city_scene("monu3", 128, 100, 70, 1)
    desc.flags = pkg.abi.VPX_FLAG_AA
    acc_ref, rgb_ref, _ = render_gpu(pkg, desc, frames=3)
    ctx = make_ctx(pkg, desc)
    R = 3
    W, H = desc.width, desc.height
    L = ctx.packed_len(W, H, R)
    accs = [torch.zeros(L * 4, dtype=torch.float32, device="cuda") for _ in range(R)]
    gathered = torch.zeros(R * L, dtype=torch.int32, device="cuda")
    rgb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    for f in range(3):
        p = desc.frame_params(f)
        for rank in range(R):
            ctx.render_tiles_accum(p, rank, R, accs[rank].data_ptr(), gathered.data_ptr() + rank * L * 4)
        ctx.composite_rgb8(p, R, gathered.data_ptr(), rgb.data_ptr())
    ctx.synchronize()
    assert np.array_equal(rgb.cpu().numpy().view(np.uint32), rgb_ref)
    acc_img = pkg.dist.unpack(np.concatenate([a.cpu().numpy() for a in accs]), W, H, R)
    assert np.array_equal(bits(acc_img), bits(acc_ref))
    ctx.close()


def test_fused_frame_equals_two_launch_frame(pkg):
    """The depth-0 frame runs as one launch (k_frame0) up to kFuseFrameTiles (12288)
    tiles and as k_primary + k_shadow_finish above.  The same 2048x1600 frame (12800 tiles)
    rendered whole (two launches) and as two ranks' halves (6400 tiles each: fused) must
    agree bit for bit over 2 AA frames with the city's point and directional lights (one
    shadow slot per path: k_frame0 keeps it in LDS; area lights take the split frame and the
    shadow pool); the profile names the stage each path ran (frame vs primary + shadow) and
    the cells add up."""
    sc = pkg.scene
    desc = sc.city_scene("monu3", 128, 2048, 1600, 0)
    desc.flags = pkg.abi.VPX_FLAG_AA
    W, H = desc.width, desc.height
    ctx = make_ctx(pkg, desc)
    acc = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
    rgb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    R = 2
    L = ctx.packed_len(W, H, R)
    accs = [torch.zeros(L * 4, dtype=torch.float32, device="cuda") for _ in range(R)]
    gathered = torch.zeros(R * L, dtype=torch.int32, device="cuda")
    rgb_sh = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ctx.profile_enable(64)
    for f in range(2):
        p = desc.frame_params(f)
        ctx.profile_read(reset=True)
        ctx.render(p, acc.data_ptr(), rgb.data_ptr())
        whole = ctx.profile_read(reset=True)
        for rank in range(R):
            ctx.render_tiles_accum(p, rank, R, accs[rank].data_ptr(), gathered.data_ptr() + rank * L * 4)
        halves = ctx.profile_read(reset=True)
        ctx.composite_rgb8(p, R, gathered.data_ptr(), rgb_sh.data_ptr())
        assert whole["frame"][1] == 0 and whole["primary"][1] == 1 and whole["shadow"][1] == 1
        assert halves["frame"][1] == R and halves["primary"][1] == 0 and halves["shadow"][1] == 0
        assert sum(v[2] for v in whole.values()) == sum(v[2] for v in halves.values()) > 0
    ctx.synchronize()
    assert np.array_equal(rgb_sh.cpu().numpy(), rgb.cpu().numpy())
    acc_img = pkg.dist.unpack(np.concatenate([a.cpu().numpy() for a in accs]), W, H, R)
    assert np.array_equal(bits(acc_img).reshape(-1), bits(acc.cpu().numpy()).reshape(-1))
    ctx.close()


def _hip_current_device():
    import ctypes as C
    d = C.c_int(-1)
    assert C.CDLL("libamdhip64.so").hipGetDevice(C.byref(d)) == 0
    return d.value


# [0, 1]: distinct devices take the in-library RCCL path (ncclCommInitAll, grouped
# ncclSend / ncclRecv into device 0); it runs only where a node has two GPUs (the one-GPU
# test box skips it and exercises the repeated-device copy path).
@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0, 0],
                                     pytest.param([0, 1], marks=pytest.mark.skipif(
                                         torch.cuda.device_count() < 2, reason="distinct-device RCCL path needs 2 GPUs"))])
def test_device_set_equals_single_device(pkg, orc, devices):
    """vpx_create_multi: the frame's tiles dealt over the members, gathered to devices[0]
    and composited there.  With an accumulator (float4 samples travel) the accumulator and
    screen equal vpx_render's bit for bit over 3 AA frames at depth 1 with area lights; with
    accum = NULL (members keep their tiles' running averages, RGB8 travels) the screen
    does; the summed counters equal one device's."""
    sc = pkg.scene
    desc = sc.city_scene("monu3", 128, 100, 70, 1, areas=sc.C3_AREAS[:2])
    desc.flags = pkg.abi.VPX_FLAG_AA
    acc_ref, rgb_ref, st_ref = render_gpu(pkg, desc, frames=3)
    torch.cuda.set_device(0)
    ctx = pkg.context.Context(devices=devices)
    ctx.load_scene(desc)
    # every forwarded call restores the caller's device (the buffers below belong on devices[0])
    assert _hip_current_device() == 0
    W, H = desc.width, desc.height
    acc = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
    rgb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    rgb2 = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ctx.counters(reset=True)
    for f in range(3):
        st = ctx.render(desc.frame_params(f), acc.data_ptr(), rgb.data_ptr(), stats=True)
    ctx.synchronize()
    assert np.array_equal(bits(acc.cpu().numpy().reshape(-1, 4)), bits(acc_ref))
    assert np.array_equal(rgb.cpu().numpy().view(np.uint32), rgb_ref)
    s, r = st, st_ref[-1]
    assert (s.primary_rays, s.shadow_rays, s.bounce_rays, s.dda_cells) == (
        r.primary_rays, r.shadow_rays, r.bounce_rays, r.dda_cells)
    for f in range(3):
        ctx.render(desc.frame_params(f), 0, rgb2.data_ptr())
    ctx.synchronize()
    assert np.array_equal(rgb2.cpu().numpy().view(np.uint32), rgb_ref)
    tot = ctx.counters()
    assert tot.primary_rays == 6 * W * H
    assert _hip_current_device() == 0
    ctx.close()


def test_zero_copy_screen_in_mapped_host_memory(pkg):
    """SURVEY §8(f) rank 2, display path without GL interop in this image: Surface::pixels
    allocated as mapped pinned host memory (hipHostMalloc(..., hipHostMallocMapped)) and its
    device alias handed to vpx_render as rgb8 — the frame's RGB8 lands in the host buffer the
    GL upload reads (template/opengl.cpp:144-149), with no hipMemcpy, byte-equal to the
    device-buffer frame."""
    import ctypes as C

    hip = C.CDLL("libamdhip64.so")
    desc = pkg.scene.city_scene("monu3", 128, 96, 64, 0)
    acc_ref, rgb_ref, _ = render_gpu(pkg, desc)
    n = desc.width * desc.height
    host = C.c_void_p()
    assert hip.hipHostMalloc(C.byref(host), C.c_size_t(4 * n), C.c_uint(0x2)) == 0  # hipHostMallocMapped
    dev = C.c_void_p()
    assert hip.hipHostGetDevicePointer(C.byref(dev), host, C.c_uint(0)) == 0
    try:
        ctx = make_ctx(pkg, desc)
        acc = torch.zeros(n * 4, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        ctx.render(desc.frame_params(0), acc.data_ptr(), dev.value)
        ctx.synchronize()
        screen = np.ctypeslib.as_array((C.c_uint32 * n).from_address(host.value)).copy()
        assert np.array_equal(screen, rgb_ref)
        ctx.close()
    finally:
        hip.hipHostFree(host)


GL_PROBE = r"""
import ctypes as C, sys
sys.path.insert(0, sys.argv[1])
import __graft_entry__ as entry
pkg = entry.load_package()
lib, abi = pkg.load_library(), pkg.abi
h = C.c_void_p()
assert lib.vpx_create(0, C.byref(h)) == abi.VPX_OK
ptr, n = C.c_void_p(), C.c_size_t()
assert lib.vpx_gl_map(h, C.byref(ptr), C.byref(n)) == abi.VPX_E_STATE      # nothing registered
assert lib.vpx_gl_unmap(h) == abi.VPX_E_STATE                              # nothing mapped
rc = lib.vpx_gl_register_buffer(h, 1)                                       # no GL context here
assert rc == abi.VPX_E_DEVICE, rc
assert b"hipGraphicsGLRegisterBuffer" in lib.vpx_last_error(h)
assert lib.vpx_gl_map(h, C.byref(ptr), C.byref(n)) == abi.VPX_E_STATE      # the failed register left none
assert lib.vpx_gl_register_buffer(h, 0) == abi.VPX_OK                       # unregister: a no-op
assert lib.vpx_destroy(h) == abi.VPX_OK
print("gl-refusal-ok")
"""


def test_gl_interop_refuses_cleanly_without_a_gl_context(pkg):
    """§8(f)2 display interop (vpx_gl_register_buffer / vpx_gl_map / vpx_gl_unmap): this image
    has libGL but no display, so no GL context can exist and the interop itself is
    unmeasured; what is checked is the failure path — out-of-order calls are VPX_E_STATE,
    registering without a current GL context is VPX_E_DEVICE with HIP's message, and the
    context stays usable.  In a child process, so a HIP runtime that mishandles the missing
    context cannot take the suite down."""
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", GL_PROBE, repo], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "gl-refusal-ok" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])


def test_sharded_accum_frame_refuses_a_foreign_stream(pkg):
    """RCCL orders the gather after torch's current stream, so the sharded flow refuses a
    context that renders on another stream instead of gathering stale RGB8."""
    desc = pkg.scene.city_scene("monu3", 128, 64, 48, 0)
    ctx = make_ctx(pkg, desc)  # the context's own stream
    with pytest.raises(ValueError):
        pkg.dist.ShardedAccumFrame(ctx, desc, 0, 2, torch.device("cuda", 0))
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        ctx.set_stream(s.cuda_stream)
        pkg.dist.ShardedAccumFrame(ctx, desc, 0, 2, torch.device("cuda", 0))
    ctx.close()


def test_tiled_world_generator_matches_oracle(pkg, orc):
    for model, n in (("monu3", 256), ("roomGlass", 320)):
        spec, _, _ = pkg.scene.tiled_grid(model, n)
        ctx = pkg.context.Context(0)
        spec.upload(ctx.lib, ctx.h, 0)
        o = orc.Oracle.__new__(orc.Oracle)
        o.lib = orc._lib(pkg.abi)
        cells = o.host_grid(spec)
        assert ctx.grid_checksum(0) == o.lib.oracle_grid_checksum(cells.ctypes.data, cells.size)
        ctx.close()


def test_multi_volume_transforms_shapes(pkg, orc):
    """Several transformed volumes sharing grids, plus spheres and triangles
    (renderer.cpp:946-1018 linear loop, ties to the lowest index)."""
    sc, abi = pkg.scene, pkg.abi
    desc = sc.model_scene("monu3", 64, 64, 48, 3, city_lights=True)
    size, vox, _ = sc.load_model("teapot")
    desc.grids.append(sc.GridSpec(n=32, dense=sc.load_model_grid(size, vox, 32)))
    vols = [sc.volume()]
    vols.append(sc.volume((0.6, 0.0, 0.2), (0.5, 0.5, 0.5), (0.0, 0.7, 0.0), grid_id=1))
    vols.append(sc.volume((-0.4, 0.1, 0.3), (1.0, 0.5, 2.0), (0.3, 0.2, 0.1), grid_id=0))
    vols.append(sc.volume((0.0, 0.0, 0.0), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0), grid_id=0))  # exact duplicate: tie
    desc.volumes = (abi.Volume * len(vols))(*vols)
    desc.spheres = [abi.Sphere(abi.vec3((0.3, 0.8, 0.4)), 0.15, 8), abi.Sphere(abi.vec3((0.8, 0.2, 0.1)), 0.1, 15)]
    tri = abi.Triangle(abi.vec3((0.5, 0.6, 0.0)), abi.vec3((-0.25, 0, 0)), abi.vec3((0, 0.25, 0)),
                       abi.vec3((0.25, 0, 0)), 5)
    desc.triangles = [tri]
    desc.spots = [sc.spot_light((0.5, 1.2, 0.5), (0.0, -1.0, 0.0), (2.0, 2.0, 2.0))]
    desc.areas = [sc.area_light((0.5, 1.5, -0.5), radius=0.3)]
    ctx = make_ctx(pkg, desc)
    o = orc.Oracle(pkg.abi, desc)
    org, dirs = random_rays(4096, 5)
    rays = pkg.context.make_rays(org, dirs)
    cmp_hits(pkg, ctx.find_nearest(rays), o.find_nearest(rays), len(rays))
    ctx.close()
    acc_g, rgb_g, _ = render_gpu(pkg, desc)
    acc_o, rgb_o, _ = o.render(desc.frame_params(0))
    assert np.array_equal(bits(acc_g), bits(acc_o)) and np.array_equal(rgb_g, rgb_o)


def test_volume_cull_grazing_rays(pkg, orc):
    """The device culls volumes whose inflated world bounding sphere a ray misses
    (vpx_trace.hpp misses_volume); rays aimed at the corners and edges of rotated, scaled
    instances, from outside and inside them, must still match the oracle's full loop."""
    sc, abi = pkg.scene, pkg.abi
    desc = sc.model_scene("monu3", 64, 32, 24, 0, city_lights=True)
    vols = [sc.volume((0.1, 0.1, 0.1), (0.1, 0.1, 0.1), (0.3, 1.1, 0.2))]
    rng = np.random.default_rng(11)
    for _ in range(12):
        pos = tuple(rng.uniform(-1.0, 1.0, 3))
        scl = tuple(rng.uniform(0.05, 0.4, 3))
        rot = tuple(rng.uniform(-3.1, 3.1, 3))
        vols.append(sc.volume(pos, scl, rot, grid_id=0))
    desc.volumes = (abi.Volume * len(vols))(*vols)
    targets = []
    for v in vols:
        m = np.array(v.matrix, np.float64).reshape(4, 4)
        b0, b1 = np.array(v.b0, np.float64), np.array(v.b1, np.float64)
        for _ in range(96):
            u = rng.integers(0, 2, 3).astype(np.float64)
            u[rng.integers(0, 3)] = rng.uniform(0, 1)  # a point on an edge (or a corner)
            p = b0 + (b1 - b0) * u + rng.normal(0, 1e-5, 3) * (b1 - b0)
            targets.append((m @ np.append(p, 1.0))[:3])
    targets = np.array(targets)
    org = targets + rng.normal(0, 1, targets.shape) * rng.choice([0.02, 0.5, 2.0], (len(targets), 1))
    org = np.concatenate([org, targets[::-1] + rng.normal(0, 1e-3, targets.shape)])
    tgt = np.concatenate([targets, targets])
    rays = pkg.context.make_rays(org.astype(np.float32), (tgt - org).astype(np.float32))
    ctx = make_ctx(pkg, desc)
    o = orc.Oracle(pkg.abi, desc)
    g = cmp_hits(pkg, ctx.find_nearest(rays), o.find_nearest(rays), len(rays))
    assert (g["vox_index"] >= 1).sum() > 50  # instances are hit, not only the main grid
    srays = pkg.context.make_rays(org.astype(np.float32), (tgt - org).astype(np.float32),
                                  tmax=rng.uniform(0.05, 5.0, len(org)))
    occ_o, _ = o.is_occluded(srays)
    assert np.array_equal(ctx.is_occluded(srays), occ_o)
    ctx.close()


@pytest.mark.parametrize("n_inst", [40, 64, 100])
def test_instance_tlas_many_volumes(pkg, orc, n_inst):
    """The instance TLAS (vpx_set_volumes builds it for 2..65 volumes; 101 volumes take the
    linear loop): a world volume plus a lattice of rotated, scaled instances (C4's shape),
    an exact duplicate (tie -> lowest index) and a degenerate scale-0 volume (no finite
    bounds: always a candidate).  Hits, cell counts, occlusion and a frame with area lights
    (the multi-volume kernels read the TLAS from LDS) equal the oracle's linear loop."""
    sc, abi = pkg.scene, pkg.abi
    desc = sc.model_scene("monu3", 64, 48, 40, 1, city_lights=True)
    size, vox, _ = sc.load_model("monu3")
    desc.grids.append(sc.GridSpec(n=32, dense=sc.load_model_grid(size, vox, 32)))
    rng = np.random.default_rng(n_inst)
    vols = [sc.volume()]
    for k in range(n_inst - 2):
        i, j, l = k % 5, (k // 5) % 5, k // 25
        pos = (0.2 * i - 0.4, 0.55 + 0.2 * j, 0.2 * l - 0.4)
        vols.append(sc.volume(pos, tuple(rng.uniform(0.05, 0.15, 3)), tuple(rng.uniform(-3, 3, 3)), grid_id=1))
    vols.append(vols[5])  # duplicate of volume 5: equal t, the lower index wins
    vols.append(sc.volume((0.3, 0.3, 0.3), (0.0, 0.1, 0.1), (0.0, 0.0, 0.0), grid_id=1))  # singular
    desc.volumes = (abi.Volume * len(vols))(*vols)
    desc.areas = [sc.area_light((0.5, 2.0, 0.5), radius=0.4)]
    ctx = make_ctx(pkg, desc)
    o = orc.Oracle(pkg.abi, desc)
    org, dirs = random_rays(4096, 17)
    cen = np.array([np.array(v.matrix, np.float64).reshape(4, 4) @ [0.5, 0.5, 0.5, 1.0] for v in vols])[:, :3]
    org2 = rng.uniform(-1.5, 2.5, (2048, 3))
    dirs2 = cen[rng.integers(1, len(vols), 2048)] - org2 + rng.normal(0, 0.02, (2048, 3))
    org, dirs = np.concatenate([org, org2]).astype(np.float32), np.concatenate([dirs, dirs2]).astype(np.float32)
    rays = pkg.context.make_rays(org, dirs)
    g = cmp_hits(pkg, ctx.find_nearest(rays), o.find_nearest(rays), len(rays))
    assert (g["vox_index"] >= 1).sum() > 200
    srays = pkg.context.make_rays(org, dirs, tmax=rng.uniform(0.05, 4.0, len(org)))
    occ_o, _ = o.is_occluded(srays)
    assert np.array_equal(ctx.is_occluded(srays), occ_o)
    ctx.close()
    acc_g, rgb_g, st = render_gpu(pkg, desc)
    acc_o, rgb_o, ost = o.render(desc.frame_params(0))
    assert np.array_equal(bits(acc_g), bits(acc_o)) and np.array_equal(rgb_g, rgb_o)
    s = st[0]
    assert (s.shadow_rays, s.bounce_rays, s.dda_cells) == (ost.shadow_rays, ost.bounce_rays, ost.dda_cells)


@pytest.mark.parametrize("n", [64, 1, 7, 512])
def test_bvh_intersect(pkg, orc, n):
    """BasicBVH::IntersectBVH on the device (LDS-staged tree, explicit stack) equals the
    oracle's recursive restatement bit for bit; n = 64 is the reference constructor's set."""
    abi = pkg.abi
    rng = np.random.default_rng(n)
    if n == 64:
        tris, _ = orc.BasicBVH.random_tris(abi)
    else:
        a = rng.uniform(-5, 4, (n, 3))
        v = np.concatenate([a, a + rng.uniform(0, 1, (n, 3)), a + rng.uniform(0, 1, (n, 3))], 1).astype(np.float32)
        tris = (abi.BvhTri * n)()
        np.frombuffer(tris, np.float32).reshape(-1, 9)[:] = v
    o = orc.BasicBVH(abi, tris)
    cen = np.frombuffer(tris, np.float32).reshape(n, 3, 3).mean(1)
    m = 8192
    org = np.concatenate([rng.uniform(-8, 8, (m // 2, 3)), cen[rng.integers(0, n, m // 2)] + rng.normal(0, 0.3, (m // 2, 3))])
    tgt = cen[rng.integers(0, n, m)] + rng.normal(0, 0.05, (m, 3))
    tmax = np.where(rng.random(m) < 0.3, rng.uniform(0.1, 10, m), 1e34)
    rays = pkg.context.make_rays(org.astype(np.float32), (tgt - org).astype(np.float32), tmax=tmax)
    ctx = pkg.context.Context(0)
    ctx.bvh_set(tris)
    t_g = ctx.bvh_intersect(rays)
    t_o = o.intersect(rays)
    assert np.array_equal(bits(t_g), bits(t_o))
    assert (t_o < 1e33).mean() > 0.1
    with pytest.raises(pkg.abi.VpxError):
        ctx.bvh_set((abi.BvhTri * (abi.BVH_MAX_TRIS + 1))())
    # a degenerate chain deeper than the device traversal stack is refused, not traversed
    with pytest.raises(pkg.abi.VpxError, match="VPX_BVH_MAX_DEPTH"):
        ctx.bvh_set(chain_tris(abi, 80))
    ctx.close()


def chain_tris(abi, n):
    """Triangles with centroids at x = 2^i: every midpoint split peels off the last one, so
    the tree is a chain n deep (the reference's recursion has no depth cap)."""
    v = np.zeros((n, 9), np.float32)
    x = np.float32(2.0) ** np.arange(n, dtype=np.float32)
    v[:, 0], v[:, 3], v[:, 6] = x, x, x
    v[:, 4], v[:, 8] = 1.0, 1.0
    tris = (abi.BvhTri * n)()
    np.frombuffer(tris, np.float32).reshape(-1, 9)[:] = v
    return tris


def test_smoke_material_exits(pkg, orc):
    """Smoke and glass volumes exercise FindSmokeExit / FindMaterialExit."""
    sc = pkg.scene
    desc = sc.model_scene("monu3", 64, 64, 48, 6, city_lights=True)
    g = desc.grids[0].dense.reshape(64, 64, 64).copy()
    g[20:40, 5:30, 20:44] = 11          # smoke block
    g[40:50, 30:40, 10:30] = 8          # glass block
    g[5:10, 40:45, 5:60] = 15           # emissive bar
    desc.grids[0].dense = g.reshape(-1)
    acc_g, rgb_g, _ = render_gpu(pkg, desc)
    acc_o, rgb_o, _ = orc.Oracle(pkg.abi, desc).render(desc.frame_params(0))
    assert np.array_equal(bits(acc_g), bits(acc_o)) and np.array_equal(rgb_g, rgb_o)


@pytest.mark.parametrize("fill", [255, 0, 7])
def test_degenerate_worlds(pkg, orc, fill):
    """Empty world (all NONE), full diffuse world, full mirror world; camera inside."""
    sc = pkg.scene
    desc = sc.model_scene("monu3", 32, 40, 24, 4, cam=((0.5, 0.5, 0.5), (0.9, 0.2, 0.7)), city_lights=True)
    desc.grids[0].dense = np.full(32 ** 3, fill, np.uint8)
    acc_g, rgb_g, _ = render_gpu(pkg, desc)
    acc_o, rgb_o, _ = orc.Oracle(pkg.abi, desc).render(desc.frame_params(0))
    assert np.array_equal(bits(acc_g), bits(acc_o)) and np.array_equal(rgb_g, rgb_o)


@pytest.mark.parametrize("devices", [None, "0", "0,0,0"])
def test_cpp_host_demo_matches_oracle(pkg, orc, tmp_path, devices):
    """The C++ host mirror (host/vpx_renderer.cpp via host/vpx_demo) drives the C-ABI like the
    integrated game loop would: 3 accumulated frames, depth 1, equal to the oracle — on one
    device, and through a device set (vpx_create_multi; this box has one GPU, so the sets
    are {0} and three members on device 0, which gather by device copies: the RCCL path of
    distinct devices is unmeasured here)."""
    import subprocess

    exe = os.path.join(os.path.dirname(pkg.__file__), "host", "vpx_demo")
    if not os.path.exists(exe):
        pytest.fail("host/vpx_demo missing: run __graft_entry__.build()")
    n, w, h, frames, depth = 64, 96, 64, 3, 1
    out = tmp_path / "frame.rgb8"
    args = [exe, str(n), str(w), str(h), str(frames), str(depth), str(out)] + (["-", devices] if devices else [])
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    rgb_cpp = np.fromfile(out, np.uint32)
    desc = pkg.scene.pillars_scene(n, w, h, depth)
    o = orc.Oracle(pkg.abi, desc)
    acc = None
    for f in range(frames):
        acc, rgb, _ = o.render(desc.frame_params(f), accum=acc)
    assert np.array_equal(rgb_cpp, rgb)


def test_cpp_host_demo_asan(pkg, orc, tmp_path):
    """The C++ host mirror built with ASan + UBSan on its host code (-Xarch_host), 3 frames
    through the device, equal to the oracle and free of sanitizer reports."""
    import subprocess

    exe = os.path.join(os.path.dirname(pkg.__file__), "host", "vpx_demo_asan")
    n, w, h, frames, depth = 64, 64, 40, 3, 1
    out = tmp_path / "frame.rgb8"
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:protect_shadow_gap=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe, str(n), str(w), str(h), str(frames), str(depth), str(out)], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Sanitizer" not in r.stderr
    desc = pkg.scene.pillars_scene(n, w, h, depth)
    o = orc.Oracle(pkg.abi, desc)
    acc = None
    for f in range(frames):
        acc, rgb, _ = o.render(desc.frame_params(f), accum=acc)
    assert np.array_equal(np.fromfile(out, np.uint32), rgb)


def demo_sky(w=64, h=32):
    """host/vpx_demo.cpp demo_sky, restated in float32."""
    v, u = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    t = np.empty((h, w, 3), np.float32)
    t[..., 0] = u.astype(np.float32) / np.float32(w - 1) * np.float32(2.0)
    t[..., 1] = v.astype(np.float32) / np.float32(h - 1)
    t[..., 2] = np.float32(0.5) + ((u + v) % 7).astype(np.float32)
    return t


def test_cpp_host_demo_static_camera_sky(pkg, orc, tmp_path):
    """The C++ mirror's static-camera Tick (vpx_render_reproject) with activateSky, against
    the oracle's static branch: 2 frames, depth 2."""
    import subprocess

    exe = os.path.join(os.path.dirname(pkg.__file__), "host", "vpx_demo")
    n, w, h, frames, depth = 64, 80, 48, 2, 2
    out = tmp_path / "frame.rgb8"
    r = subprocess.run([exe, str(n), str(w), str(h), str(frames), str(depth), str(out), "sk"], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    rgb_cpp = np.fromfile(out, np.uint32)
    sc = pkg.scene
    desc = sc.with_sky(sc.pillars_scene(n, w, h, depth), texture=demo_sky(), hdr_contribution=1.5)
    o = orc.Oracle(pkg.abi, desc)
    prev = sc.prev_camera(desc._cam_pos, desc._cam_target, w, h)
    hist = np.zeros((w * h, 4), np.float32)
    for f in range(frames):
        rgb, _ = o.render_reproject(desc.frame_params(f), prev, hist)
    assert np.array_equal(rgb_cpp, rgb)


def _render_on(pkg, r, desc, frames=1):
    r.ResetAccumulator()
    for _ in range(frames):
        r.Tick(0.0)
    torch.cuda.synchronize()
    return r.accumulator_host().reshape(-1, 4).copy(), r.screen_host().reshape(-1).copy()


def test_world_edits_partial_model_and_sphere(pkg, orc):
    """ResetGrid + dirty-box upload of a LoadModelPartial slice, then
    CreateEmmisiveSphere — device grid and frames equal the oracle on the edited world."""
    sc = pkg.scene
    n = 64
    desc = sc.model_scene("monu3", n, 64, 40, 1, city_lights=True)
    r = pkg.renderer.Renderer(desc, 0)
    r.Init()
    size, vox, _ = sc.load_model("monu3")
    grid, box = sc.load_model_partial(size, vox, n, 30, 6)
    assert box is not None
    x0, y0, z0, x1, y1, z1 = box
    r.ctx.grid_fill(0, 255)
    r.ctx.grid_write_box(0, grid.reshape(n, n, n)[z0:z1, y0:y1, x0:x1], (x0, y0, z0))
    lib = orc._lib(pkg.abi)
    assert r.ctx.grid_checksum(0) == lib.oracle_grid_checksum(grid.ctypes.data, grid.size)
    acc_g, rgb_g = _render_on(pkg, r, desc)
    acc_o, rgb_o, _ = orc.Oracle(pkg.abi, desc, grid_cells=[grid]).render(desc.frame_params(0))
    assert np.array_equal(bits(acc_g), bits(acc_o)) and np.array_equal(rgb_g, rgb_o)
    # emissive sphere on top of the slice
    r.ctx.grid_emissive_sphere(0, 15, 9.5)
    lib.oracle_emissive_sphere(grid.ctypes.data, n, 15, 9.5)
    assert r.ctx.grid_checksum(0) == lib.oracle_grid_checksum(grid.ctypes.data, grid.size)
    acc_g, rgb_g = _render_on(pkg, r, desc)
    acc_o, rgb_o, _ = orc.Oracle(pkg.abi, desc, grid_cells=[grid]).render(desc.frame_params(0))
    assert np.array_equal(bits(acc_g), bits(acc_o)) and np.array_equal(rgb_g, rgb_o)
    # ResetGrid to a material
    r.ctx.grid_fill(0, 3)
    g3 = np.full(n ** 3, 3, np.uint8)
    assert r.ctx.grid_checksum(0) == lib.oracle_grid_checksum(g3.ctypes.data, g3.size)
    r.ctx.close()


def test_world_edits_random_boxes_odd_size(pkg, orc):
    """Dirty-box uploads at a grid size that is not a multiple of 4 or 16: the region
    rebuild of the occupancy levels must match a full rebuild (checked through frames)."""
    sc = pkg.scene
    n = 100
    desc = sc.model_scene("monu3", n, 48, 32, 2, cam=((0.5, 0.5, -0.4), (0.5, 0.5, 0.5)), city_lights=True)
    r = pkg.renderer.Renderer(desc, 0)
    r.Init()
    grid = desc.grids[0].dense.copy().reshape(n, n, n)
    rng = np.random.default_rng(5)
    for it in range(6):
        d = rng.integers(1, 40, 3)
        o = [int(rng.integers(0, n - k + 1)) for k in d]
        blk = rng.choice(np.array([255, 255, 255, 0, 5, 8, 20], np.uint8), size=(d[2], d[1], d[0]))
        grid[o[2]:o[2] + d[2], o[1]:o[1] + d[1], o[0]:o[0] + d[0]] = blk
        r.ctx.grid_write_box(0, blk, (o[0], o[1], o[2]))
    flat = np.ascontiguousarray(grid.reshape(-1))
    lib = orc._lib(pkg.abi)
    assert r.ctx.grid_checksum(0) == lib.oracle_grid_checksum(flat.ctypes.data, flat.size)
    acc_g, rgb_g = _render_on(pkg, r, desc)
    acc_o, rgb_o, _ = orc.Oracle(pkg.abi, desc, grid_cells=[flat]).render(desc.frame_params(0))
    assert np.array_equal(bits(acc_g), bits(acc_o)) and np.array_equal(rgb_g, rgb_o)
    r.ctx.close()


@pytest.mark.parametrize("name,depth", [("monu3", 2), ("roomGlass", 4), ("teapot", 3), ("roomGlass", 13),
                                        ("roomGlass", 14)])
def test_static_camera_reprojection(pkg, orc, name, depth):
    """Renderer::Tick's static branch — TraceReproject, reprojection
    into the previous camera, history clamp/blend — 3 frames with the camera nudged after
    the first (prevCamera stays), RGB8 and the illumination history bit-exact."""
    sc = pkg.scene
    desc = sc.model_scene(name, 64, 56, 40, depth, city_lights=True)
    r = pkg.renderer.Renderer(desc, 0)
    r.Init()
    r.staticCamera = True
    o = orc.Oracle(pkg.abi, desc)
    hist_o = np.zeros((desc.width * desc.height, 4), np.float32)
    prev = sc.prev_camera(desc._cam_pos, desc._cam_target, desc.width, desc.height)
    for f in range(3):
        if f > 0:  # move the live camera (sub-pixel, then off-screen edges); the reference keeps prevCamera from Init
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


# ---------------------------------------------------------------- sky dome (§8(f) rank 4)
@pytest.mark.parametrize("depth", [0, 4])
def test_trace_rays_sky_texture(pkg, orc, depth):
    """Trace with activateSky: every miss samples the (synthetic) HDR texture — random
    rays through the glass room (refraction / reflection chains that leave the grid) and
    rays that miss from the start."""
    from test_sky import miss_rays

    sc = pkg.scene
    desc = sc.with_sky(SCENES["room128_d4"](sc), hdr_contribution=1.3)
    ctx = make_ctx(pkg, desc)
    o = orc.Oracle(pkg.abi, desc)
    org, dirs = random_rays(2048, 23 + depth)
    mo, md = miss_rays(512, depth)
    org, dirs = np.concatenate([org, mo]), np.concatenate([dirs, md])
    rays = pkg.context.make_rays(org, dirs, inside=(np.arange(len(org)) % 5 == 0).astype(np.uint32))
    seeds = np.random.default_rng(depth).integers(1, 2**32 - 1, len(org), dtype=np.uint64).astype(np.uint32)
    rg = ctx.trace(rays, seeds, depth, None, desc.area_samples)
    ro, _ = o.trace(rays, seeds, depth, None, desc.area_samples)
    assert np.array_equal(bits(rg), bits(ro))
    ctx.close()


@pytest.mark.parametrize("name", ["teapot128", "room128_d4", "cityglass128_d4"])
def test_render_frame_sky_texture(pkg, orc, name):
    sc = pkg.scene
    desc = sc.with_sky(SCENES[name](sc), hdr_contribution=0.8)
    acc_g, rgb_g, st = render_gpu(pkg, desc)
    o = orc.Oracle(pkg.abi, desc)
    acc_o, rgb_o, ost = o.render(desc.frame_params(0))
    assert np.array_equal(bits(acc_g), bits(acc_o))
    assert np.array_equal(rgb_g, rgb_o)
    assert (st[0].shadow_rays, st[0].dda_cells) == (ost.shadow_rays, ost.dda_cells)


def test_static_camera_reprojection_sky_texture(pkg, orc):
    """SampleSkyReproject (renderer.cpp:2328-2346) on the static-camera path."""
    sc = pkg.scene
    desc = sc.with_sky(sc.model_scene("roomGlass", 64, 48, 32, 2, city_lights=True))
    r = pkg.renderer.Renderer(desc, 0)
    r.Init()
    r.staticCamera = True
    o = orc.Oracle(pkg.abi, desc)
    hist_o = np.zeros((desc.width * desc.height, 4), np.float32)
    prev = sc.prev_camera(desc._cam_pos, desc._cam_target, desc.width, desc.height)
    for f in range(2):
        r.Tick(0.0)
        torch.cuda.synchronize()
        rgb_o, _ = o.render_reproject(desc.frame_params(f), prev, hist_o)
        assert np.array_equal(bits(r.history_host().reshape(-1, 4)), bits(hist_o)), f"frame {f}: history"
        assert np.array_equal(r.screen_host().reshape(-1), rgb_o), f"frame {f}: rgb8"
    r.ctx.close()


def test_sky_flag_without_texture_is_refused(pkg):
    desc = SCENES["teapot128"](pkg.scene)
    desc.flags |= pkg.abi.VPX_FLAG_SKY
    ctx = make_ctx(pkg, desc)
    acc = torch.zeros(desc.width * desc.height * 4, dtype=torch.float32, device="cuda")
    with pytest.raises(pkg.abi.VpxError):
        ctx.render(desc.frame_params(0), acc.data_ptr())
    ctx.close()


def test_frame_beyond_path_index_range_is_refused(pkg):
    """The shadow lists hold a path index in 27 bits: frames of more than 2^27 tile-padded
    pixels are refused before any launch (16384x8192 is exactly 2^27, 16384x8208 one tile row
    more)."""
    desc = SCENES["teapot128"](pkg.scene)
    ctx = make_ctx(pkg, desc)
    acc = torch.zeros(4, dtype=torch.float32, device="cuda")  # never written: refused before launch
    with pytest.raises(pkg.abi.VpxError, match="2\\^27"):
        ctx.render(desc.with_size(16384, 8208).frame_params(0), acc.data_ptr())
    ctx.close()


@pytest.mark.parametrize("lanes", [2, 3])
@pytest.mark.parametrize("depth", [0, 2])
def test_frames_in_flight_equal_serial_frames(pkg, lanes, depth):
    """vpx_set_pipeline: frames rendered on `lanes` library streams with only their
    accumulate / tonemap on the context's stream give the serial frames' accumulator and
    screen bit for bit (AA jitter, 5 frames, point + area lights at depth 2), counters
    included; a world edit between frames is seen by exactly the frames after it."""
    sc = pkg.scene
    desc = sc.city_scene("monu3", 128, 96, 80, depth, areas=sc.C3_AREAS[:1] if depth else ())
    desc.flags = pkg.abi.VPX_FLAG_AA
    W, H = desc.width, desc.height
    box = np.full((6, 6, 6), 1, np.uint8)  # NON_METAL_RED cells

    def run(pipe, edit=True):
        ctx = pkg.context.Context(0)
        s = torch.cuda.Stream()
        ctx.set_stream(s.cuda_stream)
        ctx.load_scene(desc)
        ctx.set_pipeline(pipe)
        acc = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
        rgb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        ctx.counters(reset=True)
        shots = []
        with torch.cuda.stream(s):
            for f in range(5):
                if f == 3 and edit:  # a prop edit (LoadModelPartial) between frames
                    rc = ctx.lib.vpx_grid_write_box(ctx.h, 0, box.ctypes.data_as(C.c_void_p), 60, 40, 60, 6, 6, 6)
                    assert rc == 0, ctx.lib.vpx_last_error(ctx.h)
                ctx.render(desc.frame_params(f), acc.data_ptr(), rgb.data_ptr())
                shots.append(rgb.clone())
        ctx.synchronize()
        st = ctx.counters()
        out = (bits(acc.cpu().numpy().reshape(-1, 4)), [x.cpu().numpy() for x in shots], st)
        ctx.close()
        return out

    a0, s0, t0 = run(0)
    a1, s1, t1 = run(lanes)
    assert np.array_equal(a0, a1)
    for x, y in zip(s0, s1):
        assert np.array_equal(x, y)
    # the edit has an effect: without it frames 0-2 are the same and frames 3-4 differ
    _, s2, _ = run(0, edit=False)
    for f in range(3):
        assert np.array_equal(s0[f], s2[f])
    for f in (3, 4):
        assert not np.array_equal(s0[f], s2[f]), f"frame {f}: the world edit changed nothing"
    assert (t0.primary_rays, t0.shadow_rays, t0.bounce_rays, t0.dda_cells) == (
        t1.primary_rays, t1.shadow_rays, t1.bounce_rays, t1.dda_cells)


@pytest.mark.parametrize("lanes", [2, 4])
def test_frames_in_flight_sharded_accumulator(pkg, lanes):
    """vpx_render_tiles_accum with lanes: a rank's packed running average and RGB8 over 4
    frames equal the serial calls' bit for bit (2 ranks on one device)."""
    sc = pkg.scene
    desc = sc.city_scene("monu3", 128, 100, 70, 1)
    desc.flags = pkg.abi.VPX_FLAG_AA
    W, H, R = desc.width, desc.height, 2

    def run(pipe):
        ctx = pkg.context.Context(0)
        s = torch.cuda.Stream()
        ctx.set_stream(s.cuda_stream)
        ctx.load_scene(desc)
        ctx.set_pipeline(pipe)
        L = ctx.packed_len(W, H, R)
        accs = [torch.zeros(L * 4, dtype=torch.float32, device="cuda") for _ in range(R)]
        rgbs = [torch.zeros(L, dtype=torch.int32, device="cuda") for _ in range(R)]
        torch.cuda.synchronize()
        for f in range(4):
            for r in range(R):
                ctx.render_tiles_accum(desc.frame_params(f), r, R, accs[r].data_ptr(), rgbs[r].data_ptr())
        ctx.synchronize()
        out = [bits(a.cpu().numpy()) for a in accs] + [g.cpu().numpy() for g in rgbs]
        ctx.close()
        return out

    for x, y in zip(run(0), run(lanes)):
        assert np.array_equal(x, y)


def test_frames_in_flight_on_a_device_set(pkg):
    """A device set ({0, 0}) with 3 lanes per member: the sharded-accumulator frames
    (accum = NULL, RGB8 gathered) and the sample frames (accum given) equal one device's
    serial frames over 4 AA frames at depth 1."""
    sc = pkg.scene
    desc = sc.city_scene("monu3", 128, 100, 70, 1)
    desc.flags = pkg.abi.VPX_FLAG_AA
    acc_ref, rgb_ref, _ = render_gpu(pkg, desc, frames=4)
    W, H = desc.width, desc.height
    torch.cuda.set_device(0)
    ctx = pkg.context.Context(devices=[0, 0])
    ctx.load_scene(desc)
    ctx.set_pipeline(3)
    acc = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
    rgb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    rgb2 = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    for f in range(4):
        ctx.render(desc.frame_params(f), acc.data_ptr(), rgb.data_ptr())
    ctx.synchronize()
    for f in range(4):
        ctx.render(desc.frame_params(f), 0, rgb2.data_ptr())
    ctx.synchronize()
    assert np.array_equal(bits(acc.cpu().numpy().reshape(-1, 4)), bits(acc_ref))
    assert np.array_equal(rgb.cpu().numpy().view(np.uint32), rgb_ref)
    assert np.array_equal(rgb2.cpu().numpy().view(np.uint32), rgb_ref)
    ctx.close()
