"""The path pool (k_path_pool, round 4) and the reference's own scene shape, on the GPU.

k_path_pool carries each path of a single-volume frame through its bounce levels in one
persistent launch.  Every frame here is compared bit for bit with the oracle
(accumulator floats, RGB8 bytes, ray and DDA-cell counts) and with the per-level kernels
(VPX_PATH_POOL=0 at context creation), over the paths' whole variety: point / area lights
(1 and several slots per path), glass and smoke interiors (roomGlass, the smoke ball),
depths 1..14 (the deepest forms word), AA, accumulated frames and frames in flight.

The zone scene (scene.zone_scene: Renderer::SetUpFirstZone's 21 volumes, 10 triangles, point
+ 5 spot + directional lights, depth 14, sky) runs the multi-volume path.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from cases import bits  # noqa: E402


def render(pkg, desc, frames, pool, lanes=0):
    old = os.environ.get("VPX_PATH_POOL")
    os.environ["VPX_PATH_POOL"] = "1" if pool else "0"
    try:
        ctx = pkg.context.Context(0)
    finally:
        if old is None:
            del os.environ["VPX_PATH_POOL"]
        else:
            os.environ["VPX_PATH_POOL"] = old
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
    out = (bits(acc.cpu().numpy().reshape(-1, 4)), rgb.cpu().numpy().view(np.uint32), st)
    ctx.close()
    return out


def oracle_frames(orc, pkg, desc, frames):
    o = orc.Oracle(pkg.abi, desc)
    acc, tot = None, None
    for f in range(frames):
        acc, rgb, st = o.render(desc.frame_params(f), accum=acc)
        d = st.as_dict()
        tot = d if tot is None else {k: tot[k] + d[k] for k in ("primary_rays", "shadow_rays", "bounce_rays", "dda_cells")}
    return bits(acc), rgb.view(np.uint32), tot


def counts(st):
    return tuple(int(getattr(st, k)) for k in ("primary_rays", "shadow_rays", "bounce_rays", "dda_cells"))


CASES = {
    "roomGlass-d1-points": lambda sc: sc.city_scene("roomGlass", 128, 80, 48, 1),
    "roomGlass-d4-points": lambda sc: sc.city_scene("roomGlass", 128, 80, 48, 4),
    "roomGlass-d14-areas": lambda sc: sc.city_scene("roomGlass", 128, 64, 40, 14, areas=sc.C3_AREAS[:2]),
    "monu3-d3-areas": lambda sc: sc.city_scene("monu3", 128, 72, 56, 3, areas=sc.C3_AREAS),
    "teapot-d13-points": lambda sc: sc.model_scene("teapot", 128, 64, 48, 13, city_lights=True),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_path_pool_bit_exact(pkg, orc, name):
    desc = CASES[name](pkg.scene)
    desc.flags = pkg.abi.VPX_FLAG_AA
    frames = 2
    a_o, r_o, t_o = oracle_frames(orc, pkg, desc, frames)
    a_p, r_p, t_p = render(pkg, desc, frames, pool=True)
    assert np.array_equal(a_p, a_o), "path pool accumulator differs from the oracle"
    assert np.array_equal(r_p, r_o)
    assert counts(t_p) == (t_o["primary_rays"], t_o["shadow_rays"], t_o["bounce_rays"], t_o["dda_cells"])
    a_l, r_l, t_l = render(pkg, desc, frames, pool=False)
    assert np.array_equal(a_l, a_p) and np.array_equal(r_l, r_p) and counts(t_l) == counts(t_p)
    assert t_p.bounce_rays > 0 and (t_p.shadow_rays > 0 or name.startswith("teapot"))  # the teapot is glass: no light samples


@pytest.mark.parametrize("lanes", [2, 3])
def test_path_pool_frames_in_flight(pkg, orc, lanes):
    """The pool in the packed-sample mode of frames in flight: 4 AA frames on `lanes` lanes
    equal the serial frames and the oracle."""
    sc = pkg.scene
    desc = sc.city_scene("roomGlass", 128, 96, 64, 4)
    desc.flags = pkg.abi.VPX_FLAG_AA
    a_o, r_o, t_o = oracle_frames(orc, pkg, desc, 4)
    a_p, r_p, t_p = render(pkg, desc, 4, pool=True, lanes=lanes)
    assert np.array_equal(a_p, a_o) and np.array_equal(r_p, r_o)
    assert counts(t_p) == (t_o["primary_rays"], t_o["shadow_rays"], t_o["bounce_rays"], t_o["dda_cells"])


def test_path_pool_smoke_and_glass_interiors(pkg, orc):
    """A world of a glass slab and a smoke ball (the interior exit marches of the shade: the
    glass and smoke branches' FindMaterialExit / FindSmokeExit, renderer.cpp:1146-1314) at
    depth 6 through the pool."""
    sc = pkg.scene
    n = 64
    z, y, x = np.meshgrid(*(np.arange(n),) * 3, indexing="ij")
    g = np.full((n, n, n), 255, np.uint8)
    g[y < 2] = 0
    g[(x > 8) & (x < 28) & (y > 4) & (y < 30) & (z > 20) & (z < 26)] = 8  # glass slab
    r = np.sqrt((x - 44.0) ** 2 + (y - 16.0) ** 2 + (z - 40.0) ** 2)
    g[r < 10] = 11  # smoke ball
    g[(x > 30) & (x < 34) & (y < 20)] = 6  # a metal pillar
    spec = sc.GridSpec(n=n, dense=g.reshape(-1))
    desc = sc._scene("glass-smoke64", [spec], [sc.volume()], sc.default_materials(), [sc.point_light((0.5, 1.5, 0.2))],
                     [], [], sc.dir_light((-0.3, -1.0, -0.2), (1.0, 1.0, 1.0)), (0.5, 0.5, -0.8), (0.5, 0.3, 0.5), 72, 56,
                     max_bounces=6)
    a_o, r_o, t_o = oracle_frames(orc, pkg, desc, 1)
    a_p, r_p, t_p = render(pkg, desc, 1, pool=True)
    assert np.array_equal(a_p, a_o) and np.array_equal(r_p, r_o)
    assert counts(t_p) == (t_o["primary_rays"], t_o["shadow_rays"], t_o["bounce_rays"], t_o["dda_cells"])


@pytest.mark.parametrize("depth", [1, 14])
def test_zone_scene_bit_exact(pkg, orc, depth):
    """The reference's own scene shape (SetUpFirstZone: 21 volumes, 10 triangles, point + 5
    spot + directional lights, sky), 2 AA frames."""
    desc = pkg.scene.zone_scene(96, 64, depth)
    desc.flags |= pkg.abi.VPX_FLAG_AA
    a_o, r_o, t_o = oracle_frames(orc, pkg, desc, 2)
    a_g, r_g, t_g = render(pkg, desc, 2, pool=True)
    assert np.array_equal(a_g, a_o) and np.array_equal(r_g, r_o)
    assert counts(t_g) == (t_o["primary_rays"], t_o["shadow_rays"], t_o["bounce_rays"], t_o["dda_cells"])
    assert t_g.bounce_rays > 0


@pytest.mark.parametrize("scene", ["areas-d0", "instances-areas-d0", "instances-areas-d2"])
@pytest.mark.parametrize("lanes", [2, 4])
def test_lane_tail_frames_in_flight(pkg, orc, scene, lanes):
    """Frames in flight whose tail is its own launch (the shadow pool's k_resolve_finish:
    area lights with several samples) blend on their lane straight into the accumulator,
    ordered by the caller's stream (no packed sample, no composite): 4 AA frames equal the
    serial frames and the oracle (single volume at depth 0, and the instanced world, where the
    depth-2 frames go through the per-level kernels with the shadow pool's tail)."""
    sc = pkg.scene
    if scene == "areas-d0":
        desc = sc.city_scene("monu3", 128, 80, 64, 0, areas=sc.C3_AREAS)
    else:
        desc = sc.instanced_scene(n=128, inst_n=32, width=80, height=64, spp=1)
        desc.max_bounces = 2 if scene.endswith("d2") else 0
    desc.flags = pkg.abi.VPX_FLAG_AA
    a_s, r_s, t_s = render(pkg, desc, 4, pool=True, lanes=0)
    a_l, r_l, t_l = render(pkg, desc, 4, pool=True, lanes=lanes)
    assert np.array_equal(a_l, a_s) and np.array_equal(r_l, r_s) and counts(t_l) == counts(t_s)
    a_o, r_o, t_o = oracle_frames(orc, pkg, desc, 4)
    assert np.array_equal(a_s, a_o) and np.array_equal(r_s, r_o)
    assert counts(t_s) == (t_o["primary_rays"], t_o["shadow_rays"], t_o["bounce_rays"], t_o["dda_cells"])
