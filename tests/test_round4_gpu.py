"""Round-4 GPU parity: bounce-level frames, the reference's own scene shape, frames in flight
that blend in their own tail launch, and the split multi-volume primary stage.

Every frame here is compared bit for bit with the oracle (accumulator floats, RGB8 bytes, ray
and DDA-cell counts): single-volume bounce frames over the paths' variety (point / area lights
with 1 and several slots per path, glass and smoke interiors, depths 1..14, AA, accumulated
frames); the zone scene (scene.zone_scene: Renderer::SetUpFirstZone's 21 volumes, 10
triangles, point + 5 spot + directional lights, depth 14, sky); frames in flight whose tail is
the shadow pool's k_resolve_finish (the lane blends into the accumulator itself); multi-volume
primary rays through the world walk + instance pass (k_instances).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from cases import bits  # noqa: E402


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
def test_bounce_frames_bit_exact(pkg, orc, name):
    desc = CASES[name](pkg.scene)
    desc.flags = pkg.abi.VPX_FLAG_AA
    frames = 2
    a_o, r_o, t_o = oracle_frames(orc, pkg, desc, frames)
    a_p, r_p, t_p = render(pkg, desc, frames)
    assert np.array_equal(a_p, a_o), "accumulator differs from the oracle"
    assert np.array_equal(r_p, r_o)
    assert counts(t_p) == (t_o["primary_rays"], t_o["shadow_rays"], t_o["bounce_rays"], t_o["dda_cells"])
    assert t_p.bounce_rays > 0 and (t_p.shadow_rays > 0 or name.startswith("teapot"))  # the teapot is glass: no light samples


def test_smoke_and_glass_interiors(pkg, orc):
    """A world of a glass slab and a smoke ball (the interior exit marches of the shade: the
    glass and smoke branches' FindMaterialExit / FindSmokeExit, renderer.cpp:1146-1314) at
    depth 6."""
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
    a_p, r_p, t_p = render(pkg, desc, 1)
    assert np.array_equal(a_p, a_o) and np.array_equal(r_p, r_o)
    assert counts(t_p) == (t_o["primary_rays"], t_o["shadow_rays"], t_o["bounce_rays"], t_o["dda_cells"])


@pytest.mark.parametrize("depth", [1, 14])
def test_zone_scene_bit_exact(pkg, orc, depth):
    """The reference's own scene shape (SetUpFirstZone: 21 volumes, 10 triangles, point + 5
    spot + directional lights, sky), 2 AA frames."""
    desc = pkg.scene.zone_scene(96, 64, depth)
    desc.flags |= pkg.abi.VPX_FLAG_AA
    a_o, r_o, t_o = oracle_frames(orc, pkg, desc, 2)
    a_g, r_g, t_g = render(pkg, desc, 2)
    assert np.array_equal(a_g, a_o) and np.array_equal(r_g, r_o)
    assert counts(t_g) == (t_o["primary_rays"], t_o["shadow_rays"], t_o["bounce_rays"], t_o["dda_cells"])
    assert t_g.bounce_rays > 0


@pytest.mark.parametrize("scene", ["areas-d0", "instances-areas-d0", "instances-areas-d2", "roomGlass-d14-areas"])
@pytest.mark.parametrize("lanes", [2, 4])
def test_lane_tail_frames_in_flight(pkg, orc, scene, lanes):
    """Frames in flight whose tail is its own launch (the shadow pool's k_resolve_finish:
    area lights with several samples) blend on their lane straight into the accumulator,
    ordered by the caller's stream (no packed sample, no composite): 4 AA frames equal the
    serial frames and the oracle (single volume at depth 0, and the instanced world, where the
    depth-2 frames go through the per-level kernels with the shadow pool's tail; and a depth-14
    area-light frame, whose deep levels end in k_tail + k_finish: that blend waits for the
    caller's stream too)."""
    sc = pkg.scene
    if scene == "areas-d0":
        desc = sc.city_scene("monu3", 128, 80, 64, 0, areas=sc.C3_AREAS)
    elif scene in CASES:  # depth 14: the deep levels run in k_tail, then k_finish blends on the lane
        desc = CASES[scene](sc)
    else:
        desc = sc.instanced_scene(n=128, inst_n=32, width=80, height=64, spp=1)
        desc.max_bounces = 2 if scene.endswith("d2") else 0
    desc.flags = pkg.abi.VPX_FLAG_AA
    a_s, r_s, t_s = render(pkg, desc, 4, lanes=0)
    a_l, r_l, t_l = render(pkg, desc, 4, lanes=lanes)
    assert np.array_equal(a_l, a_s) and np.array_equal(r_l, r_s) and counts(t_l) == counts(t_s)
    a_o, r_o, t_o = oracle_frames(orc, pkg, desc, 4)
    assert np.array_equal(a_s, a_o) and np.array_equal(r_s, r_o)
    assert counts(t_s) == (t_o["primary_rays"], t_o["shadow_rays"], t_o["bounce_rays"], t_o["dda_cells"])


@pytest.mark.parametrize("scene", ["roomGlass-d4-points", "monu3-d3-areas"])
def test_level_fork_frames_bit_exact(pkg, orc, scene):
    """The level fork (a level's bounce walks on a second stream beside its shadow walks,
    joined before the next shade): frames on the context's stream (fork), 2 lanes (fork on
    each lane, single-volume scenes) and 3 lanes (no fork) equal each other and the oracle,
    with the tile shadow kernels (point lights) and the shadow pool (area lights)."""
    desc = CASES[scene](pkg.scene)
    desc.flags = pkg.abi.VPX_FLAG_AA
    frames = 3
    a_o, r_o, t_o = oracle_frames(orc, pkg, desc, frames)
    for lanes in (0, 2, 3):
        a_p, r_p, t_p = render(pkg, desc, frames, lanes=lanes)
        assert np.array_equal(a_p, a_o), f"{lanes} lanes: accumulator differs from the oracle"
        assert np.array_equal(r_p, r_o), f"{lanes} lanes: RGB8 differs"
        assert counts(t_p) == (t_o["primary_rays"], t_o["shadow_rays"], t_o["bounce_rays"], t_o["dda_cells"])
