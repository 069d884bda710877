"""Round-5 GPU parity: world updates between frames that the instance kernels' culls depend on.

The shadow pool lists only the slots whose segment meets the instance TLAS's root box, and
the instance walks cull by the TLAS and the volumes' world boxes, so d_volumes, d_vbounds and
the TLAS must change together (vpx_set_volumes rebuilds all three).  Here the instances move between two
accumulated frames (their transforms permuted, so every index gets another place) and the
accumulator, screen and counts must still equal the oracle's, which has no culls at all.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from cases import bits  # noqa: E402


@pytest.mark.parametrize("depth", [0, 1])
@pytest.mark.parametrize("lanes", [0, 3])
def test_instances_moved_between_frames(pkg, orc, depth, lanes):
    sc, abi = pkg.scene, pkg.abi
    desc = sc.instanced_scene(n=128, inst_n=32, width=96, height=64, spp=2)
    desc.max_bounces = depth
    desc.flags |= abi.VPX_FLAG_AA
    vols0 = desc.volumes
    moved = [vols0[0]] + [vols0[i] for i in range(len(vols0) - 1, 0, -1)]  # instances permuted
    moved[1] = sc.volume((0.1, 0.45, 0.2), (0.3, 0.3, 0.3), (0.0, 0.7, 0.0), grid_id=1)  # one brought low
    vols1 = (abi.Volume * len(moved))(*moved)

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
        ctx.render(desc.frame_params(0), acc.data_ptr(), rgb.data_ptr())
        ctx._chk(ctx.lib.vpx_set_volumes(ctx.h, vols1, len(moved)), "vpx_set_volumes")
        ctx.render(desc.frame_params(1), acc.data_ptr(), rgb.data_ptr())
    ctx.synchronize()
    st = ctx.counters()
    acc_g, rgb_g = bits(acc.cpu().numpy().reshape(-1, 4)), rgb.cpu().numpy().view(np.uint32)
    ctx.close()

    o = orc.Oracle(abi, desc)
    a, _, s0 = o.render(desc.frame_params(0))
    o.s.volumes, o.s.num_volumes = vols1, len(moved)
    o._keep.append(vols1)
    a, r, s1 = o.render(desc.frame_params(1), accum=a)
    assert np.array_equal(acc_g, bits(a)) and np.array_equal(rgb_g, r.view(np.uint32))
    tot = tuple(int(getattr(s0, k)) + int(getattr(s1, k)) for k in ("shadow_rays", "bounce_rays", "dda_cells"))
    assert (int(st.shadow_rays), int(st.bounce_rays), int(st.dda_cells)) == tot
    assert int(s1.dda_cells) != int(s0.dda_cells)  # the move changed the walks
