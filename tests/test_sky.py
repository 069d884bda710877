"""Sky dome: SampleSky with a texture (renderer.cpp:2308-2326).

The reference's HDR (assets/sky_19.hdr) is missing from its tree, so the
texture is the build's synthetic equirectangular image (scene.synthetic_sky).  CPU:
the oracle's SampleSky (reached through Trace on rays that miss every volume) against an
independent numpy-float32 restatement of atan2_approximation2 / FastAcos
(template/tmpl8math.cpp:405-443) and the index arithmetic.  Parity of the sky functions
with the reference itself is unpinned (no reference output exists for them).
"""
import numpy as np

from cases import bits

F = np.float32
PI_F = F(3.14159265358979323846264)


def atan2_approx(y, x):
    q1 = F(np.float64(PI_F) / 4.0)
    q3 = F(3.0 * np.float64(PI_F) / 4.0)
    ay = np.abs(y) + F(1e-10)
    with np.errstate(all="ignore"):
        rn = (x + ay) / (ay - x)
        rp = (x - ay) / (x + ay)
    neg = x < 0
    r = np.where(neg, rn, rp).astype(F)
    angle = np.where(neg, q3, q1).astype(F)
    angle = angle + (F(0.1963) * r * r - F(0.9817)) * r
    return np.where(y < 0, -angle, angle).astype(F)


def fast_acos(x):
    negate = (x < 0).astype(F)
    x = np.abs(x)
    ret = np.full_like(x, F(-0.0187293))
    ret = ret * x
    ret = ret + F(0.0742610)
    ret = ret * x
    ret = ret - F(0.2121144)
    ret = ret * x
    ret = ret + F(1.5707288)
    with np.errstate(invalid="ignore"):
        ret = ret * np.sqrt(F(1.0) - x)
    ret = ret - F(2) * negate * ret
    return (negate * F(3.14159265358979) + ret).astype(F)


def sample_sky_np(d, img, hdr):
    h, w, _ = img.shape
    uf = F(w) * atan2_approx(d[:, 2], d[:, 0]) * F(0.15915494309189533576888) - F(0.5)
    vf = F(h) * fast_acos(d[:, 1]) * F(0.31830988618379067153777) - F(0.5)
    u, v = np.trunc(uf).astype(np.int64), np.trunc(vf).astype(np.int64)
    idx = np.clip(np.maximum(0, u + v * w), 0, w * h - 1)
    return (F(hdr) * img.reshape(-1, 3)[idx]).astype(F)


def normalize_like_ray(d):
    """Ray(origin, direction) normalisation: d * (1 / sqrtf(dot(d, d))) (scene.cpp:83-93)."""
    d = d.astype(F)
    dd = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
    inv = F(1) / np.sqrt(dd)
    return (d * inv[:, None]).astype(F)


def miss_rays(n, seed):
    """Rays from outside the unit cube pointing away from it (they miss every volume)."""
    rng = np.random.default_rng(seed)
    d = rng.normal(size=(n, 3)).astype(F)
    axes = np.array([[0, 1, 0], [0, -1, 0], [1, 0, 0], [-1, 0, 0], [0, 0, 1], [0, 0, -1], [1, 1, 0], [-1, 0, -1e-7],
                     [-1, 0, 1e-7], [-1, 0, 0.0], [1e-30, 1, 0]], F)
    d[: len(axes)] = axes
    d = normalize_like_ray(d)
    o = (F(0.5) + F(4.0) * d).astype(F)  # 3.5 units out along the direction
    return o, d


def test_sky_functions_known_answers():
    # D = (0, 1, 0): atan2(0, 0) = pi/4 - 0.9817 - ... (x >= 0 branch), FastAcos(1) = 0
    assert fast_acos(np.array([1.0], F))[0] == F(0.0)
    assert abs(float(fast_acos(np.array([-1.0], F))[0]) - np.pi) < 1e-6
    a = atan2_approx(np.array([0.0, 1.0, -1.0], F), np.array([1.0, 0.0, 0.0], F))
    assert abs(float(a[0])) < 1e-3 and abs(float(a[1]) - np.pi / 2) < 1e-2 and abs(float(a[2]) + np.pi / 2) < 1e-2


def test_oracle_sample_sky_matches_numpy(pkg, orc):
    sc = pkg.scene
    desc = sc.with_sky(sc.model_scene("teapot", 128, 32, 16, 0), hdr_contribution=1.7)
    o = orc.Oracle(pkg.abi, desc)
    org, d = miss_rays(4096, 5)
    rays = pkg.context.make_rays(org, d)
    seeds = np.arange(1, len(org) + 1, dtype=np.uint32)
    rad, st = o.trace(rays, seeds, 0, None)
    assert st.dda_cells == 0  # every ray missed the grid
    want = sample_sky_np(d, desc.sky_texture, 1.7)
    assert np.array_equal(bits(rad), bits(want))
    # the constant sky is unchanged when a colour is passed
    rad_c, _ = o.trace(rays, seeds, 0, pkg.abi.SKY_DEFAULT)
    assert np.array_equal(bits(rad_c), bits(np.broadcast_to(np.array(pkg.abi.SKY_DEFAULT, F), rad_c.shape)))


def test_oracle_render_with_sky_changes_only_misses(pkg, orc):
    sc = pkg.scene
    base = sc.model_scene("monu3", 128, 48, 32, 0, city_lights=True)
    sky = sc.with_sky(base)
    acc0, _, st0 = orc.Oracle(pkg.abi, base).render(base.frame_params(0))
    acc1, _, st1 = orc.Oracle(pkg.abi, sky).render(sky.frame_params(0))
    assert (st0.dda_cells, st0.shadow_rays) == (st1.dda_cells, st1.shadow_rays)
    const = np.all(acc0[:, :3] == np.array(pkg.abi.SKY_DEFAULT, F), axis=1)
    assert const.any() and not np.array_equal(acc0[const], acc1[const])
    assert np.array_equal(bits(acc0[~const]), bits(acc1[~const]))
