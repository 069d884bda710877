"""Shared parity cases (scenes, ray sets) for the GPU and CPU test suites."""
import numpy as np


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def random_rays(n, seed, inside_frac=0.3, axis_frac=0.1):
    rng = np.random.default_rng(seed)
    o = rng.uniform(-0.6, 1.6, (n, 3)).astype(np.float32)
    k = int(n * inside_frac)
    o[:k] = rng.uniform(0.0, 1.0, (k, 3)).astype(np.float32)
    target = rng.uniform(0.1, 0.9, (n, 3)).astype(np.float32)
    d = (target - o).astype(np.float32)
    d[k:2 * k] = rng.normal(size=(k, 3)).astype(np.float32)
    a = int(n * axis_frac)
    if a:  # axis-aligned and zero-component directions (rD = +-inf)
        axes = rng.integers(0, 3, a)
        d[-a:] = 0
        d[-a:][np.arange(a), axes] = rng.choice([-1.0, 1.0], a)
    return o, d


SCENES = {
    "teapot128": lambda sc: sc.model_scene("teapot", 128, 96, 64, 0),
    "monu3_128": lambda sc: sc.model_scene("monu3", 128, 96, 64, 0),
    "room128_d4": lambda sc: sc.model_scene("roomGlass", 128, 96, 64, 4, city_lights=True),
    "city128_d0": lambda sc: sc.city_scene("monu3", 128, 96, 64, 0),
    "cityglass128_d4": lambda sc: sc.city_scene("roomGlass", 256, 96, 64, 4),
}


