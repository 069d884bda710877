"""BasicBVH (src/BVH/BasicBVH.{h,cpp}): the library's host build and
triangle generator against the oracle restatement, and structural properties of the tree.

The traversal itself runs on the device (vpx_bvh_intersect); its bit-exact parity with
oracle_bvh_intersect is in test_gpu_parity.py.  Parity against the reference itself is
unpinned; the reference's own construction (64 random triangles) is
reproduced from its RandomFloat stream with the three draws of a float3 taken left to right.
"""
import ctypes as C

import numpy as np
import pytest


def lib_build(pkg, tris):
    abi, lib = pkg.abi, pkg.load_library()
    n = len(tris)
    nodes = (abi.BvhNode * max(1, 2 * n - 1))()
    idx = (C.c_uint32 * max(1, n))()
    used = C.c_uint32()
    assert lib.vpx_bvh_build_host(tris, n, nodes, idx, C.byref(used)) == 0
    return nodes, idx, used.value


def tri_array(abi, v):
    v = np.asarray(v, np.float32).reshape(-1, 9)
    arr = (abi.BvhTri * len(v))()
    np.frombuffer(arr, np.float32).reshape(-1, 9)[:] = v
    return arr


def tri_sets(abi, orc):
    ref, _ = orc.BasicBVH.random_tris(abi)
    rng = np.random.default_rng(5)
    sets = {"reference-ctor": ref}
    for n in (1, 2, 3, 5, 64, 200, 512):
        a = rng.uniform(-5, 4, (n, 3))
        sets[f"random{n}"] = tri_array(abi, np.concatenate([a, a + rng.uniform(0, 1, (n, 3)), a + rng.uniform(0, 1, (n, 3))], 1))
    same = np.tile(np.float32([0, 0, 0, 1, 0, 0, 0, 1, 0]), (9, 1))  # identical: every split aborts
    sets["identical9"] = tri_array(abi, same)
    line = np.array([[i, 0, 0, i + 0.5, 0, 0, i, 0.5, 0] for i in range(40)], np.float32)  # centroids on a line
    sets["line40"] = tri_array(abi, line)
    return sets


def test_random_tris_match_oracle(pkg, orc):
    abi, lib = pkg.abi, pkg.load_library()
    for seed in (0x12345678, 1, 0xdeadbeef):
        ref, after = orc.BasicBVH.random_tris(abi, seed)
        out = (abi.BvhTri * 64)()
        s = C.c_uint32(seed)
        assert lib.vpx_bvh_random_tris(C.byref(s), out) == 0
        assert bytes(out) == bytes(ref) and s.value == after
        v = np.frombuffer(out, np.float32).reshape(64, 3, 3)
        assert (v[:, 0] >= -5).all() and (v[:, 0] <= 4).all()  # r0 * 9 - 5, r0 in [0, 1)


def test_host_build_matches_oracle_and_is_a_valid_tree(pkg, orc):
    abi = pkg.abi
    for name, tris in tri_sets(abi, orc).items():
        n = len(tris)
        nodes, idx, used = lib_build(pkg, tris)
        o = orc.BasicBVH(abi, tris)
        assert used == o.used, name
        assert bytes(nodes)[: 32 * used] == bytes(o.nodes)[: 32 * used], name
        assert list(idx) == list(o.idx), name
        assert sorted(idx) == list(range(n)), name
        v = np.frombuffer(tris, np.float32).reshape(n, 3, 3)
        lo, hi = v.min(1), v.max(1)
        seen = []
        def walk(i, depth):
            nd = nodes[i]
            if nd.tri_count:
                ids = [idx[nd.left_first + k] for k in range(nd.tri_count)]
                seen.extend(ids)
                assert (lo[ids] >= np.float32(nd.aabb_min)).all() and (hi[ids] <= np.float32(nd.aabb_max)).all()
                return depth
            assert nd.left_first + 1 < used
            return max(walk(nd.left_first, depth + 1), walk(nd.left_first + 1, depth + 1))
        walk(0, 1)
        assert sorted(seen) == list(range(n)), name
        if name == "identical9":
            assert used == 1  # the split of identical centroids aborts (BasicBVH.cpp:123-124)


def test_depth_of_degenerate_chain(pkg, orc):
    """vpx_bvh_depth (what vpx_bvh_set checks against VPX_BVH_MAX_DEPTH): centroids at
    x = 2^i make every midpoint split peel off one triangle, a chain as deep as the set."""
    abi, lib = pkg.abi, pkg.load_library()
    for n, want in ((80, 79), (40, 39), (2, 1), (1, 1)):  # leaves hold <= 2 triangles
        v = np.zeros((n, 9), np.float32)
        x = np.float32(2.0) ** np.arange(n, dtype=np.float32)
        v[:, 0], v[:, 3], v[:, 6] = x, x, x
        v[:, 4], v[:, 8] = 1.0, 1.0
        nodes, idx, used = lib_build(pkg, tri_array(abi, v))
        o = orc.BasicBVH(abi, tri_array(abi, v))
        assert used == o.used and bytes(nodes)[: 32 * used] == bytes(o.nodes)[: 32 * used]
        assert lib.vpx_bvh_depth(nodes, used) == want, n
    assert lib.vpx_bvh_depth(nodes, 0) == 0
    nodes, idx, used = lib_build(pkg, orc.BasicBVH.random_tris(abi)[0])
    assert 1 < lib.vpx_bvh_depth(nodes, used) <= abi.BVH_MAX_DEPTH  # the reference's own set fits


def test_oracle_traversal_equals_a_linear_loop(pkg, orc):
    """Sanity of the restatement: the BVH's nearest t is the nearest over all triangles
    (up to rays whose hit lies on a box face within float rounding)."""
    abi = pkg.abi
    tris, _ = orc.BasicBVH.random_tris(abi)
    o = orc.BasicBVH(abi, tris)
    rng = np.random.default_rng(2)
    org = rng.uniform(-8, 8, (4000, 3)).astype(np.float32)
    cen = np.frombuffer(tris, np.float32).reshape(64, 3, 3).mean(1)
    tgt = (cen[rng.integers(0, 64, 4000)] + rng.normal(0, 0.05, (4000, 3))).astype(np.float32)
    rays = pkg.context.make_rays(org, tgt - org)
    t_bvh = o.intersect(rays)
    flat = orc.BasicBVH(abi, tris)
    flat.nodes[0].tri_count, flat.nodes[0].left_first = 64, 0  # one leaf holding everything = the linear loop
    for k in range(64):
        flat.idx[k] = k
    t_lin = flat.intersect(rays)
    assert (t_bvh < 1e33).mean() > 0.3
    assert (t_bvh == t_lin).mean() > 0.999
