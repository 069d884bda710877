"""The C-ABI library loads without a GPU and exports every symbol include/vpx.h declares."""
import ctypes as C
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(REPO, "include", "vpx.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(vpx_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_exported(pkg):
    lib = pkg.load_library()
    syms = declared_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(pkg.abi.SIGNATURES), set(syms) ^ set(pkg.abi.SIGNATURES)
    out = subprocess.run(["nm", "-D", "--defined-only", pkg.abi.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (vpx_\w+)", out))
    assert set(syms) <= exported


def test_library_is_gfx950_code_object(pkg):
    data = open(pkg.abi.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data  # embedded offload bundle target


def test_struct_layouts(pkg):
    for s, size in pkg.abi.STRUCT_SIZES.items():
        assert C.sizeof(s) == size, s


def test_abi_version_matches_header(pkg):
    text = open(os.path.join(REPO, "include", "vpx.h")).read()
    hdr = int(re.search(r"#define VPX_ABI_VERSION (\d+)", text).group(1))
    assert hdr == pkg.abi.ABI_VERSION == pkg.load_library().vpx_abi_version() == 2


@pytest.mark.parametrize("iv,want", [
    ([], 0.0),
    ([(0.0, 1.0)], 1.0),
    ([(0.0, 1.0), (0.5, 2.0)], 2.0),          # overlap counted once
    ([(0.0, 1.0), (3.0, 4.0)], 2.0),          # disjoint
    ([(-3.0, -1.0), (0.0, 1.0)], 3.0),        # a lane's launch before the first event (negative start)
    ([(-2.0, 0.5), (0.0, 1.0)], 3.0),
    ([(1.0, 2.0), (-5.0, -4.5), (1.5, 1.7)], 1.5),
])
def test_profile_busy_union(pkg, iv, want):
    """vpx_profile_read's busy time is the union of the launch intervals, also when a launch
    on another lane started before the first recorded event (the old sentinels
    clipped such intervals to [0, hi])."""
    lib = pkg.load_library()
    flat = (C.c_float * max(1, 2 * len(iv)))(*[x for ab in iv for x in ab])
    assert abs(lib.vpx_profile_busy_union(flat, len(iv)) - want) < 1e-6


def test_create_without_gpu_fails_cleanly(pkg):
    torch = pytest.importorskip("torch")
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is present")
    lib = pkg.load_library()
    h = C.c_void_p()
    assert lib.vpx_create(0, C.byref(h)) == -2  # VPX_E_DEVICE, no abort
    assert lib.vpx_destroy(None) == -1


def test_host_helpers_reject_bad_arguments(pkg):
    lib = pkg.load_library()
    assert lib.vpx_camera_look_at(None, None, 0, 0, None) == -1
    assert lib.vpx_default_materials(None) == -1
    assert lib.vpx_tiles_packed_len(0, 10, 16, 16, 1) == 0
    assert lib.vpx_tiles_packed_len(33, 17, 16, 16, 2) == 3 * 256  # 6 tiles over 2 ranks


def test_cpp_host_mirror_links_and_fails_cleanly_without_gpu(pkg):
    """host/vpx_demo (the C++ Renderer mirror) is built, links libvpx_hip.so, and reports a
    clean error (no abort) when no GPU is visible."""
    import os
    import subprocess

    torch = pytest.importorskip("torch")
    exe = os.path.join(os.path.dirname(pkg.__file__), "host", "vpx_demo")
    assert os.path.exists(exe), "run __graft_entry__.build()"
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is present (covered by test_gpu_parity)")
    r = subprocess.run([exe, "16", "8", "8", "1"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "no usable HIP device" in r.stderr
