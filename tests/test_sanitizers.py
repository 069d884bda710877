"""Sanitizer runs (ASan/UBSan on the CPU restatement and the host code).

- oracle: `make -C oracle sanitize` builds oracle/selftest.c + vpx_oracle.c with
  -fsanitize=address,undefined,float-cast-overflow -fno-sanitize-recover=all and runs every
  entry of the restatement over a small world (frames at depths -1/0/3/14 with AA, DOF and
  the sky, the static-camera path, per-ray entries with axis-parallel rays, BasicBVH, the
  world edits); any report aborts.
- host mirror: host/vpx_demo_asan (ASan + UBSan on the C++ host code only, -Xarch_host) runs
  the failure path here (no GPU: vpx_create must fail cleanly) and a full 3-frame run on
  the GPU box (tests/test_gpu_parity.py::test_cpp_host_demo_asan).
"""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oracle_under_asan_ubsan():
    r = subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "sanitize"], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "0 failure(s)" in r.stdout


def test_host_mirror_asan_fails_cleanly_without_gpu(pkg):
    import torch

    if torch.cuda.is_available():
        return  # the GPU run is test_gpu_parity.py::test_cpp_host_demo_asan
    exe = os.path.join(os.path.dirname(pkg.__file__), "host", "vpx_demo_asan")
    assert os.path.exists(exe), "build host/vpx_demo_asan (__graft_entry__.build())"
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe, "32", "16", "16", "1", "0"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 1 and "vpx_create failed" in r.stderr, r.stderr[-2000:]
    assert "Sanitizer" not in r.stderr
