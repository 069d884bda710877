"""CPU suite: the exact empty-space-skipping math (csrc/vpx_skip.hpp, shared verbatim by the
device walker) against plain IEEE accumulation and the cell-by-cell reference march
(template/scene.cpp:751-811, restated).  Builds tests/native/*.cpp with g++."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "raytracer-voxpopuli_amd", "csrc")


@pytest.mark.parametrize("name,expect", [("skip_math_test", ["udiv bad=0", "ceil/floor div bad=0", "bad=0"]),
                                         ("skip_walk_test", ["bad=0"])])
def test_native_skip(tmp_path, name, expect):
    exe = tmp_path / name
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", CSRC,
                    os.path.join(HERE, "native", f"{name}.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    for e in expect:
        assert e in r.stdout, r.stdout
    if name == "skip_math_test":
        assert "skip_box_lean:" in r.stdout and ", bad=0" in r.stdout.split("skip_box_lean:")[1]
