"""Regenerate the decoded-model fixtures in tests/golden/ (run in the survey container).

The fixtures are the OUTPUT of the reference's own vendored .vox decoder, ogt_vox v0.997
(`/root/reference/lib/ogt_vox.h`), compiled where it lies by `oracle/Makefile` into
`oracle/_ref/ogt_ref_dump`.  Each `<model>.npz` holds exactly what `Scene::LoadModel`
receives (template/scene.cpp:474-475): `size` = (size_x, size_y, size_z), `voxels` =
voxel_data (palette index, x + y*sx + z*sx*sy, 0 = empty) and `palette` = 256 x RGBA.

Usage:  make -C oracle && python tests/golden/make_golden.py [/root/reference]
"""
import os
import struct
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
MODELS = ("teapot", "monu3", "roomGlass", "monu1", "monu2", "room", "player", "SmallBuilding01",
          "SmallBuilding02", "TallBuilding01", "Text", "textWin")  # every .vox in the reference's assets/


def dump(tool, vox_path):
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "m.bin")
        subprocess.run([tool, vox_path, out], check=True)
        raw = open(out, "rb").read()
    assert raw[:4] == b"VPXM"
    sx, sy, sz = struct.unpack_from("<3I", raw, 4)
    pal = np.frombuffer(raw, np.uint8, 1024, 16).reshape(256, 4)
    vox = np.frombuffer(raw, np.uint8, sx * sy * sz, 16 + 1024)
    return np.array([sx, sy, sz], np.uint32), vox.copy(), pal.copy()


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    tool = os.path.join(REPO, "oracle", "_ref", "ogt_ref_dump")
    if not os.path.exists(tool):
        sys.exit("build oracle/_ref/ogt_ref_dump first: make -C oracle")
    for name in MODELS:
        size, vox, pal = dump(tool, os.path.join(ref, "assets", name + ".vox"))
        np.savez_compressed(os.path.join(HERE, name + ".npz"), size=size, voxels=vox, palette=pal)
        hist = {int(k): int(v) for k, v in zip(*np.unique(vox[vox > 0], return_counts=True))}
        print(name, size.tolist(), hist)


if __name__ == "__main__":
    main()
