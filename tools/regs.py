"""Per-kernel register / spill / occupancy table from hipcc -Rpass-analysis=kernel-resource-usage.

  python tools/regs.py [extra hipcc flags...]     (compiles csrc/vpx_kernels.hip device-only)
"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "raytracer-voxpopuli_amd", "csrc", "vpx_kernels.hip")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-fgpu-flush-denormals-to-zero", "--cuda-device-only", "-c", "-o", "/tmp/regs_k.o"]


def main():
    out = subprocess.run(["hipcc", *FLAGS, *sys.argv[1:], SRC, "-Rpass-analysis=kernel-resource-usage"],
                         capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: (?:.*?: )?([A-Za-z ]+(?:\[[^\]]*\])?): (.*?) \[-Rpass", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2).strip()
        if k == "Function Name":
            cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    print(f"{'VGPR':>5} {'vSpl':>5} {'sSpl':>5} {'scr':>5} {'occ':>4}  kernel")
    for r in rows:
        n = re.sub(r"\(.*", "", r["name"].replace("(anonymous namespace)::", "")).replace("vpx::", "")
        print(f"{r.get('VGPRs', '?'):>5} {r.get('VGPRs Spill', '?'):>5} {r.get('SGPRs Spill', '?'):>5} "
              f"{r.get('ScratchSize [bytes/lane]', '?'):>5} {r.get('Occupancy [waves/SIMD]', '?'):>4}  {n}")


if __name__ == "__main__":
    main()
