"""Per-kernel HBM traffic per launch from rocprofv3 --pmc passes (tools/gpu_pmc.sh) ->
profiles/<tag>_pmc_traffic.json, read by bench.py for roofline.traffic.

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE (KiB) reports half the
bytes of wide coalesced reads -> x2; WRITE_SIZE (KiB) is exact for 16-B streaming stores.
usage: python tools/pmc_traffic.py gpurun_out/<pmc tag> profiles/r01_pmc_traffic.json C1 1920 1080
"""
import collections
import csv
import glob
import json
import sys

root, out, config, W, H = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        kn = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        name = kn.split("(")[0].split("::")[-1].split("<")[0].replace("void ", "").strip()
        vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
kernels = {}
for k, d in vals.items():
    if "FETCH_SIZE" not in d or "WRITE_SIZE" not in d:
        continue  # (every pass of tools/gpu_pmc.sh sees every kernel)
    fetch = sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"])
    write = sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"])
    kernels[k] = {"fetch_kib": round(fetch, 1), "write_kib": round(write, 1), "launches_sampled": len(d["FETCH_SIZE"]),
                  "hbm_bytes_per_launch": round((2.0 * fetch + write) * 1024.0)}
    mean = lambda c: sum(d[c]) / len(d[c])
    if "SQ_ACTIVE_INST_VALU" in d and "GRBM_GUI_ACTIVE" in d:
        # VALU busy: SQ_ACTIVE_INST_VALU counts quad-cycles summed over the chip's 1024 SIMDs,
        # GRBM_GUI_ACTIVE cycles summed over its 8 XCDs (MI355X_MICROARCH.md, cycle constants
        # and DVFS rows): busy = VALU x 4 / 1024 / (GUI_ACTIVE / 8), per (serialised) dispatch
        gui = mean("GRBM_GUI_ACTIVE") / 8.0
        kernels[k]["valu_busy"] = round(mean("SQ_ACTIVE_INST_VALU") * 4.0 / 1024.0 / gui, 4) if gui > 0 else None
        kernels[k]["gui_active_cycles"] = round(gui)
    if "SQ_WAIT_ANY" in d and "SQ_WAVE_CYCLES" in d and mean("SQ_WAVE_CYCLES") > 0:
        kernels[k]["wait_frac"] = round(mean("SQ_WAIT_ANY") / mean("SQ_WAVE_CYCLES"), 4)
    if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d:
        h, m = mean("TCC_HIT_sum"), mean("TCC_MISS_sum")
        kernels[k]["l2_hit_rate"] = round(h / (h + m), 4) if h + m > 0 else None
import os
sha = None
if os.path.exists(f"{root}/lib.sha256"):  # written on the GPU box by tools/gpu_pmc.sh
    sha = open(f"{root}/lib.sha256").read().split()[0]
json.dump({"config": config, "width": W, "height": H, "source": root, "lib_sha256": sha,
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over bench.py; "
                     "bytes = (2 x FETCH_SIZE + WRITE_SIZE) KiB x 1024 per launch (gfx950 FETCH_SIZE correction)",
           "kernels": kernels}, open(out, "w"), indent=1)
print(json.dumps(kernels, indent=1))
