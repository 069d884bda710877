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
    if "SQ_INSTS_VALU" in d and "GRBM_GUI_ACTIVE" in d:
        # VALU busy: the fraction of the chip's 1024 SIMDs' cycles spent issuing VALU, at the
        # 2 cycles a wave64 VALU instruction holds a SIMD (MI355X_MICROARCH.md, v_fma_f32 row);
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs (DVFS row) -> /8 = the dispatch's cycles.
        # (SQ_ACTIVE_INST_VALU counts one per instruction on gfx950 -- measured 1.00-1.04 x
        # SQ_INSTS_VALU -- so it is an instruction count, not quad-cycles: x4 overstated it 2x.)
        gui = mean("GRBM_GUI_ACTIVE") / 8.0
        kernels[k]["valu_busy"] = round(mean("SQ_INSTS_VALU") * 2.0 / 1024.0 / gui, 4) if gui > 0 else None
        kernels[k]["gui_active_cycles"] = round(gui)
        if "SQ_WAVE_CYCLES" in d and gui > 0:  # quad-cycles, summed over waves
            kernels[k]["waves_per_simd"] = round(mean("SQ_WAVE_CYCLES") * 4.0 / 1024.0 / gui, 2)
    if "SQ_WAIT_ANY" in d and "SQ_WAVE_CYCLES" in d and mean("SQ_WAVE_CYCLES") > 0:
        # a wave's cycles split three ways (MI355X_MICROARCH.md, PMC slots): parked on
        # s_waitcnt / barrier, ready but not issued (dependency or arbitration), issuing
        wc = mean("SQ_WAVE_CYCLES")
        kernels[k]["wait_frac"] = round(mean("SQ_WAIT_ANY") / wc, 4)
        if "SQ_WAIT_INST_ANY" in d and "SQ_ACTIVE_INST_ANY" in d:
            kernels[k]["issue_stall_frac"] = round(mean("SQ_WAIT_INST_ANY") / wc, 4)
            kernels[k]["issuing_frac"] = round(mean("SQ_ACTIVE_INST_ANY") / wc, 4)
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
