"""Summarise the FETCH_SIZE / WRITE_SIZE calibration (tools/gpu_calib.sh, native/fetch_calib.hip)
-> profiles/<tag>_fetch_calibration.json: per probe kernel, the known bytes it must move, the
counters, and counter bytes / known bytes.

usage: python tools/fetch_calib.py gpurun_out/calib profiles/r03_fetch_calibration.json
"""
import collections
import csv
import json
import re
import sys

root, out = sys.argv[1], sys.argv[2]
LINES = 1 << 22  # distinct random lines per probe (fetch_calib.hip: n)
known = {}  # probe name -> (bytes that must move, what)
times = {}
for ln in open(f"{root}/plain.log"):
    m = re.match(r"(\S+)\s+known_bytes (\d+)\s+ms ([0-9.]+)", ln)
    if m:
        known[m.group(1)] = int(m.group(2))
        times[m.group(1)] = float(m.group(3))
# dispatch order of the probes (each after a write + read eviction sweep)
order = ["rand_read_1B", "rand_read_4B", "rand_read_8B", "rand_read_16B", "rand_read_1B_hi", "rand_read_halves",
         "stream_read_16B", "rand_write_4B", "rand_write_16B", "stream_write_16B"]
ctr = collections.defaultdict(dict)
for p in ("p1", "p2", "p3", "p4"):
    for r in csv.DictReader(open(f"{root}/{p}/run_counter_collection.csv")):
        k = (int(r["Dispatch_Id"]), r["Kernel_Name"].split("(")[0].replace("void ", ""))
        ctr[k][r["Counter_Name"]] = ctr[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
disp = sorted(ctr)
# the probes are the dispatches right after each eviction pair (stream_write, stream_read)
probes = []
i = 0
while i < len(disp):
    if disp[i][1] == "stream_write" and i + 2 < len(disp) and disp[i + 1][1] == "stream_read":
        probes.append(disp[i + 2])
        i += 3
    else:
        i += 1
res = {}
for name, k in zip(order, probes):
    c = ctr[k]
    kb = known[name]
    fetch_b = c.get("FETCH_SIZE", 0.0) * 1024.0
    write_b = c.get("WRITE_SIZE", 0.0) * 1024.0
    res[name] = {"kernel": k[1], "known_bytes": kb, "ms": times[name],
                 "FETCH_SIZE_bytes": round(fetch_b), "WRITE_SIZE_bytes": round(write_b),
                 "TCC_EA0_RDREQ": round(c.get("TCC_EA0_RDREQ_sum", 0.0)), "TCC_MISS": round(c.get("TCC_MISS_sum", 0.0)),
                 "fetch_over_known": round(fetch_b / kb, 4), "write_over_known": round(write_b / kb, 4)}
json.dump({"source": root, "probe": "tools/native/fetch_calib.hip (8 GiB buffer, 1 GiB write+read eviction sweep before each probe; "
           f"random probes: one access per lane to {LINES} distinct 128-B lines, known bytes = lines x 128 B)",
           "probes": res}, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
