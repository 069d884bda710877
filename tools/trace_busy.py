"""Per-kernel launch statistics from a rocprofv3 kernel trace (run_kernel_trace.csv):
dispatches, mean start-to-end duration (what --stats averages) and the BUSY time per
dispatch — the union of the kernel's dispatch intervals divided by the dispatches — which
is what bench.py's roofline.kernel_ms measures with HIP events when frames are in flight
(overlapping dispatches of consecutive frames counted once).

  python tools/trace_busy.py gpurun_out/x/prof_C1/run_kernel_trace.csv [kernel-substring ...] [--json out.json]
"""
import csv
import json
import sys


def busy(intervals):
    tot, lo, hi = 0, None, None
    for a, b in sorted(intervals):
        if hi is None or a > hi:
            if hi is not None:
                tot += hi - lo
            lo, hi = a, b
        elif b > hi:
            hi = b
    if hi is not None:
        tot += hi - lo
    return tot


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    if out_json in args:
        args.remove(out_json)
    path, keys = args[0], args[1:]
    per = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if keys and not any(k in name for k in keys):
                continue
            per.setdefault(name, []).append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
    res = {}
    for name, iv in per.items():
        n = len(iv)
        res[name] = {"dispatches": n, "mean_launch_us": sum(b - a for a, b in iv) / n / 1e3,
                     "busy_per_dispatch_us": busy(iv) / n / 1e3}
        print(f"{n:6d}  launch {res[name]['mean_launch_us']:10.2f} us  busy/dispatch "
              f"{res[name]['busy_per_dispatch_us']:10.2f} us  {name[:110]}")
    if out_json:
        with open(out_json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
