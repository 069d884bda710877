"""Which hardware queue each stream's kernels ran on, from a rocprofv3 kernel trace:
dispatch counts per (kernel, Queue_Id, Stream_Id).

  python tools/queue_map.py <run_kernel_trace.csv> [kernel-substring ...]
"""
import collections
import csv
import sys


def main():
    path, keys = sys.argv[1], sys.argv[2:]
    c = collections.Counter()
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if keys and not any(k in name for k in keys):
                continue
            c[(row["Queue_Id"], row["Stream_Id"], name[:40])] += 1
    for (q, s, name), n in sorted(c.items()):
        print(f"queue {q:>3}  stream {s:>3}  {n:6d}  {name}")


if __name__ == "__main__":
    main()
