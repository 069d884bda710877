"""Per-queue timeline of a rank share run's kernel trace (rocprofv3 run_kernel_trace.csv):
for each queue, its dispatches in order with the idle gap before each, and the summary of gaps
— where a lane waits between its frames.  python tools/share_trace.py TRACE.csv [kernel-substr]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
sub = sys.argv[2] if len(sys.argv) > 2 else "vpx"
q = defaultdict(list)
for r in rows:
    if sub not in r["Kernel_Name"] and "blend" not in r["Kernel_Name"] and "composite" not in r["Kernel_Name"]:
        continue
    q[r.get("Queue_Id", r.get("Queue_ID", "?"))].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                                                        r["Kernel_Name"].split("(")[0][-40:]))
t0 = min(s for v in q.values() for s, _, _ in v)
for qid, v in sorted(q.items()):
    v.sort()
    busy = sum(e - s for s, e, _ in v)
    span = v[-1][1] - v[0][0]
    gaps = [v[i][0] - v[i - 1][1] for i in range(1, len(v))]
    names = defaultdict(lambda: [0, 0])
    for s, e, n in v:
        names[n][0] += 1
        names[n][1] += e - s
    print(f"queue {qid}: {len(v)} dispatches, busy {busy / 1e3:.1f} us of span {span / 1e3:.1f} us "
          f"({100 * busy / max(span, 1):.0f} %), mean gap {sum(gaps) / max(len(gaps), 1) / 1e3:.1f} us")
    for n, (c, d) in sorted(names.items(), key=lambda x: -x[1][1]):
        print(f"    {c:5d} x {d / max(c, 1) / 1e3:8.1f} us  {n}")
