#!/usr/bin/env python3
"""Per-step timeline of a rocprofv3 kernel trace: the last `adamw_kernel` delimits steps.
    python scripts/trace_step.py run_kernel_trace.csv [step index from the end, default 1]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
back = int(sys.argv[2]) if len(sys.argv) > 2 else 1
ends = [i for i, r in enumerate(rows) if "adamw_kernel" in r["Kernel_Name"]]
lo, hi = ends[-back - 1] + 1, ends[-back] + 1
step = rows[lo:hi]
t0 = int(step[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in step)
print(f"step wall (first start -> last end): {(t1 - t0) / 1e6:.2f} ms, {len(step)} kernels")
busy = collections.defaultdict(float)
per = collections.defaultdict(lambda: [0, 0.0])
for r in step:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    busy[r["Queue_Id"]] += d
    k = r["Kernel_Name"].split("(")[0][:60]
    per[(r["Queue_Id"], k)][0] += 1
    per[(r["Queue_Id"], k)][1] += d
for q, b in sorted(busy.items()):
    print(f"queue {q}: busy {b:.2f} ms")
for (q, k), (n, d) in sorted(per.items(), key=lambda kv: -kv[1][1])[:30]:
    print(f"  q{q} {k:60s} x{n:3d} {d:8.2f} ms")
# union of busy intervals = time with >= 1 kernel running
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in step)
u, cs, ce = 0, iv[0][0], iv[0][1]
for s, e in iv[1:]:
    if s > ce:
        u += ce - cs; cs, ce = s, e
    else:
        ce = max(ce, e)
u += ce - cs
print(f"time with >=1 kernel running: {u / 1e6:.2f} ms")
if len(sys.argv) > 3:
    for r in step:
        print(f"{(int(r['Start_Timestamp']) - t0) / 1e6:9.3f} {(int(r['End_Timestamp']) - t0) / 1e6:9.3f} q{r['Queue_Id']} {r['Kernel_Name'].split('(')[0][:70]} g={r['Grid_Size_X']}")
