#!/usr/bin/env python3
"""Condense rocprofv3 --pmc counter_collection CSVs into one per-kernel summary (mean per dispatch).

    python scripts/pmc_summary.py out.csv pass1/run_counter_collection.csv [pass2/... ...]
"""
import collections
import csv
import sys

out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(lambda: collections.defaultdict(set))
for path in sys.argv[2:]:
    for r in csv.DictReader(open(path)):
        k = (r["Kernel_Name"], r.get("Grid_Size", ""))
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k][r["Counter_Name"]].add((path, r["Dispatch_Id"]))
counters = sorted({c for v in acc.values() for c in v})
with open(out, "w", newline="") as f:
    wr = csv.writer(f)
    wr.writerow(["kernel", "grid_size", "dispatches"] + [c + "_per_dispatch" for c in counters])
    for k, v in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0.0)):
        n = max(len(s) for s in disp[k].values())
        wr.writerow([k[0], k[1], n] + [f"{v[c] / max(len(disp[k][c]), 1):.1f}" if c in v else "" for c in counters])
print("wrote", out)
