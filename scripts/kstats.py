#!/usr/bin/env python3
"""Per-step kernel table of a rocprofv3 --stats CSV: python scripts/kstats.py <kernel_stats.csv> <steps> [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 16
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total device time per step {tot / steps / 1e6:.2f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f"{float(r['TotalDurationNs']) / steps / 1e6:8.3f} ms/step {int(r['Calls']) / steps:6.1f}/step "
          f"avg {float(r['AverageNs']) / 1e6:7.3f} ms  {r['Name'][:90]}")
