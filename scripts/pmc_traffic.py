#!/usr/bin/env python3
"""Per-launch HBM traffic of the bench's roofline kernel from rocprofv3 PMC passes.

    python scripts/pmc_traffic.py <pmc dir with FETCH_SIZE> <pmc dir with WRITE_SIZE> <kernel substring> <key>

FETCH_SIZE / WRITE_SIZE are in KB per dispatch.  On gfx950 FETCH_SIZE reports half of the bytes of a
wide (16 B/lane) streaming read, so it is doubled; WRITE_SIZE is exact for 16-B stores
(MI355X_MICROARCH.md, HBM section).  Writes/updates profiles/pmc_traffic.json, which bench.py reads.
"""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(d, counter, sub):
    vals = {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if sub in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    fdir, wdir, sub, key = sys.argv[1:5]
    f = per_dispatch(fdir, "FETCH_SIZE", sub)
    w = per_dispatch(wdir, "WRITE_SIZE", sub)
    fetch_kb, write_kb = statistics.median(f), statistics.median(w)
    out_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    table = json.load(open(out_path)) if os.path.exists(out_path) else {}
    table[key] = {"kernel": sub, "dispatches": [len(f), len(w)], "fetch_size_kb": fetch_kb, "write_size_kb": write_kb,
                  "bytes_per_launch": int((2 * fetch_kb + write_kb) * 1024),
                  "source": f"{os.path.basename(fdir)}, {os.path.basename(wdir)} (medians over dispatches)"}
    json.dump(table, open(out_path, "w"), indent=1)
    print(key, table[key])


if __name__ == "__main__":
    main()
