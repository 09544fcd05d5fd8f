#!/usr/bin/env python3
"""Per-launch HBM traffic of the bench's roofline kernel class from rocprofv3 PMC passes.

    python scripts/pmc_traffic.py <pmc dir with FETCH_SIZE> <pmc dir with WRITE_SIZE> <key> \
        <launches per step> <kernel substring> [<kernel substring> ...]

FETCH_SIZE / WRITE_SIZE are in KB per dispatch.  On gfx950 FETCH_SIZE reports half of the bytes of a
wide (16 B/lane) streaming read, so it is doubled; WRITE_SIZE is exact for 16-B stores
(MI355X_MICROARCH.md, HBM section).

A class launch (bench.py's unit) may be several kernels (the weight gradients: pgemm_x6w_kernel + its
split-K pgemm_reduce_kernel).  bytes_per_launch = the class's bytes summed over every dispatch of
the listed kernels / the number of class launches (dispatches of the FIRST substring): the same mean
per launch over the same dispatch mix as bench.py's `achieved` (mean FLOPs per launch / mean launch
time).  bench.py uses the entry only when its launches_per_step equals the run's.
Writes/updates profiles/pmc_traffic.json.
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(d, counter, sub):
    vals = {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if sub in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return vals


def main():
    fdir, wdir, key, per_step = sys.argv[1:5]
    subs = sys.argv[5:]
    launches = len(per_dispatch(fdir, "FETCH_SIZE", subs[0]))
    fetch_kb = sum(sum(per_dispatch(fdir, "FETCH_SIZE", s).values()) for s in subs)
    write_kb = sum(sum(per_dispatch(wdir, "WRITE_SIZE", s).values()) for s in subs)
    out_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    table = json.load(open(out_path)) if os.path.exists(out_path) else {}
    table[key] = {"kernels": subs, "launches": launches, "launches_per_step": int(per_step),
                  "fetch_size_kb_per_launch": fetch_kb / launches, "write_size_kb_per_launch": write_kb / launches,
                  "bytes_per_launch": int((2 * fetch_kb + write_kb) * 1024 / launches),
                  "source": f"{os.path.basename(fdir)}, {os.path.basename(wdir)} (sum over dispatches / launches)"}
    json.dump(table, open(out_path, "w"), indent=1)
    print(key, table[key])


if __name__ == "__main__":
    main()
