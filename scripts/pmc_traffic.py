#!/usr/bin/env python3
"""Per-launch HBM traffic of a bench kernel class from rocprofv3 PMC passes.

    python scripts/pmc_traffic.py <pmc dir with FETCH_SIZE> <pmc dir with WRITE_SIZE> <key> \
        <launches per step> <kernel substring> [<follower substring>]

FETCH_SIZE / WRITE_SIZE are in KB per dispatch.  On gfx950 FETCH_SIZE reports half of the bytes of a
wide (16 B/lane) streaming read, so it is doubled; WRITE_SIZE is exact for 16-B stores
(MI355X_MICROARCH.md, HBM section).

A class launch (bench.py's unit) may be a kernel plus a follower kernel that the same launcher enqueues
right after it (the weight gradients: pgemm_x6w_kernel or pgemm_b16_kernel, then the split-K
pgemm_reduce_kernel).  A follower dispatch belongs to the class when the closest preceding dispatch of
any kernel whose name starts with the class kernel's family ("pgemm_") is one of the class's own
(dispatch ids are assigned in enqueue order, and the launcher enqueues the pair back to back).
bytes_per_launch = the class's bytes over all its dispatches / the number of class dispatches: the
same mean per launch over the same dispatch mix as bench.py's `achieved` (mean FLOPs per launch / mean
launch time).  bench.py uses the entry only when its launches_per_step equals the run's.
Writes/updates profiles/pmc_traffic.json.
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnot-replication_amd"))
from gnot_amd._lib import source_hash  # noqa: E402


def dispatches(d, counter):
    """{dispatch id: (kernel name, summed counter value)}"""
    out = {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if r["Counter_Name"] != counter:
            continue
        i = int(r["Dispatch_Id"])
        name, v = out.get(i, (r["Kernel_Name"], 0.0))
        out[i] = (name, v + float(r["Counter_Value"]))
    return out


def class_kb(d, counter, sub, follow):
    disp = dispatches(d, counter)
    fam = sub.split("_")[0] + "_" if follow else None
    total, n, owner = 0.0, 0, False
    for i in sorted(disp):
        name, v = disp[i]
        if sub in name:
            total, n, owner = total + v, n + 1, True
        elif follow and follow in name:
            if owner:
                total += v
        elif fam and fam in name:
            owner = False
    return total, n


def main():
    fdir, wdir, key, per_step = sys.argv[1:5]
    sub = sys.argv[5]
    follow = sys.argv[6] if len(sys.argv) > 6 else None
    fetch_kb, launches = class_kb(fdir, "FETCH_SIZE", sub, follow)
    write_kb, wl = class_kb(wdir, "WRITE_SIZE", sub, follow)
    assert launches and launches == wl, (launches, wl)
    out_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    table = json.load(open(out_path)) if os.path.exists(out_path) else {}
    table[key] = {"kernels": [sub] + ([follow] if follow else []), "launches": launches,
                  "launches_per_step": int(per_step), "source_hash": source_hash(),
                  "fetch_size_kb_per_launch": fetch_kb / launches, "write_size_kb_per_launch": write_kb / launches,
                  "bytes_per_launch": int((2 * fetch_kb + write_kb) * 1024 / launches),
                  "source": f"{os.path.basename(fdir)}, {os.path.basename(wdir)} (sum over dispatches / launches)"}
    json.dump(table, open(out_path, "w"), indent=1)
    print(key, table[key])


if __name__ == "__main__":
    main()
