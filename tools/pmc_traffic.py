#!/usr/bin/env python
"""Per-kernel HBM traffic from rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE in separate
runs, kilobytes per dispatch).  gfx950: FETCH_SIZE reports half the bytes of wide
streaming reads (MI355X_MICROARCH.md, HBM section) -> doubled here.  Writes
profiles/pmc_traffic.json: per kernel family (name prefix) the mean per launch.
usage: pmc_traffic.py <fetch_dir> <write_dir> [out.json]"""
import collections
import csv
import json
import sys


def load(d, counter):
    vals = collections.defaultdict(dict)
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].replace("nqk::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        fam = name.split("<")[0]
        vals[fam][r["Dispatch_Id"]] = vals[fam].get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return {f: list(v.values()) for f, v in vals.items()}


fetch, write = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
out = {"note": "HBM bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE (KB counters x 1024); gfx950 FETCH_SIZE "
               "correction per MI355X_MICROARCH.md; mean over the profiled launches", "kernels": {}}
for fam in sorted(set(fetch) | set(write)):
    f = fetch.get(fam, [0.0])
    w = write.get(fam, [0.0])
    fb = 2 * 1024 * sum(f) / len(f)
    wb = 1024 * sum(w) / len(w)
    out["kernels"][fam] = {"launches": len(f), "fetch_bytes": round(fb), "write_bytes": round(wb),
                           "hbm_bytes_per_launch": round(fb + wb)}
json.dump(out, open(sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_traffic.json", "w"), indent=1)
for k, v in out["kernels"].items():
    print(k, v)
