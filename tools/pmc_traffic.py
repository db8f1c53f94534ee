#!/usr/bin/env python
"""Per-kernel HBM traffic from rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE in separate
runs, kilobytes per dispatch).  gfx950: FETCH_SIZE reports half the bytes of wide
streaming reads (MI355X_MICROARCH.md, HBM section) -> doubled here.  Writes
profiles/pmc_traffic.json:
  kernels         per kernel family (name prefix): the mean per launch over every launch;
  per_shape       the int8 ViT-Base projection GEMMs (k_pg, int8 weights) of the B = 256 forward,
                  one entry per shape (qkv / out / up / down, told apart by the template's
                  epilogue and k-step count), launches at that template's largest grid only
                  (calibration batches and half-batch launches excluded; profile with NQK_SPLIT=0);
  per_shape_tiny  the same for ViT-Ti's k_pg launches (K = 192: qkv, up).
bench.py reads per_shape / per_shape_tiny for roofline.traffic.
usage: pmc_traffic.py <fetch_dir> <write_dir> [out.json]"""
import collections
import csv
import glob
import json
import os
import re
import sys

PG = re.compile(r"k_pg<(\d+), (\d+), (true|false), (true|false), (true|false)(?:, (\d+))?(?:, (true|false))?>")


def load(d, counter):
    """{dispatch id: (name, grid, KB)} for one counter."""
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].replace("nqk::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            key = r["Dispatch_Id"]
            prev = out.get(key, (name, int(r["Grid_Size"]), 0.0))
            out[key] = (name, int(r["Grid_Size"]), prev[2] + float(r["Counter_Value"]))
    return out


def shape_of(name):
    m = PG.match(name)
    if not m or m.group(4) == "true":  # not k_pg, or int4 weights
        return None, None
    epi, nk = int(m.group(1)), int(m.group(2))
    cfg = "tiny" if nk == 3 else "base"
    if epi == 0:
        return cfg, "qkv"
    if epi in (4, 5):
        return cfg, "up"
    if epi == 3:
        return cfg, "down" if nk == 48 else "out"
    return None, None


def main(argv):
    fetch, write = load(argv[0], "FETCH_SIZE"), load(argv[1], "WRITE_SIZE")
    out = {"note": "HBM bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE (KB counters x 1024); gfx950 FETCH_SIZE "
                   "correction per MI355X_MICROARCH.md; kernels: mean over the profiled launches; per_shape / "
                   "per_shape_tiny: the int8 k_pg launches of the B = 256 forward (largest grid per template)",
           "kernels": {}, "per_shape": {}, "per_shape_tiny": {}}
    fam_f, fam_w = collections.defaultdict(list), collections.defaultdict(list)
    for _, (name, _, v) in fetch.items():
        fam_f[name.split("<")[0]].append(v)
    for _, (name, _, v) in write.items():
        fam_w[name.split("<")[0]].append(v)
    for fam in sorted(set(fam_f) | set(fam_w)):
        f, w = fam_f.get(fam, [0.0]), fam_w.get(fam, [0.0])
        fb, wb = 2 * 1024 * sum(f) / len(f), 1024 * sum(w) / len(w)
        out["kernels"][fam] = {"launches": len(f), "fetch_bytes": round(fb), "write_bytes": round(wb),
                               "hbm_bytes_per_launch": round(fb + wb)}
    # per template: the launches at its largest grid
    by_t = collections.defaultdict(lambda: {"f": [], "w": [], "grid": 0})
    for src, key in ((fetch, "f"), (write, "w")):
        grids = collections.defaultdict(int)
        for name, grid, _ in src.values():
            grids[name] = max(grids[name], grid)
        for name, grid, v in src.values():
            if grid == grids[name]:
                by_t[name][key].append(v)
                by_t[name]["grid"] = grid
    for name, d in sorted(by_t.items()):
        cfg, shape = shape_of(name)
        if not shape or not d["f"] or not d["w"]:
            continue
        fb, wb = 2 * 1024 * sum(d["f"]) / len(d["f"]), 1024 * sum(d["w"]) / len(d["w"])
        ent = {"kernel": name, "grid_threads": d["grid"], "launches": len(d["f"]), "fetch_bytes": round(fb),
               "write_bytes": round(wb), "hbm_bytes_per_launch": round(fb + wb)}
        tgt = out["per_shape" if cfg == "base" else "per_shape_tiny"]
        if shape in tgt:  # two templates of one shape (e.g. GELU table on some layers only): launch-weighted
            old = tgt[shape]
            n = old["launches"] + ent["launches"]
            for k in ("fetch_bytes", "write_bytes", "hbm_bytes_per_launch"):
                ent[k] = round((old[k] * old["launches"] + ent[k] * ent["launches"]) / n)
            ent["kernel"] = old["kernel"] + " + " + name
            ent["launches"] = n
        tgt[shape] = ent
    path = argv[2] if len(argv) > 2 else "profiles/pmc_traffic.json"
    json.dump(out, open(path, "w"), indent=1)
    for k in ("per_shape", "per_shape_tiny"):
        for s, v in out[k].items():
            print(k, s, v)


if __name__ == "__main__":
    main(sys.argv[1:])
