"""Per-kernel PMC table from rocprofv3 --pmc passes: for every kernel name (template
arguments kept, namespaces stripped) the mean over its dispatches of each counter and of the
kernel-trace duration, across any number of pass directories.
Usage: python tools/pmc_kernels.py <pass dir> [<pass dir> ...] [--match SUBSTR] [--json OUT] [--by-grid]
(--by-grid: one row per kernel name and grid size, e.g. to keep a bench's B = 256 forward apart
from its small calibration batch)"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = name.replace("nqk::(anonymous namespace)::", "").replace("void ", "")
    name = re.sub(r"\(.*$", "", name)
    return name


def main(argv):
    dirs, match, out, by_grid = [], "", None, False
    i = 0
    while i < len(argv):
        if argv[i] == "--match":
            match = argv[i + 1]
            i += 2
        elif argv[i] == "--by-grid":
            by_grid = True
            i += 1
        elif argv[i] == "--json":
            out = argv[i + 1]
            i += 2
        else:
            dirs.append(argv[i])
            i += 1
    vals = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(float)
            names = {}
            for row in csv.DictReader(open(f)):
                k = short(row["Kernel_Name"])
                if match not in k:
                    continue
                if by_grid:
                    k += f" [grid {row['Grid_Size']}]"
                per[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
                names[row["Dispatch_Id"]] = k
            for (disp, c), v in per.items():
                vals[names[disp]][c].append(v)
        for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                k = short(row["Kernel_Name"])
                if match not in k:
                    continue
                if by_grid:
                    k += f" [grid {int(row['Grid_Size_X']) * int(row['Grid_Size_Y']) * int(row['Grid_Size_Z'])}]"
                vals[k]["duration_us"].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    res = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}
    for k in sorted(res):
        print(k)
        for c in sorted(res[k]):
            print(f"    {c:32s} {res[k][c]:16.5g}")
    if out:
        json.dump(res, open(out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:])
