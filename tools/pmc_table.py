"""Average per-dispatch PMC values of one kernel name pattern from the pmc_<tag>_<pass>
directories written by tools/pmc_passes.sh.  Usage: python tools/pmc_table.py <tag> [kernel-substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict

tag = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "k_proj"
vals = defaultdict(list)
for d in sorted(glob.glob(f"gpurun_out/pmc_{tag}_[0-9]")):
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        for row in csv.DictReader(open(f)):
            if pat not in row["Kernel_Name"]:
                continue
            per[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
        byc = defaultdict(list)
        for (disp, c), v in per.items():
            byc[c].append(v)
        for c, v in byc.items():
            vals[c].append(sum(v) / len(v))
for c in sorted(vals):
    print(f"{c:34s} {sum(vals[c]) / len(vals[c]):16.4g}")
