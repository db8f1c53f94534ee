#!/usr/bin/env python
"""Summarise a rocprofv3 kernel trace: per (kernel, grid) average duration, calls and
total, sorted by total time.  usage: prof_summary.py run_kernel_trace.csv [N]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
agg = collections.defaultdict(list)
for r in rows:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    name = r["Kernel_Name"].replace("nqk::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    agg[(name[:48], r["Grid_Size_X"], r["Grid_Size_Z"])].append(d)
tot = sum(sum(v) for v in agg.values())
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print(f"{k[0]:48s} grid={k[1]:>9s}x{k[2]:<5s} calls={len(v):5d} avg={sum(v)/len(v):9.1f}us "
          f"total={sum(v)/1e3:8.2f}ms {100*sum(v)/tot:5.1f}%")
