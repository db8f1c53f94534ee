#!/usr/bin/env python
"""The patch embedding's two half-batch launches in a rocprofv3 kernel trace of the default
(two-stream) bench.py: per forward, each half's [start, end], the union of the two, how long both
ran together, and which kernels of the other stream ran beside the later half's tail.

usage: embed_overlap.py run_kernel_trace.csv
"""
import collections
import csv
import sys


def short(name):
    return name.replace("nqk::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:40]


rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"])
             for r in rows), key=lambda k: k[0])
emb = [k for k in ks if k[2].startswith("k_embed_q")]
pairs = []
i = 0
while i + 1 < len(emb):
    a, b = emb[i], emb[i + 1]
    if b[0] < a[1] + 2_000_000 and a[3] != b[3]:  # the two halves of one forward (different queues)
        pairs.append((a, b))
        i += 2
    else:
        i += 1
print(f"{len(emb)} k_embed_q launches, {len(pairs)} two-queue pairs")
tail_k = collections.Counter()
for a, b in pairs:
    d0, d1 = (a[1] - a[0]) / 1e3, (b[1] - b[0]) / 1e3
    u = (max(a[1], b[1]) - min(a[0], b[0])) / 1e3
    both = max(0, min(a[1], b[1]) - max(a[0], b[0])) / 1e3
    first_end, last_end = min(a[1], b[1]), max(a[1], b[1])
    beside = [k for k in ks if k[0] < last_end and k[1] > first_end and not k[2].startswith("k_embed_q")]
    for k in beside:
        tail_k[k[2]] += 1
    print(f"halves {d0:7.1f} / {d1:7.1f} us, start offset {abs(b[0] - a[0]) / 1e3:6.1f} us, union {u:7.1f} us, "
          f"both running {both:7.1f} us, tail {(last_end - first_end) / 1e3:6.1f} us with {len(beside)} other kernels beside it")
print("kernels beside the tails:", dict(tail_k.most_common(8)))
