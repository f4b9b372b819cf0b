#!/usr/bin/env python3
"""Per-kernel sums of the SQ counters collected by tools/sq_counters.sh."""
import collections
import csv
import os
import sys

src = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
for sub in ("p1", "p2"):
    path = os.path.join(src, sub, "run_counter_collection.csv")
    if not os.path.exists(path):
        continue
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k][r["Counter_Name"]] += 1
for k, d in agg.items():
    if "pqg" not in k:
        continue
    calls = max(cnt[k].values())
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:22s} {v / max(cnt[k][c], 1):16.0f} per dispatch")
