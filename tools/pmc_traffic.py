#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/: per-kernel average duration (rocprofv3
--kernel-trace --stats) and HBM traffic per launch from the PMC passes.

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE counts half the bytes of wide coalesced streaming reads, so it is
doubled; WRITE_SIZE is exact for 16-B-per-lane stores.

  python tools/pmc_traffic.py gpurun_out/r01_levels profiles/r01/levels
"""
import collections
import csv
import json
import os
import shutil
import sys


def short(name):
    return name.split("(")[0].replace("void ", "")


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    stats = {}
    with open(os.path.join(src, "trace", "run_kernel_stats.csv")) as fh:
        for r in csv.DictReader(fh):
            stats[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                                       "total_ms": float(r["TotalDurationNs"]) / 1e6}
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for sub in ("pmc_fetch", "pmc_write"):
        path = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        with open(path) as fh:
            for r in csv.DictReader(fh):
                pmc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, s in stats.items():
        e = dict(s)
        c = pmc.get(k, {})
        if "FETCH_SIZE" in c:
            e["fetch_bytes"] = 2 * 1024 * sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"])
        if "WRITE_SIZE" in c:
            e["write_bytes"] = 1024 * sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"])
        if "fetch_bytes" in e and "write_bytes" in e:
            e["traffic_bytes"] = e["fetch_bytes"] + e["write_bytes"]
        out[k] = e
    with open(os.path.join(dst, "kernels.json"), "w") as fh:
        json.dump({"source": src, "corrections": "FETCH_SIZE KiB x2 (gfx950 wide reads), WRITE_SIZE KiB",
                   "kernels": out}, fh, indent=1)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    if os.path.exists(os.path.join(src, "bench.json")):
        shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, "bench.json"))
    for k, e in sorted(out.items(), key=lambda kv: -kv[1]["total_ms"])[:8]:
        print(f"{k[:60]:60s} {e['avg_ms']:9.4f} ms  traffic {e.get('traffic_bytes', 0) / 1e9:7.3f} GB")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
