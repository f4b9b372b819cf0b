#!/usr/bin/env python3
"""Effective GPU clock per kernel from one rocprofv3 run with --pmc GRBM_GUI_ACTIVE --kernel-trace
(MI355X_MICROARCH.md, DVFS give-back: clock = GRBM_GUI_ACTIVE / 8 / kernel wall time; rocprofv3
sums the counter over the 8 XCDs; it reads high on dispatches shorter than ~0.3 ms).

  python tools/diag/clock.py gpurun_out/<tag>/clk     (the -d directory, output prefix "run")
"""
import collections
import csv
import os
import sys


def short(name):
    return name.split("(")[0].replace("void ", "")


def main(d):
    dur = {}
    with open(os.path.join(d, "run_kernel_trace.csv")) as fh:
        for r in csv.DictReader(fh):
            dur[r["Dispatch_Id"]] = (short(r["Kernel_Name"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    act = collections.defaultdict(float)
    with open(os.path.join(d, "run_counter_collection.csv")) as fh:
        for r in csv.DictReader(fh):
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                act[r["Dispatch_Id"]] += float(r["Counter_Value"])
    per = collections.defaultdict(lambda: [0.0, 0, 0])
    for k, a in act.items():
        if k not in dur:
            continue
        name, ns = dur[k]
        e = per[name]
        e[0] += a
        e[1] += ns
        e[2] += 1
    for name, (a, ns, n) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        if ns / max(n, 1) < 20_000:
            continue
        print(f"{name[:50]:50s} {n:4d} dispatches  {ns / n / 1e3:9.1f} us  {a / 8 / ns * 1e3:7.0f} MHz")


if __name__ == "__main__":
    main(sys.argv[1])
