#!/usr/bin/env python3
"""Per-kernel SQ counter summary of a tools/sq_counters.sh run (the two --pmc passes):
instructions per unit and the wave-cycle split. Labels follow MI355X_MICROARCH.md (SQ table):
SQ_WAIT_ANY = wave parked on s_waitcnt / barrier, SQ_WAIT_INST_ANY = issue stall,
SQ_ACTIVE_INST_ANY = issuing; the three are disjoint and sum to ~SQ_WAVE_CYCLES.

  python tools/sq_summary.py gpurun_out/<tag> <units> <unit name> [kernel substrings...]
"""
import collections
import csv
import os
import sys


def short(name):
    return name.split("(")[0].replace("void ", "")


def main(d, units, uname, keys):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    for sub in ("p1", "p2"):
        with open(os.path.join(d, sub, "run_counter_collection.csv")) as fh:
            for r in csv.DictReader(fh):
                k = short(r["Kernel_Name"])
                if keys and not any(s in k for s in keys):
                    continue
                tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
    print(f"| kernel | VALU / {uname} | SALU / {uname} | LDS / {uname} | VMEM rd+wr / {uname} | issuing "
          f"(ACTIVE_INST_ANY) | parked on s_waitcnt / barrier (WAIT_ANY) | issue-stalled (WAIT_INST_ANY) |")
    print("|---|---|---|---|---|---|---|---|")
    for k, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        print(f"| `{k}` | {c['SQ_INSTS_VALU'] / units:.0f} | {c['SQ_INSTS_SALU'] / units:.0f} | "
              f"{c['SQ_INSTS_LDS'] / units:.0f} | {(c['SQ_INSTS_VMEM_RD'] + c['SQ_INSTS_VMEM_WR']) / units:.1f} | "
              f"{c['SQ_ACTIVE_INST_ANY'] / wc:.2f} | {c['SQ_WAIT_ANY'] / wc:.2f} | {c['SQ_WAIT_INST_ANY'] / wc:.2f} |")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]), sys.argv[3], sys.argv[4:])
