"""Per-kernel duration summary from a rocprofv3 results database (--kernel-trace, default
sqlite output) or kernel_stats.csv: name, calls, average and total microseconds."""
import collections
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, start, end from kernels").fetchall()
    agg = collections.OrderedDict()
    for n, s, e in rows:
        a = agg.setdefault(n, [0, 0.0])
        a[0] += 1
        a[1] += (e - s) / 1e3
    return agg


def main(path):
    if os.path.isdir(path):
        dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
        path = dbs[0]
    agg = from_db(path)
    tot = sum(v[1] for v in agg.values())
    print(f"{'kernel':70s} {'calls':>6s} {'avg_us':>10s} {'total_us':>11s} {'pct':>6s}")
    for n, (k, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        short = n if len(n) < 70 else n[:67] + "..."
        print(f"{short:70s} {k:6d} {t / k:10.1f} {t:11.1f} {100 * t / tot:6.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
