#!/usr/bin/env python3
"""Top kernels of a rocprofv3 --stats kernel_stats.csv: calls, average / max microseconds, total ms.

  python tools/kstat_csv.py gpurun_out/<tag>/run_kernel_stats.csv [N]"""
import csv
import sys


def main(path, n=30):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:n]:
        print(f"{r['Name'].split('(')[0][:62]:62s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs']) / 1e3:9.1f} "
              f"max_us={float(r['MaxNs']) / 1e3:9.1f} tot_ms={float(r['TotalDurationNs']) / 1e6:8.2f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30)
