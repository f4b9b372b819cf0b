"""Per-column kernel breakdown of tools/diag/at_cols.py from a rocprofv3 kernel trace (decodes split
at each k_prepare launch: the row-group check's 11 decodes first, then reps + 1 per column)."""
import collections
import csv
import sys

sys.path.insert(0, "tools/gen")
import pqgtools  # noqa: E402

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
decodes, cur = [], None
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pqg::", "")
    if n == "k_prepare":
        cur = []
        decodes.append(cur)
    if cur is not None:
        cur.append((n, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
decodes = decodes[11:]
for j, (name, _) in enumerate(pqgtools.ALLTYPES):
    ds = decodes[j * (reps + 1) + 1:(j + 1) * (reps + 1)]
    agg = collections.OrderedDict()
    span = 0.0
    for d in ds:
        span += (d[-1][3] - d[0][2]) / 1e3
        for n, us, _, _ in d:
            agg[n] = agg.get(n, 0.0) + us / len(ds)
    busy = sum(agg.values())
    print(f"{name:16s} span {span / len(ds):8.1f} us  kernels {busy:8.1f} us  launches {len(ds[0])}")
    for n, us in sorted(agg.items(), key=lambda x: -x[1])[:8]:
        print(f"      {n[:40]:40s} {us:8.1f}")
