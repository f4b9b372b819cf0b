"""Concurrency profile of a rocprofv3 kernel trace: over the last `span_ms` of the trace, the
busy time, average kernels in flight and the kernels with the most device time."""
import collections
import csv
import sys

rows = [(r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pqg::", ""), int(r["Start_Timestamp"]),
         int(r["End_Timestamp"]), r.get("Queue_Id", ""), r.get("Stream_Id", "")) for r in csv.DictReader(open(sys.argv[1]))]
rows.sort(key=lambda x: x[1])
span = float(sys.argv[2]) * 1e6 if len(sys.argv) > 2 else 20e6
t1 = max(r[2] for r in rows)
t0 = t1 - span
sel = [r for r in rows if r[1] >= t0]
busy = sum(e - s for _, s, e, _, _ in sel)
ev = sorted([(s, 1) for _, s, e, _, _ in sel] + [(e, -1) for _, s, e, _, _ in sel])
cur = mx = 0
covered = 0
last = t0
for t, d in ev:
    if cur > 0:
        covered += t - last
    cur += d
    mx = max(mx, cur)
    last = t
print(f"window {span / 1e6:.1f} ms: kernels {len(sel)}, busy {busy / 1e6:.2f} ms, avg in flight {busy / span:.2f}, "
      f"max {mx}, GPU-idle {(span - covered) / 1e6:.2f} ms")
agg = collections.Counter()
cnt = collections.Counter()
for n, s, e, _, _ in sel:
    agg[n] += e - s
    cnt[n] += 1
for n, t in agg.most_common(14):
    print(f"  {n[:44]:44s} {cnt[n]:6d} {t / 1e6:8.2f} ms  avg {t / cnt[n] / 1e3:7.1f} us")
q = collections.Counter(r[3] for r in sel)
print("queues:", dict(q))
