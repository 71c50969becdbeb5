#!/usr/bin/env python3
"""Timeline view of a rocprofv3 kernel trace of the bench: scripts/kt_timeline.py <run_kernel_trace.csv> [skip_frac].

Over the steady part of the trace (kernels after the first `skip_frac` of its span, default 0.5): the fraction of
wall time with at least one kernel running, the mean number of kernels in flight, per-stream busy fractions and
per-kernel share of the summed kernel time, so one can tell a latency-bound step (gaps, one kernel at a time) from a
throughput-bound one (always several in flight).
"""
import collections
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if not r["Kernel_Name"].startswith("__amd")]
skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
t0 = min(int(r["Start_Timestamp"]) for r in rows)
t1 = max(int(r["End_Timestamp"]) for r in rows)
lo = t0 + (t1 - t0) * skip
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1],
       r["Stream_Id"], r["Queue_Id"]) for r in rows if int(r["Start_Timestamp"]) >= lo]
a, b = min(k[0] for k in ks), max(k[1] for k in ks)
span = b - a
ev = sorted([(k[0], 1) for k in ks] + [(k[1], -1) for k in ks])
busy = 0
area = 0
cur = 0
last = a
hist = collections.Counter()
for t, d in ev:
    if cur > 0:
        busy += t - last
    area += cur * (t - last)
    hist[min(cur, 6)] += t - last
    cur += d
    last = t
print(f"window {span / 1e3:.1f} us, {len(ks)} kernels; busy {busy / span:.3f}; mean in flight {area / span:.2f}")
print("in-flight histogram:", {k: round(v / span, 3) for k, v in sorted(hist.items())})
per_stream = collections.defaultdict(int)
for s, e, n, st, q in ks:
    per_stream[(st, q)] += e - s
for k, v in sorted(per_stream.items()):
    print(f"stream {k[0]} queue {k[1]}: summed kernel time {v / span:.3f} of the window")
per = collections.defaultdict(lambda: [0, 0])
for s, e, n, st, q in ks:
    per[n][0] += e - s
    per[n][1] += 1
tot = sum(v[0] for v in per.values())
for n, (d, c) in sorted(per.items(), key=lambda kv: -kv[1][0])[:20]:
    print(f"{n[:28]:28s} n={c:4d} sum={d / 1e3:9.1f} us  {d / tot:6.3f} of kernel time  {d / span:6.3f} of wall")
