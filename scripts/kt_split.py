#!/usr/bin/env python3
"""Per-(kernel, grid) average durations from a rocprofv3 kernel trace: scripts/kt_split.py <run_kernel_trace.csv> [n]."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].split("(")[0].split("::")[-1]
    agg[(n, r["Grid_Size_X"], r["Grid_Size_Y"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[: int(sys.argv[2]) if len(sys.argv) > 2 else 24]:
    v = sorted(v)
    print(f"{k[0][:26]:26s} {k[1]:>9}x{k[2]:<4} n={len(v):3d} avg={sum(v)/len(v):8.1f} med={v[len(v)//2]:8.1f} us")
