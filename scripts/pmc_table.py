#!/usr/bin/env python3
"""Per-kernel mean of every counter in rocprofv3 counter_collection CSVs: pmc_table.py <csv> [<csv> ...]"""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
names = []
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].split("::")[-1]
        if not k.startswith("k_"):
            continue
        c = r["Counter_Name"]
        if c not in names:
            names.append(c)
        agg[k][c].append(float(r["Counter_Value"]))
print("kernel".ljust(18) + "".join(n[:14].rjust(15) for n in names))
for k, d in agg.items():
    print(k.ljust(18) + "".join(("%.3g" % (sum(d[n]) / len(d[n])) if d[n] else "-").rjust(15) for n in names))
