#!/usr/bin/env python3
"""C3 all-pairs profile summary (scripts/prof_c3.sh output): per launch shape of k_bf_tile / k_bf_merge*, the average
kernel-trace duration and SQ_INSTS_VALU x 64 against the VALU peak.  usage: scripts/c3_summary.py <dir> <tag> <out.json>"""
import collections
import csv
import json
import sys

PEAK = 256 * 128 * 2.4e9 / 1e12
base, tag, out_path = sys.argv[1], sys.argv[2], sys.argv[3]
kt = collections.defaultdict(list)
for r in csv.DictReader(open(f"{base}/kt/run_kernel_trace.csv")):
    n = r["Kernel_Name"].split("(")[0].split("::")[-1]
    if "k_bf" in n:
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        kt[(n, g)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
sq = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for r in csv.DictReader(open(f"{base}/sq/run_counter_collection.csv")):
    n = r["Kernel_Name"].split("(")[0].split("::")[-1]
    if "k_bf" in n:
        g = int(r["Grid_Size"])
        sq[(n, g)][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(n, g)].add(r["Dispatch_Id"])
out = {"tag": tag, "source": "scripts/prof_c3.sh (kernel trace + one SQ pass of bench.py --steps 1 --warmup 1 with the "
                             "C3 block)", "peak_valu_tops": PEAK, "launches": {}}
for (n, g), v in sorted(kt.items()):
    avg = sum(v) / len(v)
    c = sq.get((n, g), {})
    nd = len(cnt.get((n, g), [])) or 1
    ops = c.get("SQ_INSTS_VALU", 0) / nd * 64
    e = {"kernel": n, "grid": g, "launches": len(v), "avg_us": round(avg / 1e3, 2), "valu_lane_ops": ops,
         "valu_tops": round(ops / (avg * 1e-9) / 1e12, 3) if ops else None,
         "valu_frac": round(ops / (avg * 1e-9) / 1e12 / PEAK, 4) if ops else None,
         "lds_bank_conflicts": c.get("SQ_LDS_BANK_CONFLICT")}
    out["launches"][f"{n} grid {g}"] = e
    print(e)
json.dump(out, open(out_path, "w"), indent=1)
