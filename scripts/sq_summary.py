#!/usr/bin/env python3
"""Per-kernel SQ counter summary of a scripts/prof_sq.sh run (kernel trace + two --pmc passes).

usage: scripts/sq_summary.py gpurun_out/<TAG> <out.json> [config batch_images steps_traced]

Derived per kernel (averages per dispatch):
  valu_lane_ops      = SQ_INSTS_VALU * 64 (wave instructions x lanes; an upper bound: exec-masked lanes count)
  valu_tops          = valu_lane_ops / kernel time                      [T lane-ops/s]
  valu_frac          = valu_tops / 78.64 (256 CU x 128 lanes/clk x 2.4 GHz, MI355X_MICROARCH.md: 4 SIMD-32 per CU)
  clock_ghz          = GRBM_GUI_ACTIVE / 8 XCDs / kernel time
  valu_issue_frac    = SQ_ACTIVE_INST_VALU*4 / (SQ_WAVE_CYCLES*4): share of wave-cycles issuing VALU
  wait_frac          = SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt / barrier)
  lds_conflict_frac  = SQ_LDS_BANK_CONFLICT / (SQ_ACTIVE_INST_LDS*4)
  occupancy_waves    = SQ_WAVE_CYCLES*4 / (kernel cycles at the measured clock x 256 CUs): mean resident waves per CU
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles (MI355X_MICROARCH.md, per-instruction constants).
"""
import collections
import csv
import json
import sys

PEAK_VALU_TOPS = 256 * 128 * 2.4e9 / 1e12


def short(name):
    return name.split("(")[0].split("::")[-1]


def counters(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def main():
    base, out = sys.argv[1], sys.argv[2]
    import os
    sep = "/" if os.path.isdir(base + "/kt") else "_"      # prof_round.sh (TAG/kt) or prof_sq.sh (TAG_kt) layout
    stats = {}
    for r in csv.DictReader(open(base + sep + "kt/run_kernel_stats.csv")):
        stats[short(r["Name"])] = dict(calls=int(r["Calls"]), avg_ns=float(r["AverageNs"]), pct=float(r["Percentage"]))
    c = counters(base + sep + "sqa/run_counter_collection.csv")
    for k, d in counters(base + sep + "sqb/run_counter_collection.csv").items():
        c.setdefault(k, {}).update(d)
    res = {}
    for k, s in sorted(stats.items(), key=lambda kv: -kv[1]["pct"]):
        if k not in c:
            continue
        d = c[k]
        t = s["avg_ns"] * 1e-9
        e = dict(s)
        e["counters"] = {n: round(v, 1) for n, v in sorted(d.items())}
        lane_ops = d.get("SQ_INSTS_VALU", 0.0) * 64
        e["valu_lane_ops"] = lane_ops
        e["valu_tops"] = round(lane_ops / t / 1e12, 3)
        e["valu_frac"] = round(lane_ops / t / 1e12 / PEAK_VALU_TOPS, 4)
        if d.get("GRBM_GUI_ACTIVE"):
            clk = d["GRBM_GUI_ACTIVE"] / 8 / t
            e["clock_ghz"] = round(clk / 1e9, 3)
            if d.get("SQ_WAVE_CYCLES"):
                e["occupancy_waves_per_cu"] = round(d["SQ_WAVE_CYCLES"] * 4 / (d["GRBM_GUI_ACTIVE"] / 8) / 256, 2)
        if d.get("SQ_WAVE_CYCLES"):
            e["valu_issue_frac"] = round(d.get("SQ_ACTIVE_INST_VALU", 0) / d["SQ_WAVE_CYCLES"], 4)
            e["wait_frac"] = round(d.get("SQ_WAIT_ANY", 0) / d["SQ_WAVE_CYCLES"], 4)
            e["wait_inst_frac"] = round(d.get("SQ_WAIT_INST_ANY", 0) / d["SQ_WAVE_CYCLES"], 4)
            e["lds_issue_frac"] = round(d.get("SQ_ACTIVE_INST_LDS", 0) / d["SQ_WAVE_CYCLES"], 4)
        if d.get("SQ_ACTIVE_INST_LDS"):
            e["lds_conflict_frac"] = round(d.get("SQ_LDS_BANK_CONFLICT", 0) / (d["SQ_ACTIVE_INST_LDS"] * 4), 4)
        res[k] = e
    tag = base.rstrip("/").split("/")[-1]
    steps = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    if steps:
        for k, e in res.items():
            e["launches_per_step"] = round(e["calls"] / steps, 3)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from kernel_share import source_sha16
    meta = {"tag": tag, "config": sys.argv[3] if len(sys.argv) > 3 else "kitti", "source_sha16": source_sha16(),
            "batch_images": int(sys.argv[4]) if len(sys.argv) > 4 else 128,
            "note": "per-dispatch averages of a short bench run (scripts/prof_sq.sh); SQ_* wave counters summed over "
                    "the chip by rocprofv3; valu_lane_ops = SQ_INSTS_VALU x 64"}
    json.dump(dict(meta, peak_valu_tops=PEAK_VALU_TOPS, kernels=res), open(out, "w"), indent=1)
    for k, e in list(res.items())[:14]:
        print(f"{k:24s} {e['avg_ns']/1e3:8.1f}us {e['pct']:5.1f}% valu {e['valu_tops']:6.2f}T ({100*e['valu_frac']:4.1f}%) "
              f"clk {e.get('clock_ghz', 0):.2f} occ {e.get('occupancy_waves_per_cu', 0):5.1f} issue {e.get('valu_issue_frac', 0):.3f} "
              f"wait {e.get('wait_frac', 0):.3f} winst {e.get('wait_inst_frac', 0):.3f} lds {e.get('lds_issue_frac', 0):.3f} "
              f"conf {e.get('lds_conflict_frac', 0):.3f}")


if __name__ == "__main__":
    main()
