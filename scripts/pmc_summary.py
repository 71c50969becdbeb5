#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace run and its separate FETCH_SIZE / WRITE_SIZE PMC passes (scripts/prof_round.sh)
into profiles/<tag>_kernel_stats.csv, profiles/<tag>_pmc_summary.json and profiles/pmc_traffic.json.

Only the bench's batch launches are summarised (the extractor launches over all 2 x batch images: the largest grid of
each kernel).  Traffic correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE / WRITE_SIZE are KiB per dispatch; on gfx950
FETCH_SIZE under-reports wide coalesced reads and is uncalibrated for other widths, so the read side is calibrated on
the first k_resize4 launch of the batch (level 0 -> level 1): it reads every level-0 byte of the batch from HBM once
(batch x rows x cols; its 8-byte window loads overlap only inside L2), with the same 8-byte load pattern k_fast_cells
uses.  WRITE_SIZE is taken as reported.

usage: scripts/pmc_summary.py <prof_dir> <tag> <batch_images> <rows> <cols> [dominant_kernel] [steps_traced] [out_dir]

Per-step totals (hbm_bytes_per_step) sum every launch of a kernel family over the run / steps traced: k_fast_band and
k_quadtree are two launches per step (level 0 and levels 1..7), k_blur7 two, k_resize4 seven.
"""
import collections
import csv
import json
import os
import shutil
import sys


def short(name):
    return name.split("(")[0].split("::")[-1]


def launches(path, value_col=None):
    """{(kernel, grid_x, grid_y): [values]} with durations (kernel trace) or counter values (PMC)."""
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        gx = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
        gy = int(r.get("Grid_Size_Y", 1) or 1)
        v = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) if value_col is None else float(r[value_col])
        out[(short(r["Kernel_Name"]), gx, gy)].append(v)
    return out


def biggest(d):
    """kernel -> values of its largest-grid launches (the batch launches; resize: per level, keep all)."""
    best = {}
    for (k, gx, gy), v in d.items():
        if k not in best or gx * gy > best[k][0]:
            best[k] = (gx * gy, v)
    return {k: v for k, (_, v) in best.items()}


def main():
    prof, tag, batch, rows, cols = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    dom = sys.argv[6] if len(sys.argv) > 6 else "k_fast_cells"
    steps = int(sys.argv[7]) if len(sys.argv) > 7 else 0
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = sys.argv[8] if len(sys.argv) > 8 else os.path.join(root, "profiles")
    os.makedirs(out, exist_ok=True)
    shutil.copy(os.path.join(prof, "kt", "run_kernel_stats.csv"), os.path.join(out, f"{tag}_kernel_stats.csv"))
    dur_all = launches(os.path.join(prof, "kt", "run_kernel_trace.csv"))
    fetch_all = launches(os.path.join(prof, "fetch", "run_counter_collection.csv"), "Counter_Value")
    write_all = launches(os.path.join(prof, "write", "run_counter_collection.csv"), "Counter_Value")
    dur, fetch, write = biggest(dur_all), biggest(fetch_all), biggest(write_all)

    def family_total(d, k):
        return sum(sum(v) for (kk, _, _), v in d.items() if kk == k)
    calib = batch * rows * cols / (sum(fetch["k_resize4"]) / len(fetch["k_resize4"]) * 1024.0)
    summary = {"tag": tag, "batch_images": batch, "image": [rows, cols], "fetch_calibration": calib,
               "calibration_kernel": "k_resize4 (level 0 -> 1): reads batch x rows x cols bytes once",
               "note": "bytes per batch launch; read = FETCH_SIZE*1024*calibration, write = WRITE_SIZE*1024",
               "kernels": {}}
    for k in sorted(fetch):
        if not k.startswith("k_"):
            continue
        f = sum(fetch[k]) / len(fetch[k])
        w = sum(write.get(k, [0.0])) / max(len(write.get(k, [])), 1)
        t = dur.get(k)
        rd, wr = f * 1024.0 * calib, w * 1024.0
        summary["kernels"][k] = dict(read_bytes=rd, write_bytes=wr, hbm_bytes=rd + wr,
                                     avg_ns=(sum(t) / len(t)) if t else None,
                                     hbm_GBps=((rd + wr) / (sum(t) / len(t))) if t else None)
        if steps:
            rs = family_total(fetch_all, k) * 1024.0 * calib / steps
            ws = family_total(write_all, k) * 1024.0 / steps
            summary["kernels"][k].update(read_bytes_per_step=rs, write_bytes_per_step=ws, hbm_bytes_per_step=rs + ws,
                                         ms_per_step=family_total(dur_all, k) / 1e6 / steps)
    json.dump(summary, open(os.path.join(out, f"{tag}_pmc_summary.json"), "w"), indent=1)
    fam = [k for k in summary["kernels"] if k.split("<")[0] == dom.split("<")[0]]
    dom = max(fam, key=lambda k: summary["kernels"][k].get("hbm_bytes_per_step") or summary["kernels"][k]["hbm_bytes"])
    d = summary["kernels"][dom]
    json.dump({"tag": tag, "kernel": dom, "batch_images": batch, "config": "kitti" if cols == 1242 else "euroc",
               "hbm_bytes_per_launch": d["hbm_bytes"], "avg_ns": d["avg_ns"],
               "hbm_bytes_per_step": d.get("hbm_bytes_per_step"), "ms_per_step": d.get("ms_per_step"),
               # the whole step: every kernel family's HBM bytes per step (FETCH calibrated + WRITE), summed
               "step_hbm_bytes": sum(v.get("hbm_bytes_per_step") or 0.0 for v in summary["kernels"].values()) or None,
               "step_kernel_ms": sum(v.get("ms_per_step") or 0.0 for v in summary["kernels"].values()) or None,
               "source": f"profiles/{tag}_pmc_summary.json"},
              open(os.path.join(out, "pmc_traffic.json"), "w"), indent=1)
    for k, v in sorted(summary["kernels"].items(), key=lambda kv: -(kv[1]["avg_ns"] or 0))[:14]:
        print(f"{k:24s} {v['avg_ns'] / 1e3 if v['avg_ns'] else 0:8.1f} us  read {v['read_bytes'] / 1e6:8.2f} MB  "
              f"write {v['write_bytes'] / 1e6:8.2f} MB  {v['hbm_GBps'] or 0:7.1f} GB/s")


if __name__ == "__main__":
    main()
