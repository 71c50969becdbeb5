#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace/stats run and its separate FETCH_SIZE / WRITE_SIZE PMC passes
into profiles/<tag>_*.  Traffic correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE/WRITE_SIZE are KiB;
on gfx950 FETCH_SIZE under-reports wide coalesced reads by 2x and is uncalibrated for other widths, so
the read side is calibrated on k_copy_level0, whose bytes are known exactly (it reads every input image
once with coalesced byte loads: batch x rows x cols bytes), and the same factor is applied to the other
kernels (all of them read bytes or dwords, never 16-B vectors).

usage: scripts/pmc_summary.py <prof_dir> <tag> <batch_images> <rows> <cols> [dominant_stage]
"""
import collections
import csv
import json
import os
import shutil
import sys

R1A_CALIBRATION = 1.3265335392964581
STAGE_OF = {"k_copy_level0": "copy_level0", "k_resize": "resize", "k_fast_cells": "fast_cells", "k_blur7": "blur7",
            "k_quadtree": "quadtree", "k_describe": "describe", "k_stereo": "stereo_match",
            "k_stereo_sad": "stereo_refine", "k_bow_pairs": "keyframe_bow_fusion"}


def short(name):
    n = name.split("(")[0]
    return n.split("::")[-1]


def per_kernel(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    prof, tag, batch, rows, cols = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    dom = sys.argv[6] if len(sys.argv) > 6 else None
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = os.path.join(root, "profiles")
    os.makedirs(out, exist_ok=True)
    shutil.copy(os.path.join(prof, "kt", "run_kernel_stats.csv"), os.path.join(out, f"{tag}_kernel_stats.csv"))
    fetch = per_kernel(os.path.join(prof, "fetch", "run_counter_collection.csv"))
    write = per_kernel(os.path.join(prof, "write", "run_counter_collection.csv"))
    if "k_copy_level0" in fetch:
        calib = batch * rows * cols / (fetch["k_copy_level0"] * 1024.0)
    else:
        # level 0 is now read in place (no copy kernel): reuse the factor measured on k_copy_level0 in r1a
        # (profiles/r1a_pmc_summary.json), the same byte-load pattern
        calib = R1A_CALIBRATION
    stats = {}
    for r in csv.DictReader(open(os.path.join(prof, "kt", "run_kernel_stats.csv"))):
        stats[short(r["Name"])] = dict(calls=int(r["Calls"]), avg_ns=float(r["AverageNs"]), pct=float(r["Percentage"]))
    summary = {"tag": tag, "batch_images": batch, "image": [rows, cols], "fetch_calibration": calib,
               "note": "bytes per dispatch; read = FETCH_SIZE*1024*calibration, write = WRITE_SIZE*1024",
               "kernels": {}}
    for k in sorted(fetch):
        if not k.startswith("k_"):
            continue
        rd, wr = fetch[k] * 1024.0 * calib, write.get(k, 0.0) * 1024.0
        summary["kernels"][k] = dict(stage=STAGE_OF.get(k), read_bytes=rd, write_bytes=wr, hbm_bytes=rd + wr,
                                     **stats.get(k, {}))
    json.dump(summary, open(os.path.join(out, f"{tag}_pmc_summary.json"), "w"), indent=1)
    if dom is None:
        dom_k = max((k for k in stats if k.startswith("k_") and k != "k_resize"), key=lambda k: stats[k]["pct"])
    else:
        dom_k = [k for k, s in STAGE_OF.items() if s == dom][0]
    d = summary["kernels"][dom_k]
    json.dump({"tag": tag, "kernel": dom_k, "kernel_stage": d["stage"], "batch_images": batch,
               "hbm_bytes_per_launch": d["hbm_bytes"], "avg_ns": d.get("avg_ns")},
              open(os.path.join(out, "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
