#!/usr/bin/env python3
"""Kernel shares of a profiled bench command -> profiles/kernel_share.json (read by bench.py to pick the dominant
kernel of its roofline line).

  python scripts/kernel_share.py <run_kernel_trace.csv> <tag> <timed_steps_in_trace> [--out profiles/kernel_share.json]

Per kernel name: launches, total / average duration, share of all kernel time, launches and milliseconds per step
(per step = trace total / steps traced, every launch of the run counted: warmup and setup steps run the same
kernels), the per-grid breakdown (a kernel launched with two grids, e.g. k_fast_wave's level-0 and levels-1..7
launches, which run on two streams and overlap each other), and busy_ms_per_step: the union of the kernel's launch
intervals (the wall time during which it runs), which is what bench.py's roofline divides by.  The traced command must
run the bench steps only (scripts/prof_r4.sh: --alone-reps 0 and every side block off), so launches_per_step is exact.
source_sha16 = hash of the HIP sources the trace was taken with (bench.py compares it to the tree)."""
import argparse
import collections
import csv
import hashlib
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def source_sha16(root=ROOT):
    h = hashlib.sha256()
    for p in sorted(glob.glob(os.path.join(root, "multiagent_orb_slam2_amd", "csrc", "*.hip")) +
                    glob.glob(os.path.join(root, "multiagent_orb_slam2_amd", "csrc", "*.h"))):
        h.update(os.path.basename(p).encode())
        h.update(open(p, "rb").read())
    return h.hexdigest()[:16]


def short(name):
    n = name.split("(")[0].replace("void ", "").strip()
    return n.split("::")[-1]


def union_ns(iv):
    """Total length of the union of [start, end] intervals."""
    tot, cur_s, cur_e = 0, None, None
    for a, b in sorted(iv):
        if cur_e is None or a > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = a, b
        else:
            cur_e = max(cur_e, b)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("tag")
    ap.add_argument("steps", type=int, help="bench steps in the traced run (setup + warmup + timed)")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "kernel_share.json"))
    ap.add_argument("--config", default="kitti")
    ap.add_argument("--batch-images", type=int, default=256)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    per = collections.defaultdict(list)
    ivs = collections.defaultdict(list)
    grids = collections.defaultdict(list)
    for r in rows:
        n = short(r["Kernel_Name"])
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        per[n].append(d)
        ivs[n].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        grids[(n, int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1) * int(r.get("Grid_Size_Z", 1) or 1))].append(d)
    tot = sum(sum(v) for v in per.values())
    ks = []
    for n, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        g = [{"grid": gg, "launches": len(d), "avg_us": round(sum(d) / len(d) / 1e3, 2)}
             for (nn, gg), d in sorted(grids.items(), key=lambda kv: -sum(kv[1])) if nn == n]
        ks.append({"kernel": n, "launches": len(v), "total_ms": round(sum(v) / 1e6, 3), "avg_us": round(sum(v) / len(v) / 1e3, 2),
                   "pct": round(100.0 * sum(v) / tot, 2), "launches_per_step": round(len(v) / a.steps, 2),
                   "ms_per_step": round(sum(v) / a.steps / 1e6, 4),
                   "busy_ms_per_step": round(union_ns(ivs[n]) / a.steps / 1e6, 4), "grids": g})
    t0 = min(int(r["Start_Timestamp"]) for r in rows) if rows else 0
    t1 = max(int(r["End_Timestamp"]) for r in rows) if rows else 0
    out = {"tag": a.tag, "config": a.config, "batch_images": a.batch_images, "steps_traced": a.steps,
           "source_sha16": source_sha16(), "trace": os.path.relpath(a.trace, ROOT),
           "dominant": ks[0]["kernel"] if ks else None, "kernel_ms_per_step_total": round(tot / a.steps / 1e6, 4),
           "trace_span_ms_per_step": round((t1 - t0) / a.steps / 1e6, 4),
           "gpu_busy_ms_per_step": round(union_ns([iv for v in ivs.values() for iv in v]) / a.steps / 1e6, 4),
           "kernels": ks}
    json.dump(out, open(a.out, "w"), indent=1)
    print(f"{a.out}: dominant {out['dominant']} ({ks[0]['pct']} %), {len(ks)} kernels, sha {out['source_sha16']}")


if __name__ == "__main__":
    main()
