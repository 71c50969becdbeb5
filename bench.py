#!/usr/bin/env python3
"""bench.py — frames/s of the ORB stereo front-end (extract L + extract R + stereo L<->R Hamming match)
at KITTI size 1242x375, 8 levels, 2000 keypoints, on 1..N MI355X (one agent per GPU).

A "step" = one batch of --batch synthetic stereo frames per GPU through the hot path:
  ORBextractor on 2*batch images (src/ORBextractor.cc:1043-1105)  +  the descriptor search of
  Frame::ComputeStereoMatches on batch pairs (src/Frame.cc:466-552)
and, when N > 1, the keyframe exchange: every rank's new keyframes (1 in 5 frames: keypoints +
descriptors) are all-gathered over RCCL into every rank's MapFusion store (src/MapFusion.cc:83-88
replaced by ncclAllGather).  Inputs are resident in HBM before the timed region; weak scaling.

Prints ONE JSON line on rank 0 (driver contract).  Run: python bench.py [--gpus N --steps K --warmup W]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "frames/sec ORB extract+match, KITTI 1242×375 @2000 kpts, 1/2/4/8 GPU"
ROWS, COLS, NFEAT, NLEV, SCALE, INI, MINTH = 375, 1242, 2000, 8, 1.2, 20, 7
BF, BASELINE_B = 386.1448, 0.537165          # KITTI stereo (Examples/Stereo/KITTI00-02.yaml)
HBM_PEAK_GBS = 8000.0                         # MI355X HBM3E peak (MI355X_MICROARCH.md)
KF_EVERY = 5


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64, help="stereo frames per GPU per step")
    ap.add_argument("--distinct", type=int, default=16, help="distinct synthetic stereo pairs (tiled to batch)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget (0 = skip)")
    ap.add_argument("--no-timing", action="store_true", help="skip per-stage event timing")
    return ap.parse_args()


def level_pixels():
    from multiagent_orb_slam2_amd.orbx import load_library  # noqa: F401  (geometry comes from the extractor)
    return None


def algorithmic_bytes(ex, mean_cand, mean_kps):
    """Compulsory HBM bytes per image for each stage."""
    sizes = ex.level_sizes(ROWS, COLS)
    px = [h * w for h, w in sizes]
    P = sum(px)
    return {
        "resize": sum(px[l - 1] + px[l] for l in range(1, len(px))),
        "fast_cells": P + 5 * mean_cand,                 # read every level once, write candidates (xy + score)
        "blur7": 2 * P,                                  # read + write every level
        "quadtree": 2 * 5 * mean_cand + 5 * mean_kps,     # read slots, write compacted keys, write kept keys
        "describe": mean_kps * (749 + 512 + 28 + 32 + 5),  # IC disc + 512 BRIEF samples + outputs
    }


def cpu_baseline(lefts, rights, scale, seconds):
    from oracle import oracle as O
    t0 = time.perf_counter()
    n = 0
    i = 0
    while True:
        l, r = lefts[i % len(lefts)], rights[i % len(rights)]
        a = O.extract(l, nfeatures=NFEAT)
        b = O.extract(r, nfeatures=NFEAT)
        O.stereo_match(a["kps"], a["desc"], b["kps"], b["desc"], scale, ROWS, BF, BASELINE_B)
        n += 1
        i += 1
        el = time.perf_counter() - t0
        if el >= seconds and n >= 3:
            break
    return n / el, n, el


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import multiagent_orb_slam2_amd as pkg
    from multiagent_orb_slam2_amd import synthetic as S

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    B = args.batch
    nd = min(args.distinct, B)
    lefts = [S.kitti_like_image(1000 * rank + i) for i in range(nd)]
    rights = [S.shifted_right_view(l, 1000 * rank + i) for i, l in enumerate(lefts)]
    host = np.stack([lefts[i % nd] for i in range(B)] + [rights[i % nd] for i in range(B)])
    imgs = torch.from_numpy(host).to(dev)               # resident in HBM before timing

    ex = pkg.ORBextractor(NFEAT, SCALE, NLEV, INI, MINTH, device=dev.index)
    ex.reserve(ROWS, COLS, 2 * B)
    m = pkg.ORBmatcher(0.6, True, device=dev.index)
    scale = ex.GetScaleFactors()
    cap = ex.max_keypoints(ROWS, COLS)
    kps = torch.empty((2 * B, cap, 28), dtype=torch.uint8, device=dev)
    desc = torch.empty((2 * B, cap, 32), dtype=torch.uint8, device=dev)
    cnt = torch.empty((2 * B,), dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(dev)                    # one queue for extractor, matcher and RCCL
    torch.cuda.set_stream(stream)
    n_kf = max(1, B // KF_EVERY)
    kf_local = torch.empty((n_kf, cap, 60), dtype=torch.uint8, device=dev)
    kf_all = torch.empty((world * n_kf, cap, 60), dtype=torch.uint8, device=dev) if world > 1 else None

    stereo_ms = []

    def step(time_stereo=False):
        ex.extract_batch_device(imgs, kps, desc, cnt, stream=stream)
        if time_stereo:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        bi, bd = m.stereo_match_batch_device(kps[:B], desc[:B], cnt[:B], kps[B:], desc[B:], cnt[B:], cap, scale,
                                             ROWS, BF, BASELINE_B, stream=stream)
        if time_stereo:
            e1.record(stream)
            stereo_ms.append((e0, e1))
        if world > 1:
            # keyframe packets (keypoints 28 B + descriptors 32 B per slot) -> all ranks (MapFusion ingress)
            kf_local[:, :, :28].copy_(kps[0:B:KF_EVERY][:n_kf])
            kf_local[:, :, 28:].copy_(desc[0:B:KF_EVERY][:n_kf])
            dist.all_gather_into_tensor(kf_all, kf_local)
        return bi, bd

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if not args.no_timing:
        ex.enable_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(time_stereo=not args.no_timing)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    frames = B * args.steps * world
    value = frames / el
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1000 * el / args.steps, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": "C2+C3 stereo frame: ORBextractor x2 (1242x375, 8 levels, 2000 kpts) + stereo "
                               "L<->R 256-bit Hamming band match" + (" + RCCL all-gather of KF packets" if world > 1 else ""),
                   "global_batch": B * world, "frames_per_gpu_per_step": B, "image": [ROWS, COLS],
                   "nfeatures": NFEAT, "nlevels": NLEV, "parallelism": f"agent-per-gpu x{world}"},
    }

    if not args.no_timing:
        st, calls = ex.stage_times()
        per_call = {k: v / max(calls, 1) for k, v in st.items()}
        sms = [a.elapsed_time(b) for a, b in stereo_ms]
        per_call["stereo_match"] = float(np.mean(sms)) if sms else 0.0
        counts = cnt.cpu().numpy()
        mean_kps = float(counts.mean())
        mean_cand = float(mean_kps * 4)   # replaced below by the measured candidate count if available
        try:
            from oracle import oracle as O  # candidate count of the synthetic inputs (geometry only)
            mean_cand = float(np.mean([sum(len(c) for c in O.level_candidates(lefts[i])) for i in range(min(2, nd))]))
        except Exception:
            pass
        alg = algorithmic_bytes(ex, mean_cand, mean_kps)
        alg["stereo_match"] = 2 * cap * 0 + 2 * mean_kps * 60 + mean_kps * 8
        dom = max(per_call, key=per_call.get)
        n_units = 2 * B if dom != "stereo_match" else B
        bytes_launch = alg[dom] * n_units
        achieved = bytes_launch / (per_call[dom] * 1e-3) / 1e9
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc):
            try:
                d = json.load(open(pmc))
                if d.get("kernel_stage") == dom and d.get("batch_images") == n_units:
                    traffic = d.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        out["roofline"] = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic, "kernel": dom,
                           "kernel_ms_per_launch": round(per_call[dom], 4), "algorithmic_bytes_per_launch": bytes_launch}
        out["stage_ms_per_step"] = {k: round(v, 4) for k, v in per_call.items()}

    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        fps, n, secs = cpu_baseline(lefts, rights, scale, args.cpu_seconds)
        out["cpu_baseline"] = {"value": round(fps, 3), "unit": "frames/s", "cores": 1, "kind": "port",
                               "sample": f"{n} stereo frames (2 extractions + stereo match each) of the same synthetic "
                                         f"inputs, oracle/orb_oracle.cpp -O2, 1 thread, {secs:.1f} s"}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
