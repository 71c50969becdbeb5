#!/usr/bin/env python3
"""Throughput of the projection / radius matchers on one MI355X: B tracking frames per launch, each a
KITTI-size view (2000 keypoints, 1242x375) searched by Q projected MapPoints: the local-map search
(SearchByProjection(Frame&, vpMapPoints), src/ORBmatcher.cc:45-131, called by Tracking::SearchLocalPoints,
Tracking.cc:1204) and the motion-model search (SearchByProjection(Frame&, LastFrame), :1330-1472).
Synthetic cases from tests/proj_cases.py; grid build + search timed with HIP events on one stream.
Prints one JSON line."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def main():
    import torch

    import multiagent_orb_slam2_amd as pkg
    from proj_cases import MODES, make_case
    B = int(os.environ.get("BENCH_PROJ_B", "64"))
    Q = int(os.environ.get("BENCH_PROJ_Q", "4000"))
    dev = torch.device("cuda", 0)
    m = pkg.ORBmatcher(0.8, True)
    out = {}
    for name in ("mappoints", "lastframe"):
        base = [make_case(1000 + i, MODES[name], n_target=2000, n_query=Q, W=1242, H=375) for i in range(min(B, 8))]
        cases = [base[i % len(base)] for i in range(B)]
        cap = 2048
        kps = torch.zeros((B, cap, 28), dtype=torch.uint8)
        desc = torch.zeros((B, cap, 32), dtype=torch.uint8)
        ur = torch.full((B, cap), -1.0)
        bl = torch.zeros((B, cap), dtype=torch.uint8)
        qs = torch.zeros((B, Q, 40), dtype=torch.uint8)
        qd = torch.zeros((B, Q, 32), dtype=torch.uint8)
        for i, c in enumerate(cases):
            n = len(c["kps"])
            kps[i, :n] = torch.from_numpy(c["kps"].view(np.uint8).reshape(n, 28))
            desc[i, :n] = torch.from_numpy(c["desc"])
            ur[i, :n] = torch.from_numpy(c["uright"])
            bl[i, :n] = torch.from_numpy(c["blocked"])
            qs[i] = torch.from_numpy(c["queries"].view(np.uint8).reshape(Q, 40))
            qd[i] = torch.from_numpy(c["qdesc"])
        kps, desc, ur, bl, qs, qd = (t.to(dev) for t in (kps, desc, ur, bl, qs, qd))
        counts = torch.full((B,), 2000, dtype=torch.int32, device=dev)
        grid = cases[0]["grid"]
        cs = torch.empty((B, grid.cols * grid.rows + 1), dtype=torch.int32, device=dev)
        ci = torch.empty((B, cap), dtype=torch.int32, device=dev)
        q_idx = torch.empty((B, Q), dtype=torch.int32, device=dev)
        q_dist = torch.empty((B, Q), dtype=torch.int32, device=dev)
        owner = torch.empty((B, cap), dtype=torch.int32, device=dev)
        nm = torch.empty((B,), dtype=torch.int32, device=dev)
        probs = (pkg.ProjProblem * B)()
        for i in range(B):
            probs[i] = pkg.ProjProblem(qs[i].data_ptr(), qd[i].data_ptr(), Q, kps[i].data_ptr(), desc[i].data_ptr(),
                                       ur[i].data_ptr(), bl[i].data_ptr(), 2000, cs[i].data_ptr(), ci[i].data_ptr(),
                                       q_idx[i].data_ptr(), q_dist[i].data_ptr(), owner[i].data_ptr(),
                                       nm[i:i + 1].data_ptr())
        dprobs = torch.frombuffer(bytearray(bytes(probs)), dtype=torch.uint8).to(dev)
        params = cases[0]["params"]

        def run():
            m.grid_build_device(grid, kps, counts, out=(cs, ci))
            m.proj_search_batch_device(params, grid, dprobs, cap, Q)

        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        out[name] = {"ms_per_launch": round(ms, 4), "frames_per_launch": B, "queries_per_frame": Q,
                     "frames_per_s": round(B / (ms * 1e-3), 1), "queries_per_s": round(B * Q / (ms * 1e-3)),
                     "mean_nmatches": float(nm.float().mean())}
    print(json.dumps({"bench": "projection matchers (SearchByProjection local map / motion model)", "results": out}))


if __name__ == "__main__":
    main()
