"""The bench's Python per-call block alone (bench.host_api_rate): python3 scripts/micro/host_api_py.py [frames] [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
import multiagent_orb_slam2_amd as pkg  # noqa: E402
from multiagent_orb_slam2_amd import synthetic as S  # noqa: E402

cfg = bench.CONFIGS["kitti"]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
lefts = [S.kitti_like_image(s, rows=cfg["rows"], cols=cfg["cols"]) for s in range(8)]
rights = [S.shifted_right_view(l, s) for s, l in enumerate(lefts)]
for _ in range(reps):
    r = bench.host_api_rate(pkg, cfg, lefts, rights, n, 0)
    r.pop("path", None)
    nat = r.pop("native", {})
    print(json.dumps(r), "native", nat.get("frames_per_s"), nat.get("frame_ms"), nat.get("slowest"), flush=True)
