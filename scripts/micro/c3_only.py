"""The bench's C3 block alone (bench.c3_bench): python3 scripts/micro/c3_only.py [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import multiagent_orb_slam2_amd as pkg  # noqa: E402

dev = torch.device("cuda", 0)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 1):
    r = bench.c3_bench(pkg, dev)
    print(json.dumps({**{k: (v.get("us_per_launch"), v.get("us_per_launch_windows")) for k, v in r.items() if isinstance(v, dict) and "us_per_launch" in v}, "mfma_equals_tile": r.get("mfma_equals_tile")}))
