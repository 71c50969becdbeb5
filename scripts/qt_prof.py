#!/usr/bin/env python3
"""k_quadtree stage stamps (diagnostics build, `make qtprof`): one bench-size batch, then the wall-clock stamps of the
level-0 workgroup of image 0 (row 0) and the level-1 workgroup of image 0 (row 1).  100 MHz wall clock."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import multiagent_orb_slam2_amd as pkg  # noqa: E402
from multiagent_orb_slam2_amd import orbx  # noqa: E402
from multiagent_orb_slam2_amd import synthetic as S  # noqa: E402

lib = orbx.load_library(os.path.join(ROOT, "build/qtprof/liborbx.so"))
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dev = torch.device("cuda", 0)
lefts = [S.kitti_like_image(s, rows=375, cols=1242) for s in range(8)]
host = np.stack([lefts[i % 8] for i in range(2 * B)])
imgs = torch.from_numpy(host).to(dev)
ex = pkg.ORBextractor(2000, 1.2, 8, 20, 7, device=0)
ex.reserve(375, 1242, 2 * B)
cap = ex.max_keypoints(375, 1242)
kps = torch.empty((2 * B, cap, 28), dtype=torch.uint8, device=dev)
desc = torch.empty((2 * B, cap, 32), dtype=torch.uint8, device=dev)
cnt = torch.empty((2 * B,), dtype=torch.int32, device=dev)
s = torch.cuda.current_stream(dev)
for _ in range(3):
    ex.extract_batch_device(imgs, kps, desc, cnt, stream=s)
torch.cuda.synchronize()
buf = (C.c_ulonglong * 160)()
assert lib.orbx_debug_qt_prof(buf) == 0
for row in range(2):
    v = list(buf)[64 * row: 64 * row + 64]
    t0 = v[0]
    out = []
    for i in range(32):
        t, tag = v[2 * i], v[2 * i + 1]
        if t == 0:
            break
        out.append(f"{tag}:{(t - t0) / 100:.1f}")
    print(("level0 " if row == 0 else "level1 ") + " ".join(out))
for row in range(2):
    v = list(buf)[128 + 16 * row: 128 + 16 * row + 16]
    print(("fast band l0 " if row == 0 else "fast band l1+ ") + " ".join(f"{k}:{(v[k] - v[0]) / 100:.1f}" for k in range(6)),
          "survivors", v[8], "of", v[9])
