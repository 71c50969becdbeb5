"""Diagnostics: the configure-time upload race behind round 2's intermittent cross-call mismatch.

configure() zeroes the per-cell FAST counts with hipMemset on the null stream.  The null stream is delayed by D ms
(ORBX_DEBUG_UPLOAD_DELAY_MS) right before that memset; the first call's FAST then runs on the extractor's
non-blocking side stream.  If configure does not wait for the memset (build with -DORBX_LEGACY_UPLOADS, the round-2
code), a memset that lands between FAST's count stores and the quadtree's reads zeroes cells and the level loses
keypoints.  The product build waits (init_done) and must show 0 mismatches at every D.

  ORBX_LIB=build/legacy/liborbx.so python scripts/diag/upload_race.py [d_max_ms] [steps] [reps]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import multiagent_orb_slam2_amd as pkg  # noqa: E402
from multiagent_orb_slam2_amd import synthetic as S  # noqa: E402

d_max = float(sys.argv[1]) if len(sys.argv) > 1 else 0.4
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 41
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
print(f"library: {pkg.orbx.LIB_PATH}", flush=True)
batch = np.stack([S.kitti_like_image(600 + i) for i in range(3)])
ex1 = pkg.ORBextractor(2000, 1.2, 8, 20, 7)
ref = [ex1(batch[i]) for i in range(len(batch))]
t = torch.from_numpy(batch).cuda()
s_in, s_out = torch.cuda.Stream(), torch.cuda.Stream()
torch.cuda.synchronize()
bad_cfg = 0
total = 0
for k in range(steps):
    d = d_max * k / max(steps - 1, 1)
    for r in range(reps):
        os.environ["ORBX_DEBUG_UPLOAD_DELAY_MS"] = f"{d:.4f}"
        ex = pkg.ORBextractor(2000, 1.2, 8, 20, 7)
        ex.reserve(batch.shape[1], batch.shape[2], len(batch))
        kps, desc, cnt = ex.extract_batch_device(t, stream=s_in, out_stream=s_out)
        torch.cuda.synchronize()
        kps, desc, cnt = kps.cpu().numpy(), desc.cpu().numpy(), cnt.cpu().numpy()
        msgs = []
        for i, (k1, d1) in enumerate(ref):
            n = int(cnt[i])
            kb = kps[i, :n].copy().view(pkg.KP_DTYPE).reshape(-1)
            if n != len(k1) or not (np.array_equal(kb, k1) and np.array_equal(desc[i, :n], d1)):
                go = np.bincount(kb["octave"], minlength=8).tolist()
                ro = np.bincount(k1["octave"], minlength=8).tolist()
                msgs.append(f"image {i}: n {n} vs {len(k1)}, per level gpu {go} ref {ro}")
        total += 1
        if msgs:
            bad_cfg += 1
            print(f"delay {d:.4f} ms rep {r}: " + "; ".join(msgs), flush=True)
        del ex
os.environ.pop("ORBX_DEBUG_UPLOAD_DELAY_MS", None)
print(f"done: {bad_cfg} of {total} first calls differ from the host API", flush=True)
