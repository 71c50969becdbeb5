"""Diagnostics: orbx_extract_batch_device_split calls back to back (describe on a second stream), repeated; reports
which call / image / field differs from the host API.  python scripts/diag/split_race.py [iters] [ring]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import multiagent_orb_slam2_amd as pkg  # noqa: E402
from multiagent_orb_slam2_amd import synthetic as S  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
ring = int(sys.argv[2]) if len(sys.argv) > 2 else 2
batches = [np.stack([S.kitti_like_image(300 + 7 * b + i) for i in range(3)]) for b in range(4)]
ex1 = pkg.ORBextractor(2000, 1.2, 8, 20, 7)
ref = [[ex1(b[i]) for i in range(len(b))] for b in batches]
ts = [torch.from_numpy(b).cuda() for b in batches]
bad = 0
for it in range(iters):
    ex = pkg.ORBextractor(2000, 1.2, 8, 20, 7)
    ex.set_pyramid_ring(ring)
    s_in, s_out = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    outs = [ex.extract_batch_device(t, stream=s_in, out_stream=s_out) for t in ts]
    torch.cuda.synchronize()
    for bi, (kps, desc, cnt) in enumerate(outs):
        kps, desc, cnt = kps.cpu().numpy(), desc.cpu().numpy(), cnt.cpu().numpy()
        for i in range(3):
            k1, d1 = ref[bi][i]
            n = int(cnt[i])
            kb = kps[i, :n].copy().view(pkg.KP_DTYPE).reshape(-1)
            if n != len(k1) or not np.array_equal(kb, k1) or not np.array_equal(desc[i, :n], d1):
                bad += 1
                msg = f"iter {it} call {bi} image {i}: n {n} vs {len(k1)}"
                if n == len(k1):
                    for f in kb.dtype.names:
                        d = np.nonzero(kb[f] != k1[f])[0]
                        if len(d):
                            msg += f"; {f}: {len(d)} differ (first {d[0]})"
                    dd = np.nonzero((desc[i, :n] != d1).any(1))[0]
                    if len(dd):
                        msg += f"; desc rows {len(dd)}"
                else:
                    go = np.bincount(kb["octave"], minlength=8)
                    ro = np.bincount(k1["octave"], minlength=8)
                    msg += f"; per level gpu {go.tolist()} ref {ro.tolist()}"
                print(msg, flush=True)
    del ex
print(f"done: {bad} mismatching images over {iters} iterations", flush=True)
