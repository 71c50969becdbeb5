"""Teardown with work still queued on another stream (the r3w fault).

The extractor's pyramid ring is read by the stereo SAD step on the caller's stereo stream
(orbx_stereo_refine_batch_device over orbx_extractor_pyramid_device).  Destroying the extractor while that stream
still has the step queued must not free the ring under it: every destroy path drains the whole device first (hipFree
was measured to wait for other streams' kernels too, scripts/micro/free_sync.hip, but the guarantee should not rest
on that runtime behaviour).  Afterwards the device must hold no
pending error, and a fresh process must initialise the GPU and extract bit-exactly -- the r3w symptom was a fresh
process failing its first HIP call after the previous process's teardown."""
import os
import subprocess
import sys
import time

import numpy as np
import pytest

from multiagent_orb_slam2_amd import synthetic as S

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import sys
sys.path.insert(0, sys.argv[1])
import numpy as np
import multiagent_orb_slam2_amd as pkg
from multiagent_orb_slam2_amd import synthetic as S
from oracle import oracle as O
img = S.kitti_like_image(77, rows=240, cols=320)
ex = pkg.ORBextractor(500, 1.2, 8, 20, 7, device=0)
k, d = ex(img)
ref = O.extract(img, nfeatures=500)
assert np.array_equal(k, ref["kps"]) and np.array_equal(d, ref["desc"])
ex.close()
pkg.orbx.device_check(0)
print("child ok", len(k))
"""


def test_destroy_with_stereo_step_queued_then_fresh_process(gpu):
    import torch

    import multiagent_orb_slam2_amd as pkg
    B = 4
    lefts = [S.kitti_like_image(60 + i) for i in range(B)]
    rights = [S.shifted_right_view(l, 60 + i) for i, l in enumerate(lefts)]
    imgs = torch.from_numpy(np.stack(lefts + rights)).cuda()
    ex = pkg.ORBextractor(2000, 1.2, 8, 20, 7)
    m = pkg.ORBmatcher(0.6, True)
    s_front, s_stereo = torch.cuda.Stream(), torch.cuda.Stream()
    kps, desc, cnt = ex.extract_batch_device(imgs, stream=s_front)
    cap = kps.shape[1]
    done = torch.cuda.Event()
    done.record(s_front)
    s_stereo.wait_event(done)
    pyr = ex.pyramid_device()
    pkg.orbx.debug_spin(s_stereo, 150.0)            # the stereo step starts 150 ms from now
    with torch.cuda.stream(s_stereo):
        bi, _ = m.stereo_match_batch_device(kps[:B], desc[:B], cnt[:B], kps[B:], desc[B:], cnt[B:], cap,
                                            ex.GetScaleFactors(), 375, 386.1448, 0.5372, stream=s_stereo)
        ur, depth = m.stereo_refine_batch_device(kps[:B], cnt[:B], kps[B:], bi, pyr, 0, pyr, B, 386.1448, 0.5372,
                                                 stream=s_stereo)
    t0 = time.perf_counter()
    ex.close()                                       # the SAD step on s_stereo still has to read the pyramid ring
    waited_ms = 1e3 * (time.perf_counter() - t0)
    torch.cuda.synchronize()
    pkg.orbx.device_check(0)
    m.close()
    assert waited_ms > 100.0, f"destroy returned after {waited_ms:.1f} ms with the stereo step still queued"
    assert int((depth > 0).sum().item()) > 0
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "child ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
