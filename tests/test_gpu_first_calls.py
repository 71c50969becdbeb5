"""First calls racing: a stereo Frame's two extractors are first used by two threads at the same moment
(src/Frame.cc:78-81 on the first frame of a sequence), and agents start their Tracking threads together.  A fresh
extractor configures itself (device synchronisation, uploads) and captures its host-call graph on its first call; one
thread's configuration must not break another thread's capture, and no extractor may be left unusable.  Every
result equals a warm single-threaded extraction, on the first call and on the calls after it."""
import threading

import numpy as np
import pytest

from multiagent_orb_slam2_amd import synthetic as S

pytestmark = pytest.mark.gpu


def test_fresh_extractors_first_calls_concurrent(gpu):
    import multiagent_orb_slam2_amd as pkg
    imgs = [S.kitti_like_image(80 + i) for i in range(2)] + [S.kitti_like_image(82, rows=480, cols=752)]
    warm = {}
    for i, im in enumerate(imgs):
        warm[i] = pkg.ORBextractor(2000, 1.2, 8, 20, 7)(im)
    nthreads, trials = 6, 5
    for trial in range(trials):
        exs = [pkg.ORBextractor(2000, 1.2, 8, 20, 7) for _ in range(nthreads)]
        bar = threading.Barrier(nthreads)
        out, errs = [None] * nthreads, []

        def run(t):
            try:
                bar.wait()
                first = exs[t](imgs[t % 3])
                second = exs[t](imgs[t % 3])
                out[t] = (first, second)
            except Exception as e:                      # noqa: BLE001 -- reported below
                errs.append(f"thread {t}: {e}")
        th = [threading.Thread(target=run, args=(t,)) for t in range(nthreads)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errs, (trial, errs)
        for t in range(nthreads):
            (k1, d1), (k2, d2) = out[t]
            wk, wd = warm[t % 3]
            assert np.array_equal(k1, wk) and np.array_equal(d1, wd), (trial, t, "first call")
            assert np.array_equal(k2, wk) and np.array_equal(d2, wd), (trial, t, "second call")


def test_first_call_beside_foreign_device_syncs(gpu):
    """A caller's own code synchronising the device (torch.cuda.synchronize on another thread, which liborbx's lock
    cannot order) while an extractor captures its first call: the capture may be invalidated, and then the call falls
    back to per-call stream operations -- its results, and every later call's, still equal a warm extractor's."""
    import torch

    import multiagent_orb_slam2_amd as pkg
    img = S.kitti_like_image(90)
    wk, wd = pkg.ORBextractor(2000, 1.2, 8, 20, 7)(img)
    for trial in range(6):
        ex = pkg.ORBextractor(2000, 1.2, 8, 20, 7)
        stop = threading.Event()
        errs = []

        def spin():
            try:
                while not stop.is_set():
                    torch.cuda.synchronize()
            except Exception as e:                      # noqa: BLE001 -- a foreign sync refused during a capture
                errs.append(str(e))
        t = threading.Thread(target=spin)
        t.start()
        try:
            res = [ex(img) for _ in range(3)]
        finally:
            stop.set()
            t.join()
        for i, (k, d) in enumerate(res):
            assert np.array_equal(k, wk) and np.array_equal(d, wd), (trial, i)
    torch.cuda.synchronize()
