"""Where the Python per-call path's time goes beyond the native one: timestamps around each part of a frame of
bench.host_api_rate's loop (python3 scripts/micro/host_api_py_prof.py [frames])."""
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
import multiagent_orb_slam2_amd as pkg  # noqa: E402
from multiagent_orb_slam2_amd import synthetic as S  # noqa: E402

cfg = bench.CONFIGS["kitti"]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
lefts = [S.kitti_like_image(s, rows=cfg["rows"], cols=cfg["cols"]) for s in range(8)]
rights = [S.shifted_right_view(l, s) for s, l in enumerate(lefts)]
ex_l = pkg.ORBextractor(cfg["nfeatures"], 1.2, 8, 20, 7)
ex_r = pkg.ORBextractor(cfg["nfeatures"], 1.2, 8, 20, 7)
m = pkg.ORBmatcher(0.75, True)
b = cfg["bf"] / cfg["fx"]
pool = ThreadPoolExecutor(1)
T = []
for i in range(n + 10):
    t0 = time.perf_counter()
    fr = pool.submit(ex_r, rights[i % 8])
    t1 = time.perf_counter()
    kl, dl = ex_l(lefts[i % 8])
    t2 = time.perf_counter()
    kr, dr = fr.result()
    t3 = time.perf_counter()
    m.ComputeStereoMatches(ex_l, ex_r, kl, dl, kr, dr, cfg["bf"], b)
    t4 = time.perf_counter()
    if i >= 10:
        T.append((t1 - t0, t2 - t1, t3 - t2, t4 - t3, t4 - t0))
T = np.array(T) * 1e3
print("median ms: submit %.3f  left %.3f  wait-right %.3f  stereo %.3f  frame %.3f" % tuple(np.median(T, axis=0)))
# the same calls in sequence on one thread, and the bare ctypes extraction alone
T2 = []
for i in range(n):
    t0 = time.perf_counter()
    ex_l(lefts[i % 8])
    t1 = time.perf_counter()
    ex_r(rights[i % 8])
    t2 = time.perf_counter()
    T2.append((t1 - t0, t2 - t1))
print("sequential median ms: left %.3f right %.3f" % tuple(np.median(np.array(T2) * 1e3, axis=0)))
import ctypes as C  # noqa: E402
lib = pkg.orbx.load_library()
img = lefts[0]
cap = ex_l.max_keypoints(*img.shape)
kp = np.empty(cap, pkg.KP_DTYPE)
ds = np.empty((cap, 32), np.uint8)
nn = C.c_int()
T3 = []
for i in range(n):
    t0 = time.perf_counter()
    lib.orbx_extract(ex_l._h, img.ctypes.data, img.shape[0], img.shape[1], img.strides[0], kp.ctypes.data, ds.ctypes.data, cap,
                     C.byref(nn))
    T3.append(time.perf_counter() - t0)
print("bare ctypes orbx_extract median ms: %.3f" % (np.median(T3) * 1e3))
