"""Frame::UndistortKeyPoints / ComputeImageBounds (src/Frame.cc:404-464): the oracle's restatement of OpenCV 3.2
cvUndistortPoints against an independent numpy float64 restatement (bit-exact) and against the forward distortion
model (round trip), and the HIP kernel bit-exact against the oracle.  The arithmetic of cv::undistortPoints is
OpenCV's (not vendored in the reference): parity unpinned beyond the restated 3.2 semantics."""
import numpy as np
import pytest
import torch

from multiagent_orb_slam2_amd.orbx import KP_DTYPE
from oracle import oracle as O

# Examples/Monocular/TUM1.yaml:8-17 and EuRoC.yaml:8-16 (k1 k2 p1 p2 [k3])
TUM1 = (np.array([[517.306408, 0, 318.643040], [0, 516.469215, 255.313989], [0, 0, 1]], np.float32),
        np.array([0.262383, -0.953104, -0.005358, 0.002628, 1.163314], np.float32), (640, 480))
EUROC = (np.array([[458.654, 0, 367.215], [0, 457.296, 248.375], [0, 0, 1]], np.float32),
         np.array([-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05], np.float32), (752, 480))


def numpy_undistort(xy, K, d):
    k = np.zeros(14)
    k[:len(d)] = d.astype(np.float64)
    fx, fy, cx, cy = float(K[0, 0]), float(K[1, 1]), float(K[0, 2]), float(K[1, 2])
    x = (xy[:, 0].astype(np.float64) - cx) * (1.0 / fx)
    y = (xy[:, 1].astype(np.float64) - cy) * (1.0 / fy)
    x0, y0 = x.copy(), y.copy()
    for _ in range(5):
        r2 = x * x + y * y
        icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2)
        dx = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2
        dy = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2
        x = (x0 - dx) * icdist
        y = (y0 - dy) * icdist
    R = K.astype(np.float64)
    xx = R[0, 0] * x + R[0, 1] * y + R[0, 2]
    yy = R[1, 0] * x + R[1, 1] * y + R[1, 2]
    ww = 1.0 / (R[2, 0] * x + R[2, 1] * y + R[2, 2])
    return np.stack([(xx * ww).astype(np.float32), (yy * ww).astype(np.float32)], 1)


def distort(xy, K, d):
    k = np.zeros(5)
    k[:len(d)] = d
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    x, y = (xy[:, 0] - cx) / fx, (xy[:, 1] - cy) / fy
    r2 = x * x + y * y
    rad = 1 + k[0] * r2 + k[1] * r2 * r2 + k[4] * r2 ** 3
    xd = x * rad + 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x)
    yd = y * rad + k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y
    return np.stack([xd * fx + cx, yd * fy + cy], 1)


def _points(seed, w, h, n=3000):
    rng = np.random.default_rng(seed)
    return np.stack([rng.uniform(0, w, n), rng.uniform(0, h, n)], 1).astype(np.float32)


@pytest.mark.parametrize("cam", [TUM1, EUROC])
def test_oracle_matches_numpy_and_inverts_distortion(cam):
    K, d, (w, h) = cam
    xy = _points(1, w, h)
    un = O.undistort_points(xy, K, d)
    assert np.array_equal(un.view(np.uint32), numpy_undistort(xy, K, d).view(np.uint32))
    # five fixed-point iterations invert the distortion model near the centre (the reference's approximation)
    c = np.hypot(xy[:, 0] - K[0, 2], xy[:, 1] - K[1, 2]) < 0.3 * min(w, h)
    back = distort(un[c].astype(np.float64), K.astype(np.float64), d.astype(np.float64))
    assert np.max(np.abs(back - xy[c])) < 0.05


def test_oracle_zero_k1_copies():
    xy = _points(2, 100, 100, 50)
    assert np.array_equal(O.undistort_points(xy, TUM1[0], np.zeros(4, np.float32)), xy)


@pytest.mark.gpu
@pytest.mark.parametrize("cam", [TUM1, EUROC])
def test_gpu_undistort_bit_exact(gpu, cam):
    import multiagent_orb_slam2_amd as pkg
    K, d, (w, h) = cam
    m = pkg.ORBmatcher()
    xy = _points(3, w, h, 2500)
    kps = np.zeros(len(xy), KP_DTYPE)
    kps["x"], kps["y"], kps["octave"], kps["angle"] = xy[:, 0], xy[:, 1], np.arange(len(xy)) % 8, 12.5
    ref = O.undistort_points(xy, K, d)
    got = m.UndistortKeyPoints(kps, K, d)
    assert np.array_equal(np.stack([got["x"], got["y"]], 1).view(np.uint32), ref.view(np.uint32))
    assert np.array_equal(got["octave"], kps["octave"]) and np.array_equal(got["angle"], kps["angle"])
    # device batch form over an extractor-like layout (two sets, ragged counts)
    dev = torch.device("cuda", 0)
    cap = 2600
    batch = np.zeros((2, cap), KP_DTYPE)
    batch[0, :2500], batch[1, :1000] = kps, kps[:1000]
    counts = torch.tensor([2500, 1000], dtype=torch.int32, device=dev)
    dk = torch.from_numpy(batch.view(np.uint8).reshape(2, cap, 28)).to(dev)
    out = m.undistort_keypoints_device(dk, counts, K, d).cpu().numpy().view(KP_DTYPE).reshape(2, cap)
    assert np.array_equal(out[0, :2500].view(np.uint8), got.view(np.uint8))
    assert np.array_equal(out[1, :1000].view(np.uint8), got[:1000].view(np.uint8))
    # ComputeImageBounds: undistorted corners
    b = m.ComputeImageBounds(K, d, w, h)
    cu = O.undistort_points(np.array([[0, 0], [w, 0], [0, h], [w, h]], np.float32), K, d)
    assert b == (min(cu[0, 0], cu[2, 0]), max(cu[1, 0], cu[3, 0]), min(cu[0, 1], cu[1, 1]), max(cu[2, 1], cu[3, 1]))
    assert m.ComputeImageBounds(K, np.zeros(4, np.float32), w, h) == (0.0, float(w), 0.0, float(h))
