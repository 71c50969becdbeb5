"""CPU tests of the oracle (test infrastructure): known answers derived from the reference source,
independent numpy restatements, and the committed regression fixtures.

Parity status of the oracle: "parity unpinned" — the reference is not buildable here (OpenCV absent)
and has no tests or golden vectors for this path; see DESIGN.md §Oracle."""
import hashlib
import json
import math
import os

import numpy as np
import pytest

from multiagent_orb_slam2_amd import synthetic as S
from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_tables_known_answers():
    """ORBextractor ctor (src/ORBextractor.cc:410-470) at nfeatures 2000, 1.2, 8 levels."""
    t = O.tables()
    assert t["n_per_level"].tolist() == [434, 362, 302, 251, 209, 175, 145, 122]
    assert t["umax"].tolist() == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]
    assert np.allclose(t["scale"], [1.2 ** i for i in range(8)], rtol=1e-6)
    assert t["scale"].dtype == np.float32
    assert O.tables(nfeatures=1000)["n_per_level"].sum() == 1000


def test_level_geometry_known_answers():
    sizes = O.level_sizes(375, 1242)
    assert [(w, h) for h, w in sizes] == [(1242, 375), (1035, 312), (862, 260), (719, 217), (599, 181), (499, 151),
                                          (416, 126), (347, 105)]
    assert sum(h * w for h, w in sizes) == 1441432


def test_gaussian_taps_and_blur_constant():
    # taps {18,34,49,55,49,34,18} sum 257: a constant 100 image blurs to round(100*257^2/2^16)
    img = np.full((20, 30), 100, np.uint8)
    out = O.blur7(img)
    assert (out == ((100 * 257 * 257 + (1 << 15)) >> 16)).all()
    assert (O.blur7(np.full((9, 9), 255, np.uint8)) == 255).all()   # saturates


def test_blur_matches_numpy_restatement():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (23, 41), dtype=np.uint8)
    taps = np.array([18, 34, 49, 55, 49, 34, 18], np.int64)
    pad = np.pad(img.astype(np.int64), 3, mode="reflect")   # numpy 'reflect' == BORDER_REFLECT_101
    rows = sum(taps[k] * pad[:, k:k + img.shape[1]] for k in range(7))
    acc = sum(taps[k] * rows[k:k + img.shape[0], :] for k in range(7))
    ref = np.clip((acc + (1 << 15)) >> 16, 0, 255).astype(np.uint8)
    assert np.array_equal(O.blur7(img), ref)


def test_resize_constant_and_shape():
    img = np.full((375, 1242), 77, np.uint8)
    out = O.resize(img, 312, 1035)
    assert out.shape == (312, 1035) and (out == 77).all()


def test_resize_matches_numpy_restatement():
    rng = np.random.default_rng(1)
    src = rng.integers(0, 256, (50, 61), dtype=np.uint8)
    dh, dw = 42, 51
    sx, sy = 1.0 / (dw / 61), 1.0 / (dh / 50)

    def taps(n_dst, n_src, sc):
        i0, i1, a0, a1 = [], [], [], []
        for d in range(n_dst):
            f = np.float32((d + 0.5) * sc - 0.5)
            i = math.floor(f)
            f = np.float32(f - np.float32(i))
            if i < 0:
                f, i = np.float32(0), 0
            if i >= n_src - 1:
                f, i = np.float32(0), n_src - 1
            i0.append(i)
            i1.append(min(i + 1, n_src - 1))
            a0.append(int(np.rint(np.float32(np.float32(1) - f) * np.float32(2048))))
            a1.append(int(np.rint(f * np.float32(2048))))
        return map(np.array, (i0, i1, a0, a1))

    x0, x1, ax0, ax1 = taps(dw, 61, sx)
    y0, y1, by0, by1 = taps(dh, 50, sy)
    S_ = src.astype(np.int64)
    h = S_[:, x0] * ax0 + S_[:, x1] * ax1
    v = (h[y0] * by0[:, None] + h[y1] * by1[:, None] + (1 << 21)) >> 22
    assert np.array_equal(O.resize(src, dh, dw), np.clip(v, 0, 255).astype(np.uint8))


@pytest.mark.parametrize("y,x", [(0, 1), (1, 0), (1, 1), (-1, 1), (1, -1), (-1, -1), (3, -7), (-5, 2), (0, 0), (0, -2)])
def test_fast_atan2_close_to_atan2(y, x):
    a = O.fast_atan2(y, x)
    ref = math.degrees(math.atan2(y, x)) % 360
    assert 0 <= a < 360.0001
    assert abs((a - ref + 180) % 360 - 180) < 0.02 or (x == 0 and y == 0)


def test_descriptor_distance_is_popcount():
    a, b = S.random_descriptors(3, 200), S.random_descriptors(4, 200)
    ref = np.unpackbits(a ^ b, axis=1).sum(axis=1)
    assert all(O.descriptor_distance(a[i], b[i]) == ref[i] for i in range(200))


def test_bf_match_matches_numpy():
    q, t = S.planted_pairs(5, 300, 400)
    bi, b1, b2 = O.bf_match(q, t)
    D = np.unpackbits(q[:, None, :] ^ t[None, :, :], axis=2).sum(axis=2)
    assert np.array_equal(b1, D.min(axis=1))
    assert np.array_equal(bi, D.argmin(axis=1))          # first minimum
    s = np.sort(D, axis=1)
    assert np.array_equal(b2, s[:, 1])


def test_stereo_matches_bruteforce_python():
    ex = O.extract(S.kitti_like_image(12, rows=200, cols=400), nfeatures=600)
    exr = O.extract(S.shifted_right_view(S.kitti_like_image(12, rows=200, cols=400), 12), nfeatures=600)
    kl, dl, kr, dr = ex["kps"], ex["desc"], exr["kps"], exr["desc"]
    scale = O.tables()["scale"]
    n, idx, dist = O.stereo_match(kl, dl, kr, dr, scale, 200, 386.1448, 0.537165)
    maxD = np.float32(386.1448) / np.float32(0.537165)
    for i in range(len(kl)):
        v = int(kl["y"][i])
        best, bi = 100, -1
        for r in range(len(kr)):
            rad = np.float32(2.0) * scale[kr["octave"][r]]
            if not (math.floor(kr["y"][r] - rad) <= v <= math.ceil(kr["y"][r] + rad)):
                continue
            if abs(int(kr["octave"][r]) - int(kl["octave"][i])) > 1:
                continue
            if not (kl["x"][i] - maxD <= kr["x"][r] <= kl["x"][i]):
                continue
            d = int(np.unpackbits(dl[i] ^ dr[r]).sum())
            if d < best:
                best, bi = d, r
        assert dist[i] == best and idx[i] == (bi if best < 75 else -1)


def test_model_fast_and_quadtree_equal_oracle():
    """The data-parallel formulations used by the HIP kernels (tests/gpu_model.py) reproduce the oracle's
    sequential restatement exactly, level by level."""
    import gpu_model as M
    t = O.tables()
    for seed in (0, 1):
        img = S.kitti_like_image(seed)
        pyr = O.extract(img, want_pyramid=True)["pyramid"]
        cands = O.level_candidates(img)
        for l, L in enumerate(pyr):
            assert np.array_equal(M.fast_candidates(L), cands[l])
            h, w = L.shape
            N = int(t["n_per_level"][l])
            ref = O.distribute(cands[l], 16, w - 16, 16, h - 16, N)
            assert np.array_equal(M.distribute_parallel(cands[l], w - 32, h - 32, N), ref)


@pytest.mark.parametrize("N", [0, 1, 5, 50, 3000])
def test_model_quadtree_budgets(N):
    import gpu_model as M
    img = S.uniform_noise_image(7, rows=150, cols=300)
    c = O.level_candidates(img)[0]
    ref = O.distribute(c, 16, 300 - 16, 16, 150 - 16, N)
    assert np.array_equal(M.distribute_parallel(c, 300 - 32, 150 - 32, N), ref)


def test_oracle_regression_fixtures():
    """Committed fixtures (tests/golden/oracle_fixtures.json, made by tests/golden/make_golden.py) guard the
    oracle against drift between rounds."""
    fx = json.load(open(os.path.join(GOLDEN, "oracle_fixtures.json")))
    for case in fx["cases"]:
        img = S.kitti_like_image(case["seed"], rows=case["rows"], cols=case["cols"])
        assert hashlib.sha256(img.tobytes()).hexdigest() == case["image_sha256"], "synthetic generator drifted"
        r = O.extract(img, nfeatures=case["nfeatures"])
        assert len(r["kps"]) == case["n"]
        assert hashlib.sha256(r["kps"].tobytes()).hexdigest() == case["kps_sha256"]
        assert hashlib.sha256(r["desc"].tobytes()).hexdigest() == case["desc_sha256"]
        assert r["ncand"].tolist() == case["ncand"]
        k0 = r["kps"][:8]
        assert [[float(v) for v in row] for row in k0.tolist()] == case["first_kps"]


def test_model_f16_score_form():
    """k_fast_wave's f16 score form (orbx_extract.hip fast_score_from_taps_f16): pixels stored as f16 1024 + value, differences,
    arc minima / maxima and the final max in f16, the score raised to -1 when below.  Every intermediate is an integer
    below 2048, so f16 is exact; the only change is max(s, -1), which alters no corner (s >= T >= 1) and no NMS
    outcome (a neighbour below T never blocks).  Checked against the integer score map on textured and noise images."""
    import gpu_model as M
    from multiagent_orb_slam2_amd import synthetic as S
    for img in (S.kitti_like_image(5, rows=120, cols=200), S.uniform_noise_image(7, rows=96, cols=160)):
        ref = M.score_map(img)[3:-3, 3:-3]
        h, w = img.shape
        I = (1024 + img.astype(np.int32)).astype(np.float16)          # exact: integers < 2048
        v = I[3:h - 3, 3:w - 3]
        d = np.stack([v - I[3 + dy:h - 3 + dy, 3 + dx:w - 3 + dx] for dx, dy in M.CIRCLE]).astype(np.float16)
        dd = np.concatenate([d, d[:9]], axis=0)
        mins = np.stack([dd[k:k + 9].min(axis=0) for k in range(16)])
        maxs = np.stack([dd[k:k + 9].max(axis=0) for k in range(16)])
        m = np.maximum(np.maximum(mins.max(axis=0), -maxs.min(axis=0)), np.float16(0)) + np.float16(1024)
        bits = m.view(np.uint16).astype(np.int32)
        s16 = bits - 0x6401                                             # i16 subtraction of the kernel
        assert np.array_equal(s16, np.maximum(ref, -1))
