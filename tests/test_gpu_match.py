"""GPU parity of the Hamming matchers against the CPU oracle — pair-index exact."""
import numpy as np
import pytest

from multiagent_orb_slam2_amd import synthetic as S

pytestmark = pytest.mark.gpu

BF, B = 386.1448, 0.537165   # KITTI 00-02 stereo (Examples/Stereo/KITTI00-02.yaml: bf, fx)


@pytest.fixture(scope="module")
def stereo_pair():
    import multiagent_orb_slam2_amd as pkg
    left = S.kitti_like_image(42)
    right = S.shifted_right_view(left, 42)
    ex = pkg.ORBextractor(2000, 1.2, 8, 20, 7)
    kl, dl = ex(left)
    kr, dr = ex(right)
    return dict(kl=kl, dl=dl, kr=kr, dr=dr, scale=ex.GetScaleFactors(), rows=left.shape[0])


@pytest.fixture(params=["tile", "mfma"])
def bf_mode(request, monkeypatch):
    """C3 both ways: the VALU tile kernel (k_bf_tile + k_bf_merge, ORBX_BF_MFMA=0) and the matrix-core form (k_bf_mfma,
    the default: bits unpacked to 0 / 1 bytes, popcount(q & t) by v_mfma_i32_16x16x64_i8; read per call).  (Round 5's one-launch form
    with a last-arriver fold was slower and is gone)"""
    monkeypatch.setenv("ORBX_BF_MFMA", "1" if request.param == "mfma" else "0")
    return request.param


def test_descriptor_distance(gpu):
    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    a, b = S.random_descriptors(1, 1000), S.random_descriptors(2, 1000)
    m = pkg.ORBmatcher()
    d = m.DescriptorDistance(a, b)
    ref = np.array([O.descriptor_distance(a[i], b[i]) for i in range(len(a))])
    assert np.array_equal(d, ref)
    assert m.DescriptorDistance(a[0], a[0]) == 0
    assert m.DescriptorDistance(np.zeros(32, np.uint8), np.full(32, 255, np.uint8)) == 256


@pytest.mark.parametrize("nq,nt", [(2000, 2000), (1, 1), (37, 5000), (3000, 700), (64, 0)])
def test_bf_match_c3(gpu, bf_mode, nq, nt):
    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    q, t = S.planted_pairs(7, nq, max(nt, 1))
    t = t[:nt]
    m = pkg.ORBmatcher()
    got = m.bf_match(q, t)
    ref = O.bf_match(q, t)
    for g, r, name in zip(got, ref, ("best_idx", "best_dist", "second_dist")):
        assert np.array_equal(g, r), name


@pytest.mark.parametrize("P,nq,nt", [(1, 2000, 2000), (16, 2000, 2000), (5, 300, 17), (3, 64, 0), (70, 33, 1200)])
def test_bf_match_batch_device(gpu, bf_mode, P, nq, nt):
    """orbx_bf_match_batch_device: P independent all-pairs problems in one launch, each equal to the oracle's."""
    import torch
    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    qs, ts = [], []
    for z in range(P):
        q, t = S.planted_pairs(100 + z, nq, max(nt, 1))
        qs.append(q)
        ts.append(t[:nt])
    dev = torch.device("cuda", 0)
    qd = torch.from_numpy(np.stack(qs)).to(dev)
    td = torch.from_numpy(np.stack(ts).reshape(P, nt, 32)).to(dev)
    bi, bd, sd = pkg.ORBmatcher().bf_match_batch_device(qd, td)
    bi, bd, sd = bi.cpu().numpy(), bd.cpu().numpy(), sd.cpu().numpy()
    for z in range(P):
        ref = O.bf_match(qs[z], ts[z])
        for g, r, name in zip((bi[z], bd[z], sd[z]), ref, ("best_idx", "best_dist", "second_dist")):
            assert np.array_equal(g, r), (z, name)


def test_bf_match_ties_and_full_distance(gpu, bf_mode):
    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    q = np.zeros((3, 32), np.uint8)
    q[1] = 255
    t = np.stack([np.full(32, 255, np.uint8), np.zeros(32, np.uint8), np.zeros(32, np.uint8)])
    got = pkg.ORBmatcher().bf_match(q, t)
    ref = O.bf_match(q, t)
    for g, r in zip(got, ref):
        assert np.array_equal(g, r)
    # a query at distance 256 from every train row never matches (init 256, strict <)
    got = pkg.ORBmatcher().bf_match(np.zeros((1, 32), np.uint8), np.full((4, 32), 255, np.uint8))
    assert got[0][0] == -1 and got[1][0] == 256


def test_stereo_band_match(gpu, stereo_pair):
    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    p = stereo_pair
    m = pkg.ORBmatcher()
    res = m.stereo_descriptor_search(p["kl"], p["dl"], p["kr"], p["dr"], p["scale"], p["rows"], BF, B)
    n, idx, dist = O.stereo_match(p["kl"], p["dl"], p["kr"], p["dr"], p["scale"], p["rows"], BF, B)
    assert np.array_equal(res.best_idx, idx)
    assert np.array_equal(res.best_dist, dist)
    assert res.n_matched == n and n > 300


def test_stereo_batch_device(gpu):
    import torch

    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    lefts = [S.kitti_like_image(200 + i) for i in range(3)]
    rights = [S.shifted_right_view(l, 200 + i) for i, l in enumerate(lefts)]
    ex = pkg.ORBextractor(2000, 1.2, 8, 20, 7)
    imgs = torch.from_numpy(np.stack(lefts + rights)).cuda()
    kps, desc, cnt = ex.extract_batch_device(imgs)
    cap = kps.shape[1]
    m = pkg.ORBmatcher()
    bi, bd = m.stereo_match_batch_device(kps[:3], desc[:3], cnt[:3], kps[3:], desc[3:], cnt[3:], cap,
                                         ex.GetScaleFactors(), 375, BF, B)
    torch.cuda.synchronize()
    kps_h, desc_h, cnt_h = kps.cpu().numpy(), desc.cpu().numpy(), cnt.cpu().numpy()
    bi, bd = bi.cpu().numpy(), bd.cpu().numpy()
    for i in range(3):
        nl, nr = int(cnt_h[i]), int(cnt_h[3 + i])
        kl = kps_h[i, :nl].copy().view(pkg.KP_DTYPE).reshape(-1)
        kr = kps_h[3 + i, :nr].copy().view(pkg.KP_DTYPE).reshape(-1)
        n, idx, dist = O.stereo_match(kl, desc_h[i, :nl], kr, desc_h[3 + i, :nr], ex.GetScaleFactors(), 375, BF, B)
        assert np.array_equal(bi[i, :nl], idx) and np.array_equal(bd[i, :nl], dist)


def _dense_rows_kps(seed, n, y0, y1, xmax=1200.0):
    import multiagent_orb_slam2_amd as pkg
    rng = np.random.default_rng(seed)
    k = np.zeros(n, pkg.KP_DTYPE)
    k["x"] = rng.uniform(20.0, xmax, n).astype(np.float32)
    k["y"] = rng.uniform(y0, y1, n).astype(np.float32)
    k["octave"] = rng.integers(0, 8, n)
    k["size"] = 31.0
    return k


@pytest.mark.parametrize("nl,nr,band", [(3000, 3000, (100.0, 104.0)), (700, 4000, (0.0, 12.0)), (2500, 10, (360.0, 375.0))])
def test_stereo_dense_rows(gpu, nl, nr, band):
    """Keypoints crowded into a few rows: the row-block search stages more right keypoints than one LDS chunk
    (512) and more left keypoints than one left chunk (128) per block, plus rows at the image edges."""
    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    q, t = S.planted_pairs(11 + nl, nl, nr, frac=0.6, flip_p=0.03)
    kl = _dense_rows_kps(1, nl, *band)
    kr = _dense_rows_kps(2, nr, band[0] - 2.0, band[1] + 2.0)
    kr["x"] = np.clip(kr["x"], 0, 1241)
    scale = pkg.ORBextractor(2000, 1.2, 8, 20, 7).GetScaleFactors()
    res = pkg.ORBmatcher().stereo_descriptor_search(kl, q, kr, t, scale, 375, BF, B)
    n, idx, dist = O.stereo_match(kl, q, kr, t, scale, 375, BF, B)
    assert np.array_equal(res.best_idx, idx) and np.array_equal(res.best_dist, dist)
    assert n > 0 or nr < 100


def _kf(seed, n_nodes=60):
    import multiagent_orb_slam2_amd as pkg
    img = S.kitti_like_image(seed)
    ex = pkg.ORBextractor(2000, 1.2, 8, 20, 7)
    k, d = ex(img)
    fv = S.random_featvec(seed, len(k), n_nodes=n_nodes)
    rng = np.random.default_rng(seed)
    valid = (rng.random(len(k)) < 0.7).astype(np.uint8)
    return k, d, fv, valid


@pytest.mark.parametrize("check_ori", [True, False])
def test_search_by_bow_kfkf(gpu, check_ori):
    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    k1, d1, fv1, v1 = _kf(300)
    # second keyframe: a shifted view so that real matches exist
    k2, d2, fv2, v2 = _kf(300)
    k2b, d2b = k2.copy(), d2.copy()
    rng = np.random.default_rng(5)
    flip = rng.random(d2b.shape) < 0.02
    d2b = d2b ^ (flip * rng.integers(1, 256, d2b.shape)).astype(np.uint8)
    fv2 = S.random_featvec(301, len(k2b), n_nodes=60)
    m = pkg.ORBmatcher(0.75, check_ori)
    n, m12 = m.SearchByBoW_KF_KF(d1, k1["angle"], v1, fv1, d2b, k2b["angle"], v2, fv2)
    rn, rm = O.search_by_bow_kfkf(d1, k1["angle"], v1, fv1, d2b, k2b["angle"], v2, fv2, 0.75, check_ori)
    assert n == rn and np.array_equal(m12, rm)


def test_search_by_bow_kfkf_same_nodes(gpu):
    """Identical node assignment in both keyframes -> many true matches, greedy coupling exercised."""
    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    k1, d1, fv1, v1 = _kf(310, n_nodes=20)
    rng = np.random.default_rng(9)
    d2 = d1 ^ ((rng.random(d1.shape) < 0.01) * 1).astype(np.uint8)
    v2 = np.ones(len(d1), np.uint8)
    a2 = (k1["angle"] + rng.normal(0, 3, len(k1))).astype(np.float32) % 360
    m = pkg.ORBmatcher(0.75, True)
    n, m12 = m.SearchByBoW_KF_KF(d1, k1["angle"], v1, fv1, d2, a2, v2, fv1)
    rn, rm = O.search_by_bow_kfkf(d1, k1["angle"], v1, fv1, d2, a2, v2, fv1, 0.75, True)
    assert n == rn and np.array_equal(m12, rm) and n > 100


def test_search_by_bow_kf_frame(gpu):
    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    kk, dk, fvk, vk = _kf(320, n_nodes=25)
    rng = np.random.default_rng(3)
    df = dk ^ ((rng.random(dk.shape) < 0.015) * rng.integers(1, 256, dk.shape)).astype(np.uint8)
    af = kk["angle"].copy()
    m = pkg.ORBmatcher(0.7, True)
    n, mf = m.SearchByBoW_KF_F(dk, kk["angle"], vk, fvk, df, af, fvk)
    rn, rm = O.search_by_bow_kff(dk, kk["angle"], vk, fvk, df, af, fvk, 0.7, True)
    assert n == rn and np.array_equal(mf, rm) and n > 50


@pytest.mark.parametrize("only_stereo", [False, True])
def test_search_for_triangulation(gpu, only_stereo):
    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    k1, d1, fv1, _ = _kf(330, n_nodes=30)
    rng = np.random.default_rng(11)
    d2 = d1 ^ ((rng.random(d1.shape) < 0.02) * rng.integers(1, 256, d1.shape)).astype(np.uint8)
    k2 = k1.copy()
    k2["x"] += rng.normal(0, 2, len(k2)).astype(np.float32)
    k2["y"] += rng.normal(0, 2, len(k2)).astype(np.float32)
    mp1 = (rng.random(len(k1)) < 0.3).astype(np.uint8)
    mp2 = (rng.random(len(k1)) < 0.3).astype(np.uint8)
    ur1 = np.where(rng.random(len(k1)) < 0.5, rng.uniform(0, 1000, len(k1)), -1).astype(np.float32)
    ur2 = np.where(rng.random(len(k1)) < 0.5, rng.uniform(0, 1000, len(k1)), -1).astype(np.float32)
    # fundamental matrix of a small sideways motion (rank-2, float)
    F12 = np.array([[0, -1e-6, 2e-4], [1e-6, 0, -3e-3], [-2e-4, 3e-3, 0.02]], np.float32)
    scale = np.array([1.2 ** i for i in range(8)], np.float32)
    sigma2 = (scale * scale).astype(np.float32)
    m = pkg.ORBmatcher(0.6, True)
    n, m12 = m.SearchForTriangulation(d1, k1, mp1, ur1, fv1, d2, k2, mp2, ur2, fv1, F12, sigma2, scale, 600.0,
                                      180.0, only_stereo)
    rn, rm = O.search_for_triangulation(d1, k1, mp1, ur1, fv1, d2, k2, mp2, ur2, fv1, F12, sigma2, scale, 600.0,
                                        180.0, only_stereo, True)
    assert n == rn and np.array_equal(m12, rm)


def test_bf_match_ties_across_chunks(gpu, bf_mode):
    """Long train sets split into many chunks (the grouped merge): equal distances in different chunks keep the first
    train index, and the second distance counts the tie (strict '<' of ORBmatcher.cc:568-598)."""
    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    rng = np.random.Generator(np.random.PCG64(5))
    q = rng.integers(0, 256, (40, 32), dtype=np.uint8)
    t = np.repeat(rng.integers(0, 256, (3, 32), dtype=np.uint8), 1500, axis=0)   # 4500 rows, three distinct values
    t[4000:] = q[0]                                                                 # exact matches of query 0 late
    t[100] = ~q[1]                                                                  # distance 256 for query 1
    m = pkg.ORBmatcher()
    got = m.bf_match(q, t)
    ref = O.bf_match(q, t)
    for g, r, name in zip(got, ref, ("best_idx", "best_dist", "second_dist")):
        assert np.array_equal(g, r), name
    assert got[0][0] == 4000 and got[1][0] == 0 and got[2][0] == 0


def test_matchers_empty_and_degenerate_inputs(gpu, bf_mode):
    """What the reference's loops do with nothing to loop over (ORBmatcher.cc:161-290, :524-657; Frame.cc:466-549):
    no queries, no train rows, a keyframe without FeatureVector nodes, no MapPoints (every vpMapPoints entry NULL),
    an empty right image -- no matches and no error, as the oracle."""
    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    m = pkg.ORBmatcher(0.75, True)
    q, t = S.planted_pairs(3, 50, 80)
    for qq, tt in ((q[:0], t), (q, t[:0]), (q[:0], t[:0]), (q[:1], t[:1])):
        got, ref = m.bf_match(qq, tt), O.bf_match(qq, tt)
        for g, r in zip(got, ref):
            assert np.array_equal(g, r), (len(qq), len(tt))
    k1, d1, fv1, v1 = _kf(330, n_nodes=30)
    no_nodes = (np.zeros(0, np.uint32), np.zeros(1, np.int32), np.zeros(0, np.int32))
    cases = [(fv1, v1, no_nodes, v1), (no_nodes, v1, fv1, v1), (fv1, np.zeros_like(v1), fv1, v1),
             (fv1, v1, fv1, np.zeros_like(v1))]
    for i, (fa, va, fb, vb) in enumerate(cases):
        n, m12 = m.SearchByBoW_KF_KF(d1, k1["angle"], va, fa, d1, k1["angle"], vb, fb)
        rn, rm = O.search_by_bow_kfkf(d1, k1["angle"], va, fa, d1, k1["angle"], vb, fb, 0.75, True)
        assert n == rn == 0 and np.array_equal(m12, rm), i
    n, mf = m.SearchByBoW_KF_F(d1, k1["angle"], np.zeros_like(v1), fv1, d1, k1["angle"], fv1)
    rn, rm = O.search_by_bow_kff(d1, k1["angle"], np.zeros_like(v1), fv1, d1, k1["angle"], fv1, 0.75, True)
    assert n == rn == 0 and np.array_equal(mf, rm)
    scale = pkg.ORBextractor(2000, 1.2, 8, 20, 7).GetScaleFactors()
    kl = _dense_rows_kps(4, 300, 20.0, 350.0)
    for nl, nr in ((300, 0), (0, 300)):
        res = m.stereo_descriptor_search(kl[:nl], np.resize(q, (nl, 32)), kl[:nr], np.resize(t, (nr, 32)), scale, 375, BF, B)
        rn, idx, dist = O.stereo_match(kl[:nl], np.resize(q, (nl, 32)), kl[:nr], np.resize(t, (nr, 32)), scale, 375, BF, B)
        assert res.n_matched == rn == 0 and np.array_equal(res.best_idx, idx) and np.array_equal(res.best_dist, dist)
