"""Sub-pixel stereo (Frame::ComputeStereoMatches, src/Frame.cc:554-639): SAD window search, parabola fit,
disparity test, median-SAD rejection.  CPU: the oracle against a pure-Python restatement.  GPU: host
(two extractors) and batched device forms bit-exact (float32 bits of mvuRight / mvDepth) vs the oracle."""
import numpy as np
import pytest

from multiagent_orb_slam2_amd import synthetic as S
from oracle import oracle as O

BF, B = 386.1448, 0.537165      # Examples/Stereo/KITTI00-02.yaml


def _round(x):
    """C round(): half away from zero (coordinates are positive; x - floor(x) is exact)."""
    r = np.floor(x)
    return np.float32(r + 1) if x - r >= 0.5 else np.float32(r)


def _py_refine(kl, kr, best_idx, scale, inv_scale, pl, pr, bf, b):
    f = np.float32
    maxD = f(bf) / f(b)
    ur = np.full(len(kl), -1, np.float32)
    dp = np.full(len(kl), -1, np.float32)
    acc = []
    for i, k in enumerate(kl):
        if best_idx[i] < 0:
            continue
        o = int(k["octave"])
        sf = f(inv_scale[o])
        suL, svL = _round(f(k["x"]) * sf), _round(f(k["y"]) * sf)
        suR0 = _round(f(kr[best_idx[i]]["x"]) * sf)
        iuL, ivL, iuR0 = int(suL), int(svL), int(suR0)
        L, R = pl[o].astype(np.int64), pr[o].astype(np.int64)
        if ivL - 5 < 0 or ivL + 5 >= L.shape[0] or iuL - 5 < 0 or iuL + 5 >= L.shape[1] or ivL + 5 >= R.shape[0] \
                or iuR0 - 10 < 0 or suR0 + 11 >= R.shape[1]:
            continue
        IL = L[ivL - 5:ivL + 6, iuL - 5:iuL + 6]
        IL = IL - IL[5, 5]
        d = []
        for inc in range(-5, 6):
            IR = R[ivL - 5:ivL + 6, iuR0 + inc - 5:iuR0 + inc + 6]
            d.append(int(np.abs(IL - (IR - IR[5, 5])).sum()))
        bi = int(np.argmin(d)) - 5                       # first minimum
        if bi in (-5, 5):
            continue
        d1, d2, d3 = f(d[bi + 4]), f(d[bi + 5]), f(d[bi + 6])
        delta = (d1 - d3) / (f(2) * (d1 + d3 - f(2) * d2))
        if delta < -1 or delta > 1:
            continue
        u = f(scale[o]) * ((f(suR0) + f(bi)) + delta)
        disp = f(k["x"]) - u
        if disp >= 0 and disp < maxD:
            if disp <= 0:
                disp, u = f(0.01), f(float(k["x"]) - 0.01)
            ur[i], dp[i] = u, f(bf) / disp
            acc.append((d[bi + 5], i))
    if acc:
        acc.sort()
        th = f(f(1.5) * f(1.4)) * f(acc[len(acc) // 2][0])
        for dist, i in acc:
            if not f(dist) < th:
                ur[i] = dp[i] = -1
    return ur, dp


@pytest.mark.parametrize("seed", [0, 5])
def test_oracle_refine_matches_python(seed):
    l = S.kitti_like_image(seed, rows=140, cols=360)
    r = S.shifted_right_view(l, seed, max_disp=30)
    a, b = O.extract(l, nfeatures=400, want_pyramid=True), O.extract(r, nfeatures=400, want_pyramid=True)
    t = O.tables(400)
    _, bi, _ = O.stereo_match(a["kps"], a["desc"], b["kps"], b["desc"], t["scale"], l.shape[0], BF, B)
    n, ur, dp, sad = O.stereo_refine(a["kps"], b["kps"], bi, t["scale"], t["inv_scale"], a["pyramid"], b["pyramid"], BF, B)
    pur, pdp = _py_refine(a["kps"], b["kps"], bi, t["scale"], t["inv_scale"], a["pyramid"], b["pyramid"], BF, B)
    assert ur.tobytes() == pur.tobytes() and dp.tobytes() == pdp.tobytes()
    assert n == int((ur >= 0).sum()) and n > 20


def test_oracle_refine_empty_and_no_matches():
    l = S.kitti_like_image(3, rows=140, cols=360)
    a = O.extract(l, nfeatures=300, want_pyramid=True)
    t = O.tables(300)
    bi = np.full(len(a["kps"]), -1, np.int32)
    n, ur, dp, _ = O.stereo_refine(a["kps"], a["kps"], bi, t["scale"], t["inv_scale"], a["pyramid"], a["pyramid"], BF, B)
    assert n == 0 and (ur == -1).all() and (dp == -1).all()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,shape,nf", [(11, (375, 1242), 2000), (12, (375, 1242), 2000), (13, (480, 752), 1200),
                                           (14, (200, 420), 500), (15, (1080, 1920), 3000)])
def test_gpu_compute_stereo_matches_host(gpu, seed, shape, nf):
    import multiagent_orb_slam2_amd as pkg
    l = S.kitti_like_image(seed, rows=shape[0], cols=shape[1])
    r = S.shifted_right_view(l, seed)
    exl, exr = pkg.ORBextractor(nf, 1.2, 8, 20, 7), pkg.ORBextractor(nf, 1.2, 8, 20, 7)
    kl, dl = exl(l)
    kr, dr = exr(r)
    m = pkg.ORBmatcher()
    ur, dp = m.ComputeStereoMatches(exl, exr, kl, dl, kr, dr, BF, B)
    a, b = O.extract(l, nfeatures=nf, want_pyramid=True), O.extract(r, nfeatures=nf, want_pyramid=True)
    t = O.tables(nf)
    rur, rdp = O.compute_stereo_matches(a, b, t["scale"], t["inv_scale"], shape[0], BF, B)
    assert ur.tobytes() == rur.tobytes() and dp.tobytes() == rdp.tobytes()
    assert (dp > 0).sum() > 0.2 * len(kl)


@pytest.mark.gpu
def test_gpu_stereo_frame_one_call(gpu):
    """orbx_stereo_frame (the stereo Frame constructor's extractions + ComputeStereoMatches in one call, the search on the
    extractions' device outputs) equals the oracle and the two-call form, frame after frame on the same objects, over
    three image sizes up to 1920 x 1080 (reconfigurations between them) and an empty pair."""
    import multiagent_orb_slam2_amd as pkg
    exl, exr = pkg.ORBextractor(2000, 1.2, 8, 20, 7), pkg.ORBextractor(2000, 1.2, 8, 20, 7)
    m = pkg.ORBmatcher()
    t = O.tables(2000)
    for i, shape in enumerate([(375, 1242), (375, 1242), (240, 420), (1080, 1920), (375, 1242)]):
        l = S.kitti_like_image(40 + i, rows=shape[0], cols=shape[1])
        r = S.shifted_right_view(l, 40 + i)
        (kl, dl), (kr, dr), ur, dp = m.StereoFrame(exl, exr, l, r, BF, B)
        a, b = O.extract(l, nfeatures=2000, want_pyramid=True), O.extract(r, nfeatures=2000, want_pyramid=True)
        assert np.array_equal(kl, a["kps"]) and np.array_equal(dl, a["desc"]), i
        assert np.array_equal(kr, b["kps"]) and np.array_equal(dr, b["desc"]), i
        rur, rdp = O.compute_stereo_matches(a, b, t["scale"], t["inv_scale"], shape[0], BF, B)
        assert ur.tobytes() == rur.tobytes() and dp.tobytes() == rdp.tobytes(), i
        assert (dp > 0).sum() > 0.2 * len(kl)
        (kl2, dl2), (kr2, dr2) = pkg.extract_pair(exl, exr, l, r)
        ur2, dp2 = m.ComputeStereoMatches(exl, exr, kl2, dl2, kr2, dr2, BF, B)
        assert ur.tobytes() == ur2.tobytes() and dp.tobytes() == dp2.tobytes(), i
    e = np.zeros((0, 0), np.uint8)
    (kl, _), (kr, _), ur, dp = m.StereoFrame(exl, exr, e, e, BF, B)
    assert len(kl) == len(kr) == len(ur) == len(dp) == 0
    with pytest.raises(pkg.OrbxError):                  # one extractor for both sides is refused, as orbx_extract_pair
        m.StereoFrame(exl, exl, l, r, BF, B)
    # the objects stay usable after a refused call
    (kl, dl), (kr, dr), ur, dp = m.StereoFrame(exl, exr, l, r, BF, B)
    (kl2, dl2), (kr2, dr2) = pkg.extract_pair(exl, exr, l, r)
    assert np.array_equal(kl, kl2) and np.array_equal(dr, dr2)
    # refused after both extractions were enqueued (the sides' pyramids differ): the call reports that reason, and the
    # extractions it dropped leave both objects usable
    ex4 = pkg.ORBextractor(2000, 1.2, 4, 20, 7)
    with pytest.raises(pkg.OrbxError, match="differ"):
        m.StereoFrame(exl, ex4, l, r, BF, B)
    k4, d4 = ex4(r)
    k4f, d4f = pkg.ORBextractor(2000, 1.2, 4, 20, 7)(r)
    assert np.array_equal(k4, k4f) and np.array_equal(d4, d4f)
    (kl3, dl3), _, ur3, dp3 = m.StereoFrame(exl, exr, l, r, BF, B)
    assert np.array_equal(kl3, kl) and ur3.tobytes() == ur.tobytes() and dp3.tobytes() == dp.tobytes()


@pytest.mark.gpu
def test_gpu_stereo_refine_batch_device(gpu):
    import torch

    import multiagent_orb_slam2_amd as pkg
    n = 3
    lefts = [S.kitti_like_image(300 + i) for i in range(n)]
    rights = [S.shifted_right_view(x, 300 + i) for i, x in enumerate(lefts)]
    imgs = torch.from_numpy(np.stack(lefts + rights)).cuda()
    ex = pkg.ORBextractor(2000, 1.2, 8, 20, 7)
    kps, desc, cnt = ex.extract_batch_device(imgs)
    cap = kps.shape[1]
    m = pkg.ORBmatcher()
    scale = ex.GetScaleFactors()
    bi, bd = m.stereo_match_batch_device(kps[:n], desc[:n], cnt[:n], kps[n:], desc[n:], cnt[n:], cap, scale, 375, BF, B)
    pyr = ex.pyramid_device()
    ur, dp = m.stereo_refine_batch_device(kps[:n], cnt[:n], kps[n:], bi, pyr, 0, pyr, n, BF, B)
    torch.cuda.synchronize()
    urh, dph, ch = ur.cpu().numpy(), dp.cpu().numpy(), cnt.cpu().numpy()
    t = O.tables(2000)
    for i in range(n):
        a, b = O.extract(lefts[i], want_pyramid=True), O.extract(rights[i], want_pyramid=True)
        rur, rdp = O.compute_stereo_matches(a, b, t["scale"], t["inv_scale"], 375, BF, B)
        assert urh[i, :ch[i]].tobytes() == rur.tobytes() and dph[i, :ch[i]].tobytes() == rdp.tobytes()
        assert (urh[i, ch[i]:] == -1).all()


@pytest.mark.gpu
def test_gpu_stereo_refine_pyramid_ring(gpu):
    """Pyramid ring of 2 (orbx_extractor_set_pyramid_ring): step k's pyramid stays intact while step k+1 extracts
    other images, so step k's SAD refinement run after step k+1 still equals the oracle's (the bench runs it on its
    own stream beside the next extraction)."""
    import torch

    import multiagent_orb_slam2_amd as pkg
    n = 2
    lefts = [S.kitti_like_image(310 + i) for i in range(n)]
    rights = [S.shifted_right_view(x, 310 + i) for i, x in enumerate(lefts)]
    imgs = torch.from_numpy(np.stack(lefts + rights)).cuda()
    other = torch.from_numpy(np.stack([S.kitti_like_image(400 + i) for i in range(2 * n)])).cuda()
    ex = pkg.ORBextractor(2000, 1.2, 8, 20, 7)
    ex.set_pyramid_ring(2)
    kps, desc, cnt = ex.extract_batch_device(imgs)
    pyr = ex.pyramid_device()
    ex.extract_batch_device(other)                                 # writes the other pyramid set
    assert ex.pyramid_device().levels != pyr.levels
    cap = kps.shape[1]
    m = pkg.ORBmatcher()
    scale = ex.GetScaleFactors()
    bi, bd = m.stereo_match_batch_device(kps[:n], desc[:n], cnt[:n], kps[n:], desc[n:], cnt[n:], cap, scale, 375, BF, B)
    ur, dp = m.stereo_refine_batch_device(kps[:n], cnt[:n], kps[n:], bi, pyr, 0, pyr, n, BF, B)
    torch.cuda.synchronize()
    urh, dph, ch = ur.cpu().numpy(), dp.cpu().numpy(), cnt.cpu().numpy()
    t = O.tables(2000)
    for i in range(n):
        a, b = O.extract(lefts[i], want_pyramid=True), O.extract(rights[i], want_pyramid=True)
        rur, rdp = O.compute_stereo_matches(a, b, t["scale"], t["inv_scale"], 375, BF, B)
        assert urh[i, :ch[i]].tobytes() == rur.tobytes() and dph[i, :ch[i]].tobytes() == rdp.tobytes()
