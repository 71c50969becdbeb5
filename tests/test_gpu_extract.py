"""GPU parity of the ORB extractor (HIP, liborbx.so) against the CPU oracle — bit-exact on every
keypoint field (x, y, size, angle, response, octave, class_id) and every descriptor byte.

Oracle status: "parity unpinned" (the reference cannot be built here and ships no golden vectors; see
oracle/orb_oracle.cpp and DESIGN.md)."""
import numpy as np
import pytest

from multiagent_orb_slam2_amd import synthetic as S

pytestmark = pytest.mark.gpu


def _diff_report(k, d, rk, rd):
    msg = [f"n gpu={len(k)} oracle={len(rk)}"]
    if len(k) and len(rk):
        bg = np.bincount(k["octave"], minlength=8)
        bo = np.bincount(rk["octave"], minlength=8)
        msg.append(f"per level gpu={bg.tolist()} oracle={bo.tolist()}")
        n = min(len(k), len(rk))
        for f in k.dtype.names:
            bad = np.nonzero(k[f][:n] != rk[f][:n])[0]
            if len(bad):
                i = bad[0]
                msg.append(f"field {f}: {len(bad)} differ, first at {i}: gpu={k[i]} oracle={rk[i]}")
        bad = np.nonzero((d[:n] != rd[:n]).any(axis=1))[0]
        if len(bad):
            msg.append(f"descriptors: {len(bad)} rows differ, first {bad[0]}")
    return "\n".join(msg)


def _check(img, nfeatures=2000, nlevels=8, scale=1.2, ini=20, mn=7):
    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    ex = pkg.ORBextractor(nfeatures, scale, nlevels, ini, mn, device=0)
    k, d = ex(img)
    ref = O.extract(img, nfeatures=nfeatures, scale_factor=scale, nlevels=nlevels, ini_th=ini, min_th=mn)
    rk, rd = ref["kps"], ref["desc"]
    ok = len(k) == len(rk) and np.array_equal(k, rk) and np.array_equal(d, rd)
    assert ok, _diff_report(k, d, rk, rd)
    return ex, k, d


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_kitti_c2_bit_exact(gpu, seed):
    img = S.kitti_like_image(seed)
    _, k, _ = _check(img)
    assert len(k) >= 1900


def test_c1_640x480_1000(gpu):
    _check(S.kitti_like_image(21, rows=480, cols=640), nfeatures=1000)


def test_euroc_752x480_1200(gpu):
    _check(S.kitti_like_image(31, rows=480, cols=752), nfeatures=1200)


def test_uniform_noise_stress(gpu):
    _check(S.uniform_noise_image(1000))


def test_constant_image_no_keypoints(gpu):
    import multiagent_orb_slam2_amd as pkg
    ex = pkg.ORBextractor(2000, 1.2, 8, 20, 7)
    k, d = ex(np.full((375, 1242), 128, np.uint8))
    assert len(k) == 0 and d.shape == (0, 32)


def test_empty_image_returns_nothing(gpu):
    import multiagent_orb_slam2_amd as pkg
    ex = pkg.ORBextractor(2000, 1.2, 8, 20, 7)
    k, d = ex(np.zeros((0, 0), np.uint8))
    assert len(k) == 0


@pytest.mark.parametrize("shape", [(377, 1243), (120, 160), (96, 300), (500, 500), (40, 40), (1000, 200)])
def test_odd_and_small_sizes(gpu, shape):
    _check(S.kitti_like_image(5, rows=shape[0], cols=shape[1]), nfeatures=800)


@pytest.mark.parametrize("nf", [40, 300, 5000])
def test_feature_budgets(gpu, nf):
    _check(S.kitti_like_image(7), nfeatures=nf)


def test_other_params(gpu):
    _check(S.kitti_like_image(8), nfeatures=1500, nlevels=5, scale=1.3, ini=25, mn=10)


def test_pyramid_matches_oracle(gpu):
    from oracle import oracle as O
    img = S.kitti_like_image(9)
    ex, _, _ = _check(img)
    ref = O.extract(img, want_pyramid=True)["pyramid"]
    got = ex.mvImagePyramid
    assert len(got) == len(ref)
    for l, (a, b) in enumerate(zip(got, ref)):
        assert a.shape == b.shape and np.array_equal(a, b), f"level {l}"


def test_batch_device_equals_single(gpu):
    import torch

    import multiagent_orb_slam2_amd as pkg
    imgs = np.stack([S.kitti_like_image(100 + i) for i in range(5)])
    ex = pkg.ORBextractor(2000, 1.2, 8, 20, 7)
    t = torch.from_numpy(imgs).cuda()
    kps, desc, cnt = ex.extract_batch_device(t)
    torch.cuda.synchronize()
    kps, desc, cnt = kps.cpu().numpy(), desc.cpu().numpy(), cnt.cpu().numpy()
    ex1 = pkg.ORBextractor(2000, 1.2, 8, 20, 7)
    for i in range(len(imgs)):
        k1, d1 = ex1(imgs[i])
        n = int(cnt[i])
        kb = kps[i, :n].copy().view(pkg.KP_DTYPE).reshape(-1)
        assert n == len(k1)
        assert np.array_equal(kb, k1) and np.array_equal(desc[i, :n], d1)


@pytest.mark.parametrize("ring,desc_side", [(1, 0), (2, 0), (2, 1)])
def test_split_streams_back_to_back(gpu, monkeypatch, ring, desc_side):
    """orbx_extract_batch_device_split: calls issued back to back without a host sync, the descriptor stage on a
    second stream, so call k+1's front half overlaps call k's descriptor stage.  Every call must equal the
    single-image host API (the extractor orders its own buffer reuse across calls).  desc_side: the descriptor stage
    at the end of the extractor's side stream (ORBX_DESC_SIDE=1), the output stream waiting for it."""
    import torch

    import multiagent_orb_slam2_amd as pkg
    monkeypatch.setenv("ORBX_DESC_SIDE", str(desc_side))
    batches = [np.stack([S.kitti_like_image(300 + 7 * b + i) for i in range(3)]) for b in range(4)]
    ex = pkg.ORBextractor(2000, 1.2, 8, 20, 7)
    ex.set_pyramid_ring(ring)
    s_in, s_out = torch.cuda.Stream(), torch.cuda.Stream()
    ts = [torch.from_numpy(b).cuda() for b in batches]
    torch.cuda.synchronize()
    outs = []
    for t in ts:
        outs.append(ex.extract_batch_device(t, stream=s_in, out_stream=s_out))
    torch.cuda.synchronize()
    ex1 = pkg.ORBextractor(2000, 1.2, 8, 20, 7)
    for b, (kps, desc, cnt) in zip(batches, outs):
        kps, desc, cnt = kps.cpu().numpy(), desc.cpu().numpy(), cnt.cpu().numpy()
        for i in range(len(b)):
            k1, d1 = ex1(b[i])
            n = int(cnt[i])
            kb = kps[i, :n].copy().view(pkg.KP_DTYPE).reshape(-1)
            assert n == len(k1)
            assert np.array_equal(kb, k1) and np.array_equal(desc[i, :n], d1)


@pytest.mark.parametrize("kpw", [1, 2, 4])
def test_describe_keypoints_per_wave(gpu, monkeypatch, kpw):
    """k_describe (one keypoint per wave) and k_describe_m (2 or 4 per wave, levels straddling a wave) give the same
    bits: ORBX_DESC_KPW picks the form at extractor creation.  Batched, so waves also straddle images' slot ends."""
    import torch

    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    monkeypatch.setenv("ORBX_DESC_KPW", str(kpw))
    imgs = np.stack([S.kitti_like_image(400 + i) for i in range(3)])
    ex = pkg.ORBextractor(2000, 1.2, 8, 20, 7)
    kps, desc, cnt = ex.extract_batch_device(torch.from_numpy(imgs).cuda())
    torch.cuda.synchronize()
    kps, desc, cnt = kps.cpu().numpy(), desc.cpu().numpy(), cnt.cpu().numpy()
    for i in range(len(imgs)):
        ref = O.extract(imgs[i])
        n = int(cnt[i])
        kb = kps[i, :n].copy().view(pkg.KP_DTYPE).reshape(-1)
        assert np.array_equal(kb, ref["kps"]) and np.array_equal(desc[i, :n], ref["desc"]), _diff_report(
            kb, desc[i, :n], ref["kps"], ref["desc"])
    # odd feature budget and level count: level slot ranges of odd lengths
    _check(S.kitti_like_image(410, rows=240, cols=333), nfeatures=777, nlevels=5, scale=1.3)


@pytest.mark.parametrize("form", ["dot2", "row", "lds"])
def test_blurred_pyramid_bit_exact(gpu, monkeypatch, form):
    """Every pixel of every blurred level -- not only the windows around keypoints that the descriptor tests see --
    equals the oracle's GaussianBlur(7x7, sigma 2, REFLECT_101) of the oracle's pyramid level
    (ORBextractor.cc:1085-1086): interior strips, strips at a level's left / right edge (REFLECT_101 columns by byte
    selectors in k_blur7<true>), levels under 12 columns, bottom rows, saturation (a constant 255 image blurs to 255 with
    taps summing to 257), batched (image index > 0).  Forms: k_blur7 in vertical row pairs (default), one row at a time,
    and k_blur7_lds."""
    import torch

    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    monkeypatch.setenv("ORBX_BLUR_DOT2", "0" if form == "row" else "1")
    monkeypatch.setenv("ORBX_BLUR_LDS", "1" if form == "lds" else "0")
    monkeypatch.setenv("ORBX_DESC_FB", "0")
    for shape in ((375, 1242), (377, 1243), (480, 752), (1000, 200), (40, 40), (61, 97)):
        imgs = np.stack([S.kitti_like_image(700 + shape[1], rows=shape[0], cols=shape[1]),
                         S.uniform_noise_image(701, rows=shape[0], cols=shape[1]) if shape == (375, 1242)
                         else S.kitti_like_image(701, rows=shape[0], cols=shape[1]),
                         np.full(shape, 255, np.uint8)])
        ex = pkg.ORBextractor(1000, 1.2, 8, 20, 7)
        ex.extract_batch_device(torch.from_numpy(imgs).cuda())
        torch.cuda.synchronize()
        for i in range(len(imgs)):
            ref = O.extract(imgs[i], nfeatures=1000, want_pyramid=True)["pyramid"]
            got = ex.blurred_levels(i, shape)
            assert len(got) == len(ref)
            for l, (a, lv) in enumerate(zip(got, ref)):
                b = O.blur7(lv)
                bad = np.argwhere(a != b)
                assert a.shape == b.shape and len(bad) == 0, (
                    f"shape {shape} image {i} level {l} ({lv.shape}): {len(bad)} pixels differ, first {bad[:3].tolist()}")


@pytest.mark.parametrize("form", ["band", "band_blur1row", "rows", "wave", "wave_blurlds", "wave_1pass", "wave20", "wave2",
                                  "wave1", "wave_cells2", "wave_cells4"])
def test_fast_kernels_bit_exact(gpu, monkeypatch, form):
    """Every FAST form -- k_fast_band (LDS band image, pre-test and survivor list), k_fast_rows (one wave per cell
    row in registers, every pixel scored, both thresholds' lists) and k_fast_wave (one wave per cell, no barrier; 4, 2
    or 1 waves per workgroup) -- is bit-exact against the oracle (and so is k_blur7 in both forms: vertical row pairs with
    v_dot2 column sums, the default, one row at a time, and k_blur7_lds staged through LDS): KITTI size, odd, tall and tiny sizes, uniform noise (most
    pixels survive the pre-test) and another parameter set, batched."""
    import torch

    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    monkeypatch.setenv("ORBX_FAST_ROWS", "1" if form == "rows" else "0")
    monkeypatch.setenv("ORBX_FAST_WAVE", "1" if form.startswith("wave") else "0")
    monkeypatch.setenv("ORBX_FAST_WPG", {"wave1": "1", "wave2": "2"}.get(form, "4"))
    monkeypatch.setenv("ORBX_FAST_PSMIN", "20" if form == "wave20" else "24")   # pair stride 20 on KITTI-size cells
    monkeypatch.setenv("ORBX_FAST_TWOPASS", "0" if form == "wave_1pass" else "1")   # iniTh and minTh in one pass
    monkeypatch.setenv("ORBX_BLUR_DOT2", "0" if form == "band_blur1row" else "1")   # k_blur7 one row at a time
    monkeypatch.setenv("ORBX_BLUR_LDS", "1" if form == "wave_blurlds" else "0")     # k_blur7_lds
    monkeypatch.setenv("ORBX_FAST_CELLS", {"wave_cells2": "2", "wave_cells4": "4"}.get(form, "1"))   # k_fast_wave_p
    for shape, nf, kw in (((375, 1242), 2000, {}), ((377, 1243), 800, {}), ((120, 160), 300, {}),
                          ((1000, 200), 800, {}), ((40, 40), 100, {}), ((500, 500), 1000, {}),
                          ((480, 752), 1500, dict(nlevels=5, scale=1.3, ini=25, mn=10)),
                          ((375, 1242), 2000, dict(noise=True)), ((375, 1242), 2000, dict(ini=5, mn=12))):
        if kw.get("noise"):
            imgs = np.stack([S.uniform_noise_image(950 + i) for i in range(3)])
        else:
            imgs = np.stack([S.kitti_like_image(900 + i, rows=shape[0], cols=shape[1]) for i in range(3)])
        ex = pkg.ORBextractor(nf, kw.get("scale", 1.2), kw.get("nlevels", 8), kw.get("ini", 20), kw.get("mn", 7))
        kps, desc, cnt = ex.extract_batch_device(torch.from_numpy(imgs).cuda())
        torch.cuda.synchronize()
        kps, desc, cnt = kps.cpu().numpy(), desc.cpu().numpy(), cnt.cpu().numpy()
        for i in range(len(imgs)):
            ref = O.extract(imgs[i], nfeatures=nf, scale_factor=kw.get("scale", 1.2), nlevels=kw.get("nlevels", 8),
                            ini_th=kw.get("ini", 20), min_th=kw.get("mn", 7))
            n = int(cnt[i])
            kb = kps[i, :n].copy().view(pkg.KP_DTYPE).reshape(-1)
            assert np.array_equal(kb, ref["kps"]) and np.array_equal(desc[i, :n], ref["desc"]), _diff_report(
                kb, desc[i, :n], ref["kps"], ref["desc"])


@pytest.mark.parametrize("fast_wave", [0, 1])
def test_describe_fused_blur_bit_exact(gpu, monkeypatch, fast_wave):
    """k_describe_fb (the 7x7 GaussianBlur done per keypoint on its raw 43x48 window in LDS, no blurred pyramid) gives
    the oracle's descriptors bit for bit: windows that cross the level border (REFLECT_101 on the raw coordinates) occur
    on every level of these images; small and odd sizes, uniform noise, another parameter set, batched."""
    import torch

    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    monkeypatch.setenv("ORBX_DESC_FB", "1")
    monkeypatch.setenv("ORBX_FAST_WAVE", str(fast_wave))
    for shape, nf, kw in (((375, 1242), 2000, {}), ((377, 1243), 800, {}), ((40, 40), 100, {}), ((120, 160), 300, {}),
                          ((1000, 200), 800, {}), ((480, 752), 1500, dict(nlevels=5, scale=1.3, ini=25, mn=10)),
                          ((375, 1242), 2000, dict(noise=True))):
        if kw.get("noise"):
            imgs = np.stack([S.uniform_noise_image(960 + i) for i in range(3)])
        else:
            imgs = np.stack([S.kitti_like_image(920 + i, rows=shape[0], cols=shape[1]) for i in range(3)])
        ex = pkg.ORBextractor(nf, kw.get("scale", 1.2), kw.get("nlevels", 8), kw.get("ini", 20), kw.get("mn", 7))
        kps, desc, cnt = ex.extract_batch_device(torch.from_numpy(imgs).cuda())
        torch.cuda.synchronize()
        kps, desc, cnt = kps.cpu().numpy(), desc.cpu().numpy(), cnt.cpu().numpy()
        for i in range(len(imgs)):
            ref = O.extract(imgs[i], nfeatures=nf, scale_factor=kw.get("scale", 1.2), nlevels=kw.get("nlevels", 8),
                            ini_th=kw.get("ini", 20), min_th=kw.get("mn", 7))
            n = int(cnt[i])
            kb = kps[i, :n].copy().view(pkg.KP_DTYPE).reshape(-1)
            assert np.array_equal(kb, ref["kps"]) and np.array_equal(desc[i, :n], ref["desc"]), _diff_report(
                kb, desc[i, :n], ref["kps"], ref["desc"])
        # the host API (one image per call) takes the same path
        k1, d1 = ex(imgs[0])
        ref = O.extract(imgs[0], nfeatures=nf, scale_factor=kw.get("scale", 1.2), nlevels=kw.get("nlevels", 8),
                        ini_th=kw.get("ini", 20), min_th=kw.get("mn", 7))
        assert np.array_equal(k1, ref["kps"]) and np.array_equal(d1, ref["desc"])
