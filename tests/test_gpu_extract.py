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


@pytest.mark.parametrize("shape,nf", [((1080, 1920), 2000), ((1536, 2048), 4000), ((2160, 3840), 3000)])
def test_large_frames(gpu, shape, nf):
    """HD to 4K camera frames (the reference extracts any image size, ORBextractor.cc:1043-1105)."""
    _, k, _ = _check(S.kitti_like_image(12, rows=shape[0], cols=shape[1]), nfeatures=nf)
    assert len(k) >= 0.9 * nf


@pytest.mark.parametrize("kw", [dict(nlevels=1), dict(nlevels=12, scale=1.1), dict(nlevels=4, scale=2.0),
                                dict(ini=20, mn=20), dict(ini=12, mn=30), dict(ini=0, mn=0), dict(ini=255, mn=60)],
                         ids=["one_level", "12_levels", "scale2", "min_eq_ini", "min_above_ini", "zero_th", "high_th"])
def test_extreme_settings(gpu, kw):
    """Settings a YAML can hold (ORBextractor ctor :410-470, the iniTh -> minTh fallback :812-816): one level, many
    levels, a coarse scale, minThFAST equal to or above iniThFAST, thresholds at 0 and at the u8 top."""
    _check(S.kitti_like_image(13), nfeatures=kw.pop("nf", 1200), **kw)


def test_pyramid_matches_oracle(gpu):
    from oracle import oracle as O
    img = S.kitti_like_image(9)
    ex, _, _ = _check(img)
    ref = O.extract(img, want_pyramid=True)["pyramid"]
    got = ex.mvImagePyramid
    assert len(got) == len(ref)
    for l, (a, b) in enumerate(zip(got, ref)):
        assert a.shape == b.shape and np.array_equal(a, b), f"level {l}"


@pytest.mark.parametrize("shape", [(375, 1242), (2160, 3840)])
def test_batch_device_equals_single(gpu, shape):
    import torch

    import multiagent_orb_slam2_amd as pkg
    imgs = np.stack([S.kitti_like_image(100 + i, rows=shape[0], cols=shape[1]) for i in range(5 if shape[0] < 1000 else 3)])
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


@pytest.mark.parametrize("ring", [1, 2])
def test_split_streams_back_to_back(gpu, ring):
    """orbx_extract_batch_device_split: calls issued back to back without a host sync, the descriptor stage on a
    second stream, so call k+1's front half overlaps call k's descriptor stage.  Every call must equal the
    single-image host API (the extractor orders its own buffer reuse across calls)."""
    import torch

    import multiagent_orb_slam2_amd as pkg
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


def test_describe_batched_slot_ranges(gpu):
    """k_describe_m (2 keypoints per wave, levels straddling a wave) in a batch, so waves also straddle images' slot
    ends; then an odd feature budget and level count: level slot ranges of odd lengths."""
    import torch

    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
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
    _check(S.kitti_like_image(410, rows=240, cols=333), nfeatures=777, nlevels=5, scale=1.3)


@pytest.mark.parametrize("form", ["pipelined", "serial"])
def test_blurred_pyramid_bit_exact(gpu, monkeypatch, form):
    """Every pixel of every blurred level -- not only the windows around keypoints that the descriptor tests see --
    equals the oracle's GaussianBlur(7x7, sigma 2, REFLECT_101) of the oracle's pyramid level
    (ORBextractor.cc:1085-1086): interior strips, strips at a level's left / right edge (REFLECT_101 columns by byte
    selectors), levels under 12 columns, bottom rows, saturation (a constant 255 image blurs to 255 with taps summing to
    257), batched (image index > 0); two streams (default) and every stage on one stream (ORBX_PIPELINE=0)."""
    import torch

    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    monkeypatch.setenv("ORBX_PIPELINE", "0" if form == "serial" else "1")
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


@pytest.mark.parametrize("form", ["twopass", "onepass", "serial"])
def test_fast_kernels_bit_exact(gpu, monkeypatch, form):
    """k_fast_wave (one wave per cell, no barrier) is bit-exact against the oracle in both of its pass modes -- iniTh
    first with a minTh pass only for the cells left empty (default), and one pass at min(iniTh, minTh)
    (ORBX_FAST_TWOPASS=0) -- and with every stage on one stream (ORBX_PIPELINE=0, the roofline_alone schedule): KITTI
    size, odd, tall and tiny sizes, uniform noise (most pixels survive the pre-test), iniTh < minTh and another parameter
    set (pair stride 40 on 1.3-scaled cells), batched."""
    import torch

    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    monkeypatch.setenv("ORBX_FAST_TWOPASS", "0" if form == "onepass" else "1")
    monkeypatch.setenv("ORBX_PIPELINE", "0" if form == "serial" else "1")
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


@pytest.mark.parametrize("form", ["desc_sb", "resize_tail4", "resize_tail3"])
def test_opt_in_forms_bit_exact(gpu, monkeypatch, form):
    """The measured-and-opt-in forms stay bit-exact against the oracle: k_describe_sb (ORBX_DESC_SB=1: the Gaussian blur
    taken at the BRIEF sample points on the matrix cores, no blurred pyramid; ORBextractor.cc:108-147, 1085-1086) and
    k_resize_tail (ORBX_RESIZE_TAIL=l: levels l..7 of ComputePyramid, :1107-1132, in one launch of one workgroup per
    image) -- KITTI size batched, odd and tiny sizes, uniform noise, a 5-level 1.3-scale pyramid, and the host API."""
    import torch

    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    env = {"desc_sb": ("ORBX_DESC_SB", "1"), "resize_tail4": ("ORBX_RESIZE_TAIL", "4"),
           "resize_tail3": ("ORBX_RESIZE_TAIL", "3")}[form]
    monkeypatch.setenv(*env)
    for shape, nf, kw in (((375, 1242), 2000, {}), ((377, 1243), 800, {}), ((40, 40), 100, {}),
                          ((480, 752), 1500, dict(nlevels=5, scale=1.3, ini=25, mn=10)),
                          ((375, 1242), 2000, dict(noise=True))):
        if kw.get("noise"):
            imgs = np.stack([S.uniform_noise_image(960 + i) for i in range(2)])
        else:
            imgs = np.stack([S.kitti_like_image(920 + i, rows=shape[0], cols=shape[1]) for i in range(2)])
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
    ex = pkg.ORBextractor(1500, 1.2, 8, 20, 7, device=0)
    img = S.kitti_like_image(990)
    k, d = ex(img)
    ref = O.extract(img, nfeatures=1500)
    assert np.array_equal(k, ref["kps"]) and np.array_equal(d, ref["desc"]), _diff_report(k, d, ref["kps"], ref["desc"])
    ex.close()


@pytest.mark.parametrize("form", ["default", "unmerged", "forked", "no_graph"])
def test_host_api_schedules(gpu, monkeypatch, form):
    """orbx_extract (host image in, host keypoints out) on each of its schedules: the default (a hipGraph replay, every
    stage on the extractor's stream, FAST / quadtree / blur one launch over all levels), the per-level launch split
    (ORBX_HOST_MERGED=0), the level-0 branch forked onto the side stream (ORBX_HOST_SERIAL=0) and plain stream
    operations every call (ORBX_HOST_GRAPH=0): bit-exact against the oracle over repeated calls of two sizes, including
    a capture per size and replays."""
    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    env = {"unmerged": ("ORBX_HOST_MERGED", "0"), "forked": ("ORBX_HOST_SERIAL", "0"),
           "no_graph": ("ORBX_HOST_GRAPH", "0")}.get(form)
    if env:
        monkeypatch.setenv(*env)
    ex = pkg.ORBextractor(1500, 1.2, 8, 20, 7, device=0)
    for i, (rows, cols) in enumerate([(375, 1242), (375, 1242), (240, 320), (375, 1242), (240, 320)]):
        img = S.kitti_like_image(700 + i, rows=rows, cols=cols)
        k, d = ex(img)
        ref = O.extract(img, nfeatures=1500)
        assert np.array_equal(k, ref["kps"]) and np.array_equal(d, ref["desc"]), _diff_report(k, d, ref["kps"], ref["desc"])
    ex.close()


def test_extract_pair_equals_two_calls(gpu):
    """orbx_extract_pair (the stereo Frame's two extractions from one thread, Frame.cc:78-81) returns what two
    orbx_extract calls return -- and the oracle -- on repeated frames of two sizes; an empty pair gives nothing, one
    extractor for both sides is refused, a short capacity is reported as for orbx_extract."""
    import ctypes as C

    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    exl, exr = pkg.ORBextractor(2000, 1.2, 8, 20, 7), pkg.ORBextractor(2000, 1.2, 8, 20, 7)
    ex1 = pkg.ORBextractor(2000, 1.2, 8, 20, 7)
    for k, (rows, cols) in enumerate([(375, 1242), (375, 1242), (240, 320), (375, 1242)]):
        left = S.kitti_like_image(500 + k, rows=rows, cols=cols)
        right = S.shifted_right_view(left, 500 + k)
        (kl, dl), (kr, dr) = pkg.extract_pair(exl, exr, left, right)
        for img, kk, dd in ((left, kl, dl), (right, kr, dr)):
            k1, d1 = ex1(img)
            assert np.array_equal(kk, k1) and np.array_equal(dd, d1)
            ref = O.extract(img, nfeatures=2000)
            assert np.array_equal(kk, ref["kps"]) and np.array_equal(dd, ref["desc"])
        # the pyramids the stereo step reads are the pair call's
        assert np.array_equal(exr.mvImagePyramid[0], right)
    (a, b), (c, d) = pkg.extract_pair(exl, exr, np.zeros((0, 0), np.uint8), np.zeros((0, 0), np.uint8))
    assert len(a) == len(c) == 0
    with pytest.raises(pkg.OrbxError):
        pkg.extract_pair(exl, exl, left, right)
    kp = np.empty(10, pkg.KP_DTYPE)
    ds = np.empty((10, 32), np.uint8)
    nl, nr = C.c_int(), C.c_int()
    st = exl._lib.orbx_extract_pair(exl._h, exr._h, left.ctypes.data, left.strides[0], right.ctypes.data, right.strides[0],
                                    left.shape[0], left.shape[1], kp.ctypes.data, ds.ctypes.data, 10, C.byref(nl),
                                    kp.ctypes.data, ds.ctypes.data, 10, C.byref(nr))
    assert st == pkg.orbx.ORBX_ERR_CAPACITY and nl.value > 10


def test_roi_views_with_a_row_step(gpu):
    """A crop of a larger frame (a cv::Mat ROI: contiguous rows at the parent's step) goes in as it is, with its step,
    through ORBextractor, orbx_extract_pair and orbx_stereo_frame: the same results as a contiguous copy and the oracle."""
    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    big = S.kitti_like_image(14, rows=420, cols=1300)
    bigr = S.shifted_right_view(big, 14)
    roi, roir = big[17:392, 29:1271], bigr[17:392, 29:1271]
    assert roi.shape == (375, 1242) and not roi.flags.c_contiguous and roi.strides == (1300, 1)
    ex, k, d = _check(roi)
    exr = pkg.ORBextractor(2000, 1.2, 8, 20, 7)
    (kl, dl), (kr, dr) = pkg.extract_pair(ex, exr, roi, roir)
    (kl2, dl2), (kr2, dr2) = pkg.extract_pair(ex, exr, roi.copy(), roir.copy())
    assert np.array_equal(kl, k) and np.array_equal(dl, d)
    assert np.array_equal(kl, kl2) and np.array_equal(kr, kr2) and np.array_equal(dr, dr2)
    m = pkg.ORBmatcher()
    _, _, ur, dp = m.StereoFrame(ex, exr, roi, roir, 386.1448, 0.537165)
    _, _, ur2, dp2 = m.StereoFrame(ex, exr, roi.copy(), roir.copy(), 386.1448, 0.537165)
    assert ur.tobytes() == ur2.tobytes() and dp.tobytes() == dp2.tobytes() and (dp > 0).sum() > 0.2 * len(k)
    ref = O.extract(roir, nfeatures=2000)
    assert np.array_equal(kr, ref["kps"]) and np.array_equal(dr, ref["desc"])
