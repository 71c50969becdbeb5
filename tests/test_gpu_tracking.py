"""The bench's tracking and Fuse stages (multiagent.FrameTracker, multiagent.LocalFuse) against the oracle run the way the
reference's callers run the matchers:
  - TrackWithMotionModel: the last frame's stereo MapPoints (UnprojectStereo + the Frame form of the MapPoint
    constructor) projected (SearchByProjection(F, LastF), src/ORBmatcher.cc:1363-1392) and searched with
    ORBmatcher(0.9, true), th 7; then SearchLocalPoints: isInFrustum(0.5) for the points not matched yet and
    SearchByProjection(F, vpLocalMapPoints, th 1) with ORBmatcher(0.8), keypoints holding a MapPoint excluded
    (src/Tracking.cc:882-904, :1160-1205);
  - SearchInNeighbors' Fuse both ways (src/LocalMapping.cc:486-520, ORBmatcher::Fuse :830-951) with th 3.
Frames are extracted, stereo-matched and refined on the GPU; the oracle reads the same keypoints, descriptors and
stereo results, so every query index and match count must be identical."""
import numpy as np
import pytest

from multiagent_orb_slam2_amd import synthetic as S

pytestmark = pytest.mark.gpu

ROWS, COLS, BF, FX = 375, 1242, 386.1448, 718.856


def _frames(B, seed0, seeds=None):
    import torch

    import multiagent_orb_slam2_amd as pkg
    seeds = seeds or [seed0 + i for i in range(B)]
    lefts = [S.kitti_like_image(s) for s in seeds]
    rights = [S.shifted_right_view(l, s) for s, l in zip(seeds, lefts)]
    ex = pkg.ORBextractor(2000, 1.2, 8, 20, 7)
    kps, desc, cnt = ex.extract_batch_device(torch.from_numpy(np.stack(lefts + rights)).cuda())
    return ex, kps, desc, cnt


def _geometry():
    import bench
    return bench.Geometry(dict(bench.CONFIGS["kitti"]), 12)


def test_frame_tracker_vs_oracle(gpu):
    import torch

    import multiagent_orb_slam2_amd as pkg
    from multiagent_orb_slam2_amd import multiagent as MA
    from multiagent_orb_slam2_amd.orbx import (PROJ_LASTFRAME, PROJ_MAPPOINTS, PROJ_QUERY_DTYPE, QF_BLOCKS, QF_SKIP,
                                               ProjParams)
    from oracle import oracle as O
    B = 3
    ex, kps, desc, cnt = _frames(B, 880)
    cap = kps.shape[1]
    scale, isg = ex.GetScaleFactors(), ex.GetInverseScaleSigmaSquares()
    geo = _geometry()
    twc_last, v_lf, v_mp = geo.tracking_views()
    log_sf = float(np.float32(np.log(1.2)))
    grid = pkg.frame_grid(0, 0, COLS, ROWS)
    m = pkg.ORBmatcher(0.6, True)
    tr = MA.FrameTracker(pkg.ORBmatcher(0.9, True), B, cap, grid, geo.camera, BF, scale, log_sf, kps.device, 1, twc_last,
                         v_lf, v_mp, isg)
    bi, _ = m.stereo_match_batch_device(kps[:B], desc[:B], cnt[:B], kps[B:], desc[B:], cnt[B:], cap, scale, ROWS, BF, BF / FX)
    pyr = ex.pyramid_device()
    m.stereo_refine_batch_device(kps[:B], cnt[:B], kps[B:], bi, pyr, 0, pyr, B, BF, BF / FX, out=tr.stereo_out(0))
    qi1, nm1, qi2, nm2 = tr.run(0, kps[:B].contiguous(), desc[:B].contiguous(), cnt[:B])
    torch.cuda.synchronize()
    qi1, nm1, qi2, nm2 = (t.cpu().numpy() for t in (qi1, nm1, qi2, nm2))
    ur, depth = (t.cpu().numpy() for t in tr.stereo_out(0))
    kh, dh, ch = kps.cpu().numpy(), desc.cpu().numpy(), cnt.cpu().numpy()
    p_lf = ProjParams.make(PROJ_LASTFRAME, 100, 0.9, True, isg)
    p_mp = ProjParams.make(PROJ_MAPPOINTS, 100, 0.8, False, isg)
    tot1 = tot2 = dropped = 0
    for i in range(B):
        n = int(ch[i])
        k = kh[i, :n].copy().view(pkg.KP_DTYPE).reshape(-1)
        d = dh[i, :n]
        pts = O.stereo_mappoints(k, depth[i, :n], twc_last, geo.camera, scale, QF_BLOCKS)
        last = pts.copy()
        last["flags"][1::2] |= QF_SKIP                                  # the last frame holds the even keypoints' points
        q1 = O.project(PROJ_LASTFRAME, last, v_lf, scale, log_sf).view(PROJ_QUERY_DTYPE).reshape(-1)
        r1, ri1, _, own1 = O.proj_search(p_lf, grid, q1, d, k, d, uright=ur[i, :n])
        assert nm1[i] == r1 and np.array_equal(qi1[i, :n], ri1), f"motion-model search, frame {i}"
        # SearchLocalPoints skips the MapPoints in mCurrentFrame.mvpMapPoints (Tracking.cc:1158-1174): assigned AND
        # kept by the rotation filter (ORBmatcher.cc:1456-1466 resets the ones it drops, owner -2)
        fnd = MA.found_in_frame(ri1, own1)
        dropped += int(((ri1 >= 0) & ~fnd).sum())
        pts["flags"][fnd] |= QF_SKIP
        q2 = O.project(PROJ_MAPPOINTS, pts, v_mp, scale, log_sf).view(PROJ_QUERY_DTYPE).reshape(-1)
        r2, ri2, _, _ = O.proj_search(p_mp, grid, q2, d, k, d, uright=ur[i, :n], blocked=(own1 >= 0).astype(np.uint8))
        assert nm2[i] == r2 and np.array_equal(qi2[i, :n], ri2), f"local-map search, frame {i}"
        tot1, tot2 = tot1 + r1, tot2 + r2
    assert tot1 > 100 * B and tot2 > 100 * B, (tot1, tot2)
    # the case the owner rule exists for: motion-model matches the rotation filter dropped are searched again
    assert dropped > 0, "no rotation-filter drops in these frames: the local-map skip rule is not exercised"


def test_local_fuse_vs_oracle(gpu):
    import torch

    import multiagent_orb_slam2_amd as pkg
    from multiagent_orb_slam2_amd import multiagent as MA
    from multiagent_orb_slam2_amd.orbx import PROJ_FUSE, PROJ_QUERY_DTYPE, QF_BLOCKS, ProjParams
    from oracle import oracle as O
    slots = 6
    ex, kps, desc, cnt = _frames(slots, 940, seeds=[940, 941, 942, 943, 944, 944])   # slot 5 = slot 4 re-observed
    cap, dev = kps.shape[1], kps.device
    kl, dl = kps[:slots].contiguous(), desc[:slots].contiguous()
    scale, isg = ex.GetScaleFactors(), ex.GetInverseScaleSigmaSquares()
    m = pkg.ORBmatcher(0.6, True)
    bi, _ = m.stereo_match_batch_device(kps[:slots], desc[:slots], cnt[:slots], kps[slots:], desc[slots:], cnt[slots:], cap,
                                        scale, ROWS, BF, BF / FX)
    pyr = ex.pyramid_device()
    ur, depth = m.stereo_refine_batch_device(kps[:slots], cnt[:slots], kps[slots:], bi, pyr, 0, pyr, slots, BF, BF / FX)
    valid = (torch.arange(cap, device=dev)[None, :] < cnt[:slots, None]).to(torch.uint8)
    store = pkg.KfStore.from_fields(cap, desc=(dl, cap * 32), kps=(kl, cap * 28), valid=(valid, cap))
    geo = _geometry()
    twc, views = geo.slot_tables(slots, 1, slots)
    twc[5], views[5] = twc[4], views[4]                     # ... from the same pose: its MapPoints fuse into slot 4
    log_sf = float(np.float32(np.log(1.2)))
    grid = pkg.frame_grid(0, 0, COLS, ROWS)
    fu = MA.LocalFuse(m, store, slots, cap, grid, geo.camera, BF, scale, log_sf, isg, twc, views, dev)
    rows = torch.arange(slots, dtype=torch.int64, device=dev)
    fu.add_keyframes(range(0, slots), kl, dl, cnt[:slots], ur, depth, rows)
    new = np.array([4, 5])
    nb = np.array([[3, 2, 1], [4, 3, -1]])
    (qa, na), (qb, nb_) = fu.run(new, nb)
    torch.cuda.synchronize()
    qa, na, qb, nb_ = (t.cpu().numpy() for t in (qa, na, qb, nb_))
    kh, dh, ch = kl.cpu().numpy(), dl.cpu().numpy(), cnt.cpu().numpy()
    urh, dph = ur.cpu().numpy(), depth.cpu().numpy()
    P = ProjParams.make(PROJ_FUSE, 50, 0.6, False, isg)

    def kf(s):
        n = int(ch[s])
        k = kh[s, :n].copy().view(pkg.KP_DTYPE).reshape(-1)
        return k, dh[s, :n], urh[s, :n], O.stereo_mappoints(k, dph[s, :n], twc[s], geo.camera, scale, QF_BLOCKS)

    found = 0
    for j, s in enumerate(new):
        k1, d1, u1, p1 = kf(s)
        for c in range(nb.shape[1]):
            p = j * nb.shape[1] + c
            t = nb[j, c]
            if t < 0:
                assert na[p] == 0 and nb_[p] == 0
                continue
            k2, d2, u2, p2 = kf(t)
            q = O.project(PROJ_FUSE, p1, views[t], scale, log_sf).view(PROJ_QUERY_DTYPE).reshape(-1)
            r, ri, _, _ = O.proj_search(P, grid, q, d1, k2, d2, uright=u2)
            assert na[p] == r and np.array_equal(qa[p, :len(p1)], ri), (s, t, "current into neighbour")
            q = O.project(PROJ_FUSE, p2, views[s], scale, log_sf).view(PROJ_QUERY_DTYPE).reshape(-1)
            r2, ri2, _, _ = O.proj_search(P, grid, q, d2, k1, d1, uright=u1)
            assert nb_[p] == r2 and np.array_equal(qb[p, :len(p2)], ri2), (s, t, "neighbour into current")
            found += r + r2
    assert na[3] > 500 and nb_[3] > 500, (na, nb_)          # slot 5 <-> slot 4: the same scene from the same pose


def test_proj_found_device_rule(gpu):
    """orbx_proj_found_device against the oracle's rule (oracle.found_in_frame) on random assignments: unmatched
    queries (-1), queries whose keypoint the rotation filter released (owner -2) or re-assigned to another query, and
    the blocked bytes (owner >= 0); nq != n and one empty set."""
    import torch

    import multiagent_orb_slam2_amd as pkg
    from oracle.oracle import found_in_frame
    rng = np.random.default_rng(7)
    S_, nq, n = 5, 700, 450
    q_idx = np.full((S_, nq), -1, np.int32)
    owner = np.full((S_, n), -1, np.int32)
    for s in range(1, S_):                       # set 0: nothing matched
        qs = rng.choice(nq, size=300, replace=False)
        ks = rng.choice(n, size=300, replace=False)
        q_idx[s, qs] = ks
        owner[s, ks] = qs
        drop = rng.choice(300, size=40, replace=False)
        owner[s, ks[drop[:20]]] = -2             # released by the rotation filter
        owner[s, ks[drop[20:]]] = qs[(drop[20:] + 1) % 300]   # held by another query
    m = pkg.ORBmatcher(0.9, True)
    dq, do = torch.from_numpy(q_idx).cuda(), torch.from_numpy(owner).cuda()
    found = torch.empty((S_, nq), dtype=torch.int32, device="cuda")
    blocked = torch.empty((S_, n), dtype=torch.bool, device="cuda")
    m.proj_found_device(dq, do, found, blocked=blocked)
    torch.cuda.synchronize()
    for s in range(S_):
        want = np.where(found_in_frame(q_idx[s], owner[s]), 0, -1)
        assert np.array_equal(found[s].cpu().numpy(), want), s
        assert np.array_equal(blocked[s].cpu().numpy(), owner[s] >= 0), s
    assert (found[1:] == 0).sum().item() == 4 * 260
