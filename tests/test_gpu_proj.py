"""GPU parity of the keypoint grid and the projection / radius matchers against the
oracle (oracle/proj_oracle.cpp): per-query results, final MapPoint assignment and nmatches identical."""
import ctypes as C

import numpy as np
import pytest

from proj_cases import MODES, make_case

pytestmark = pytest.mark.gpu


def _check(c, got):
    from oracle import oracle as O
    ref = O.proj_search(c["params"], c["grid"], c["queries"], c["qdesc"], c["kps"], c["desc"], c["uright"], c["blocked"])
    assert got[0] == ref[0], ("nmatches", got[0], ref[0])
    for g, r, name in zip(got[1:], ref[1:], ("q_idx", "q_dist", "owner")):
        assert np.array_equal(g, r), name
    return ref


@pytest.mark.parametrize("mode", sorted(MODES))
@pytest.mark.parametrize("dense", [False, True])
def test_proj_search_modes(gpu, mode, dense):
    import multiagent_orb_slam2_amd as pkg
    m = pkg.ORBmatcher(0.8, True)
    for seed in (11, 12, 13):
        c = make_case(seed, MODES[mode], n_target=900, n_query=700, dense=dense)
        got = m.proj_search(c["params"], c["grid"], c["queries"], c["qdesc"], c["kps"], c["desc"], c["uright"],
                            c["blocked"])
        ref = _check(c, got)
        assert ref[0] > 0


@pytest.mark.parametrize("mode", ["mappoints", "lastframe", "keyframe"])
def test_proj_search_kitti_size(gpu, mode):
    """KITTI-size target (2000 keypoints, 1242x375) and a local map of 4000 projected points."""
    import multiagent_orb_slam2_amd as pkg
    m = pkg.ORBmatcher(0.8, True)
    c = make_case(21, MODES[mode], n_target=2000, n_query=4000, W=1242, H=375)
    got = m.proj_search(c["params"], c["grid"], c["queries"], c["qdesc"], c["kps"], c["desc"], c["uright"], c["blocked"])
    _check(c, got)


@pytest.mark.parametrize("mode", ["mappoints", "lastframe", "fuse"])
@pytest.mark.parametrize("size", [(1920, 1080, 3000, 5000), (3840, 2160, 4000, 8000)], ids=["1080p", "4k"])
def test_proj_search_large_frames(gpu, mode, size):
    """Camera frames of 1920 x 1080 and 3840 x 2160 with their 64 x 48 grid (Frame.cc:230-245: cells of 30-80 px) and
    a local map of 5000-8000 projected points: whichever LDS plan the launch picks, the oracle's assignment."""
    import multiagent_orb_slam2_amd as pkg
    W, H, nt, nq = size
    m = pkg.ORBmatcher(0.8, True)
    c = make_case(71, MODES[mode], n_target=nt, n_query=nq, W=W, H=H)
    got = m.proj_search(c["params"], c["grid"], c["queries"], c["qdesc"], c["kps"], c["desc"], c["uright"], c["blocked"])
    assert _check(c, got)[0] > 0


@pytest.mark.parametrize("mode", ["lastframe", "mappoints", "fuse", "best"])
def test_proj_search_lds_plans(gpu, mode):
    """The search's other LDS plans: a grid too fine to stage (320 x 240 cells: cell starts and keypoints read from
    memory), and a query set too large for candidate lists (20000 queries: every fixed-point round walks again); the
    dense case overflows the lists of the default plan."""
    import multiagent_orb_slam2_amd as pkg
    from multiagent_orb_slam2_amd.orbx import frame_grid
    m = pkg.ORBmatcher(0.8, True)
    c = make_case(61, MODES[mode], n_target=1500, n_query=1200, dense=True)
    c["grid"] = frame_grid(0.0, 0.0, 640.0, 480.0, 320, 240)
    got = m.proj_search(c["params"], c["grid"], c["queries"], c["qdesc"], c["kps"], c["desc"], c["uright"], c["blocked"])
    assert _check(c, got)[0] > 0
    c = make_case(62, MODES[mode], n_target=2000, n_query=20000, dense=True)
    got = m.proj_search(c["params"], c["grid"], c["queries"], c["qdesc"], c["kps"], c["desc"], c["uright"], c["blocked"])
    assert _check(c, got)[0] > 0


def test_proj_search_named_wrappers(gpu):
    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    m = pkg.ORBmatcher(0.9, True)
    c = make_case(31, MODES["init"], n_target=600, n_query=600, dense=True)
    got = m.SearchForInitialization(c["grid"], c["queries"], c["qdesc"], c["kps"], c["desc"])
    ref = O.proj_search(c["params"], c["grid"], c["queries"], c["qdesc"], c["kps"], c["desc"])
    assert got[0] == ref[0] and np.array_equal(got[1], ref[1])
    c = make_case(32, MODES["keyframe"], n_target=600, n_query=600)
    got = m.SearchByProjection_KeyFrame(c["grid"], c["queries"], c["qdesc"], c["kps"], c["desc"], c["blocked"], 64)
    _check(c, got)


def test_proj_search_empty(gpu):
    import multiagent_orb_slam2_amd as pkg
    m = pkg.ORBmatcher(0.8, True)
    c = make_case(41, MODES["lastframe"], n_target=50, n_query=40)
    got = m.proj_search(c["params"], c["grid"], c["queries"][:0], c["qdesc"][:0], c["kps"], c["desc"], c["uright"])
    assert got[0] == 0 and len(got[1]) == 0 and (got[3] == -1).all()
    got = m.proj_search(c["params"], c["grid"], c["queries"], c["qdesc"], c["kps"][:0], c["desc"][:0])
    assert got[0] == 0 and (got[1] == -1).all()
    # an empty problem batch (an empty slice's data pointer may be NULL: r5bab) is a no-op, not a bad argument
    import torch
    m.proj_search_batch_device(c["params"], c["grid"], torch.empty((0,), dtype=torch.uint8, device="cuda"), 64, 64)
    assert pkg.orbx.load_library().orbx_proj_search_batch_device(m._h, C.byref(c["params"]), c["grid"], None, 0, 64, 64,
                                                                  None) == 0


def test_grid_build_clustered_and_empty(gpu):
    """The grid's CSR arrays (cell starts, indices ascending inside a cell) when keypoints pile into a few cells (the
    counting kernel's per-cell ordering at its longest), when some fall outside the grid, and for an empty set."""
    import torch

    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    m = pkg.ORBmatcher(0.8, True)
    grid = make_case(7, MODES["mappoints"])["grid"]
    rng = np.random.default_rng(11)
    cap = 2100
    sets = []
    k = np.zeros(cap, pkg.KP_DTYPE)                      # 2100 keypoints in 3 cells
    k["x"] = rng.choice([100.5, 101.0, 300.25], cap).astype(np.float32)
    k["y"] = rng.choice([50.0, 50.5, 200.75], cap).astype(np.float32)
    sets.append(k)
    k = np.zeros(cap, pkg.KP_DTYPE)                      # uniform, a tenth outside the image bounds
    k["x"] = rng.uniform(-60, 700, cap).astype(np.float32)
    k["y"] = rng.uniform(-40, 520, cap).astype(np.float32)
    sets.append(k)
    sets.append(np.zeros(cap, pkg.KP_DTYPE))            # counted as 0
    kps = torch.from_numpy(np.stack([s_.view(np.uint8).reshape(cap, 28) for s_ in sets])).cuda()
    counts = torch.tensor([cap, cap - 37, 0], dtype=torch.int32, device="cuda")
    cs, ci = m.grid_build_device(grid, kps, counts)
    torch.cuda.synchronize()
    for i, (s_, n) in enumerate(zip(sets, [cap, cap - 37, 0])):
        rcs, rci = O.grid_assign(s_[:n], grid)
        assert np.array_equal(cs[i].cpu().numpy(), rcs)
        assert np.array_equal(ci[i, :rcs[-1]].cpu().numpy(), rci)


def test_grid_build_and_batched_search_device(gpu):
    """orbx_grid_build_device + orbx_proj_search_batch_device over several (query set, view) problems."""
    import torch

    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    m = pkg.ORBmatcher(0.8, True)
    cases = [make_case(50 + i, MODES["mappoints"], n_target=700 + 50 * i, n_query=500 + 40 * i) for i in range(4)]
    cap = max(len(c["kps"]) for c in cases)
    B = len(cases)
    dev = torch.device("cuda", 0)
    kps = torch.zeros((B, cap, 28), dtype=torch.uint8)
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8)
    ur = torch.full((B, cap), -1.0)
    bl = torch.zeros((B, cap), dtype=torch.uint8)
    for i, c in enumerate(cases):
        n = len(c["kps"])
        kps[i, :n] = torch.from_numpy(c["kps"].view(np.uint8).reshape(n, 28))
        desc[i, :n] = torch.from_numpy(c["desc"])
        ur[i, :n] = torch.from_numpy(c["uright"])
        bl[i, :n] = torch.from_numpy(c["blocked"])
    kps, desc, ur, bl = kps.to(dev), desc.to(dev), ur.to(dev), bl.to(dev)
    counts = torch.tensor([len(c["kps"]) for c in cases], dtype=torch.int32, device=dev)
    grid = cases[0]["grid"]
    cs, ci = m.grid_build_device(grid, kps, counts)
    torch.cuda.synchronize()
    for i, c in enumerate(cases):                       # the grid itself is exact
        rcs, rci = O.grid_assign(c["kps"], grid)
        assert np.array_equal(cs[i].cpu().numpy(), rcs)
        assert np.array_equal(ci[i, :rcs[-1]].cpu().numpy(), rci)
    nqmax = max(len(c["queries"]) for c in cases)
    qs = torch.zeros((B, nqmax, 40), dtype=torch.uint8)
    qd = torch.zeros((B, nqmax, 32), dtype=torch.uint8)
    for i, c in enumerate(cases):
        nq = len(c["queries"])
        qs[i, :nq] = torch.from_numpy(c["queries"].view(np.uint8).reshape(nq, 40))
        qd[i, :nq] = torch.from_numpy(c["qdesc"])
    qs, qd = qs.to(dev), qd.to(dev)
    q_idx = torch.empty((B, nqmax), dtype=torch.int32, device=dev)
    q_dist = torch.empty((B, nqmax), dtype=torch.int32, device=dev)
    owner = torch.empty((B, cap), dtype=torch.int32, device=dev)
    nm = torch.empty((B,), dtype=torch.int32, device=dev)
    probs = (pkg.ProjProblem * B)()
    for i, c in enumerate(cases):
        probs[i] = pkg.ProjProblem(qs[i].data_ptr(), qd[i].data_ptr(), len(c["queries"]), kps[i].data_ptr(),
                                   desc[i].data_ptr(), ur[i].data_ptr(), bl[i].data_ptr(), len(c["kps"]),
                                   cs[i].data_ptr(), ci[i].data_ptr(), q_idx[i].data_ptr(), q_dist[i].data_ptr(),
                                   owner[i].data_ptr(), nm[i:i + 1].data_ptr())
    dprobs = torch.frombuffer(bytearray(bytes(probs)), dtype=torch.uint8).to(dev)
    m.proj_search_batch_device(cases[0]["params"], grid, dprobs, cap, nqmax)
    torch.cuda.synchronize()
    for i, c in enumerate(cases):
        nq, n = len(c["queries"]), len(c["kps"])
        got = (int(nm[i]), q_idx[i, :nq].cpu().numpy(), q_dist[i, :nq].cpu().numpy(), owner[i, :n].cpu().numpy())
        _check(c, got)
    # a caller that understates max_nq / max_n (the LDS plan's bounds): the problems above them are not searched
    # (q_idx -1, nmatches -1) and the others are unaffected -- never an LDS overrun
    for max_n, max_nq in ((cap, 560), (800, nqmax)):
        m.proj_search_batch_device(cases[0]["params"], grid, dprobs, max_n, max_nq)
        torch.cuda.synchronize()
        for i, c in enumerate(cases):
            nq, n = len(c["queries"]), len(c["kps"])
            if nq > max_nq or n > max_n:
                assert int(nm[i]) == -1 and bool((q_idx[i, :nq] == -1).all()), (i, max_n, max_nq)
            else:
                got = (int(nm[i]), q_idx[i, :nq].cpu().numpy(), q_dist[i, :nq].cpu().numpy(), owner[i, :n].cpu().numpy())
                _check(c, got)


@pytest.mark.parametrize("seed", range(4))
def test_projection_step_bit_exact(gpu, seed):
    """orbx_proj_project (host form) and orbx_proj_project_device (a batch of views, ragged counts) give the oracle's
    queries bit for bit for LASTFRAME, MAPPOINTS (isInFrustum) and FUSE."""
    import torch

    import multiagent_orb_slam2_amd as pkg
    from multiagent_orb_slam2_amd.orbx import MAP_POINT_DTYPE, PROJ_FUSE, PROJ_LASTFRAME, PROJ_MAPPOINTS, VIEW_DTYPE
    from oracle import oracle as O
    from proj_cases import make_projection_case
    m = pkg.ORBmatcher(0.8, True)
    cases = [make_projection_case(10 * seed + k, n=500 + 37 * k) for k in range(3)]
    cap = max(len(c[0]) for c in cases)
    sc, lsf = cases[0][2], cases[0][3]
    for mode in (PROJ_LASTFRAME, PROJ_MAPPOINTS, PROJ_FUSE):
        pts = np.zeros((len(cases), cap), MAP_POINT_DTYPE)
        views = np.zeros(len(cases), VIEW_DTYPE)
        for i, (p, v, _, _) in enumerate(cases):
            pts[i, :len(p)] = p
            views[i] = v
        dp = torch.from_numpy(pts.view(np.uint8).reshape(len(cases), cap, 48)).cuda()
        dv = torch.from_numpy(views.view(np.uint8).reshape(len(cases), 112)).cuda()
        cnt = torch.tensor([len(c[0]) for c in cases], dtype=torch.int32, device="cuda")
        out = m.proj_project_device(mode, dp, cnt, dv, sc, lsf)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        for i, (p, v, _, _) in enumerate(cases):
            ref = O.project(mode, p, v, sc, lsf)
            assert np.array_equal(got[i, :len(p)], ref), f"mode {mode} view {i}"
            tail = got[i, len(p):].copy().view(pkg.PROJ_QUERY_DTYPE).reshape(-1)
            assert (tail["flags"] & 1).all(), "rows past the count must be skipped"
            host = m.proj_project(mode, p, v, sc, lsf).view(np.uint8).reshape(-1, 40)
            assert np.array_equal(host, ref), f"host form, mode {mode} view {i}"
        # many views of one point set (Fuse's shape): view k projects set vp[k]
        vp = torch.tensor([2, 0, 0, 1, 2], dtype=torch.int32, device="cuda")
        vv = np.stack([views[j] for j in (0, 1, 2, 2, 1)])
        dvv = torch.from_numpy(vv.view(np.uint8).reshape(5, 112)).cuda()
        outv = m.proj_project_device(mode, dp, cnt, dvv, sc, lsf, view_points=vp).cpu().numpy()
        for k, (s_, vix) in enumerate(zip((2, 0, 0, 1, 2), (0, 1, 2, 2, 1))):
            p = cases[s_][0]
            ref = O.project(mode, p, vv[k], sc, lsf)
            assert np.array_equal(outv[k, :len(p)], ref), f"mode {mode} indirect view {k}"


def test_stereo_mappoints_and_found_skip_bit_exact(gpu):
    """orbx_stereo_mappoints_device over a batch of frames equals the oracle, and orbx_proj_project_device with a
    'found' array skips exactly the points already matched (Tracking::SearchLocalPoints)."""
    import torch

    import multiagent_orb_slam2_amd as pkg
    from multiagent_orb_slam2_amd.orbx import PROJ_MAPPOINTS, QF_BLOCKS, VIEW_DTYPE
    from oracle import oracle as O
    from proj_cases import SCALE, make_projection_case, stereo_frame_case
    m = pkg.ORBmatcher(0.8, True)
    frames = [stereo_frame_case(50 + i, n=600 + 50 * i) for i in range(3)]
    cap = max(len(f[0]) for f in frames)
    kp = np.zeros((3, cap), pkg.KP_DTYPE)
    dp = np.zeros((3, cap), np.float32)
    tw = np.zeros((3, 12), np.float32)
    for i, (k, d, t, cam) in enumerate(frames):
        kp[i, :len(k)], dp[i, :len(k)], tw[i] = k, d, t
    dk = torch.from_numpy(kp.view(np.uint8).reshape(3, cap, 28)).cuda()
    dd, dt = torch.from_numpy(dp).cuda(), torch.from_numpy(tw).cuda()
    cnt = torch.tensor([len(f[0]) for f in frames], dtype=torch.int32, device="cuda")
    pts = m.stereo_mappoints_device(dk, dd, cnt, dt, frames[0][3], SCALE, QF_BLOCKS)
    torch.cuda.synchronize()
    got = pts.cpu().numpy()
    for i, (k, d, t, cam) in enumerate(frames):
        ref = O.stereo_mappoints(k, d, t, cam, SCALE, QF_BLOCKS)
        assert np.array_equal(got[i, :len(k)].reshape(-1), ref.view(np.uint8).reshape(-1)), f"frame {i}"
    # projection with 'found': the same points seen from a view close to frame 0's
    _, view, _, lsf = make_projection_case(3)
    views = np.zeros(3, VIEW_DTYPE)
    for i in range(3):
        views[i] = view
    found = torch.full((3, cap), -1, dtype=torch.int32, device="cuda")
    found[:, ::3] = 5
    dv = torch.from_numpy(views.view(np.uint8).reshape(3, 112)).cuda()
    q = m.proj_project_device(PROJ_MAPPOINTS, pts, cnt, dv, SCALE, lsf, found=found).cpu().numpy()
    for i, (k, d, t, cam) in enumerate(frames):
        p = O.stereo_mappoints(k, d, t, cam, SCALE, QF_BLOCKS)
        p["flags"][::3] |= 1
        assert np.array_equal(q[i, :len(k)], O.project(PROJ_MAPPOINTS, p, view, SCALE, lsf)), f"frame {i}"


def test_keyframe_prep_equals_oracle(gpu):
    """orbx_keyframe_prep_device (a keyframe's MapPoints and grid in one workgroup) equals the oracle's stereo MapPoints
    and Frame::AssignFeaturesToGrid, bit for bit, including an empty keyframe."""
    import torch

    import multiagent_orb_slam2_amd as pkg
    from multiagent_orb_slam2_amd.orbx import QF_BLOCKS
    from oracle import oracle as O
    from proj_cases import SCALE, stereo_frame_case
    m = pkg.ORBmatcher(0.8, True)
    grid = make_case(7, MODES["mappoints"])["grid"]
    frames = [stereo_frame_case(70 + i, n=900 + 300 * i) for i in range(3)]
    cap = max(len(f[0]) for f in frames)
    B = 4
    kp = np.zeros((B, cap), pkg.KP_DTYPE)
    dp = np.zeros((B, cap), np.float32)
    tw = np.zeros((B, 12), np.float32)
    for i, (k, d, t, cam) in enumerate(frames):
        kp[i, :len(k)], dp[i, :len(k)], tw[i] = k, d, t
    ns = [len(f[0]) for f in frames] + [0]
    dk = torch.from_numpy(kp.view(np.uint8).reshape(B, cap, 28)).cuda()
    dd, dt = torch.from_numpy(dp).cuda(), torch.from_numpy(tw).cuda()
    cnt = torch.tensor(ns, dtype=torch.int32, device="cuda")
    pts = torch.zeros((B, cap, 48), dtype=torch.uint8, device="cuda")
    cs = torch.full((B, grid.cols * grid.rows + 1), -7, dtype=torch.int32, device="cuda")
    ci = torch.full((B, cap), -7, dtype=torch.int32, device="cuda")
    m.keyframe_prep_device(grid, dk, dd, cnt, dt, frames[0][3], SCALE, QF_BLOCKS, pts, cs, ci)
    torch.cuda.synchronize()
    got, gcs, gci = pts.cpu().numpy(), cs.cpu().numpy(), ci.cpu().numpy()
    for i, n in enumerate(ns):
        k = kp[i, :n]
        if n:
            ref = O.stereo_mappoints(k, dp[i, :n], tw[i], frames[0][3], SCALE, QF_BLOCKS)
            assert np.array_equal(got[i, :n].reshape(-1), ref.view(np.uint8).reshape(-1)), f"keyframe {i}"
        rcs, rci = O.grid_assign(k, grid)
        assert np.array_equal(gcs[i], rcs), f"keyframe {i} grid"
        assert np.array_equal(gci[i, :rcs[-1]], rci), f"keyframe {i} grid"
    # the same through the two-launch form
    pts2 = m.stereo_mappoints_device(dk, dd, cnt, dt, frames[0][3], SCALE, QF_BLOCKS)
    cs2, ci2 = m.grid_build_device(grid, dk, cnt)
    torch.cuda.synchronize()
    for i, n in enumerate(ns):
        assert torch.equal(pts2[i, :n], pts[i, :n]) and torch.equal(cs2[i], cs[i])
        assert torch.equal(ci2[i, :int(cs[i, -1])], ci[i, :int(cs[i, -1])])


@pytest.mark.parametrize("mode", ["lastframe", "mappoints", "fuse", "best"])
def test_search_with_grid_built_inside(gpu, mode):
    """orbx_proj_search_grid_batch_device: each problem's grid built inside its search from the first grid_counts[p]
    keypoints -- the written cell_start / cell_idx equal the oracle's AssignFeaturesToGrid and the search results equal
    the oracle's, for problems whose target arrays hold more rows than are counted (rows past the count carry keypoints
    that must not enter the grid) and for an empty problem."""
    import torch

    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    m = pkg.ORBmatcher(0.8, True)
    cases = [make_case(80 + i, MODES[mode], n_target=600 + 90 * i, n_query=400 + 30 * i) for i in range(3)]
    cases.append(make_case(90, MODES[mode], n_target=8, n_query=50))
    B = len(cases)
    cap = max(len(c["kps"]) for c in cases) + 64
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(5)
    junk = np.zeros(cap, pkg.KP_DTYPE)                  # rows past every count: keypoints inside the image
    junk["x"] = rng.uniform(20, 600, cap).astype(np.float32)
    junk["y"] = rng.uniform(20, 460, cap).astype(np.float32)
    kps = torch.from_numpy(np.tile(junk.view(np.uint8).reshape(1, cap, 28), (B, 1, 1)))
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8)
    ur = torch.full((B, cap), -1.0)
    bl = torch.zeros((B, cap), dtype=torch.uint8)
    ncount = []
    for i, c in enumerate(cases):
        n = len(c["kps"]) if i < 3 else 0               # the last problem counts none of its keypoints
        ncount.append(n)
        kps[i, :len(c["kps"])] = torch.from_numpy(c["kps"].view(np.uint8).reshape(len(c["kps"]), 28))
        desc[i, :len(c["kps"])] = torch.from_numpy(c["desc"])
        if c["uright"] is not None:
            ur[i, :len(c["kps"])] = torch.from_numpy(c["uright"])
        if c["blocked"] is not None:
            bl[i, :len(c["kps"])] = torch.from_numpy(c["blocked"])
    kps, desc, ur, bl = kps.to(dev), desc.to(dev), ur.to(dev), bl.to(dev)
    has_ur, has_bl = cases[0]["uright"] is not None, cases[0]["blocked"] is not None
    grid = cases[0]["grid"]
    ncell = grid.cols * grid.rows
    cs = torch.full((B, ncell + 1), -7, dtype=torch.int32, device=dev)
    ci = torch.full((B, cap), -7, dtype=torch.int32, device=dev)
    nqmax = max(len(c["queries"]) for c in cases)
    qs = torch.zeros((B, nqmax, 40), dtype=torch.uint8)
    qd = torch.zeros((B, nqmax, 32), dtype=torch.uint8)
    for i, c in enumerate(cases):
        nq = len(c["queries"])
        qs[i, :nq] = torch.from_numpy(c["queries"].view(np.uint8).reshape(nq, 40))
        qd[i, :nq] = torch.from_numpy(c["qdesc"])
    qs, qd = qs.to(dev), qd.to(dev)
    q_idx = torch.empty((B, nqmax), dtype=torch.int32, device=dev)
    q_dist = torch.empty((B, nqmax), dtype=torch.int32, device=dev)
    owner = torch.full((B, cap), -1, dtype=torch.int32, device=dev)     # the non-assigning modes leave it untouched
    nm = torch.empty((B,), dtype=torch.int32, device=dev)
    probs = (pkg.ProjProblem * B)()
    for i, c in enumerate(cases):
        probs[i] = pkg.ProjProblem(qs[i].data_ptr(), qd[i].data_ptr(), len(c["queries"]), kps[i].data_ptr(),
                                   desc[i].data_ptr(), ur[i].data_ptr() if has_ur else None,
                                   bl[i].data_ptr() if has_bl else None, cap,
                                   cs[i].data_ptr(), ci[i].data_ptr(), q_idx[i].data_ptr(), q_dist[i].data_ptr(),
                                   owner[i].data_ptr(), nm[i:i + 1].data_ptr())
    dprobs = torch.frombuffer(bytearray(bytes(probs)), dtype=torch.uint8).to(dev)
    counts = torch.tensor(ncount, dtype=torch.int32, device=dev)
    m.proj_search_batch_device(cases[0]["params"], grid, dprobs, cap, nqmax, grid_counts=counts)
    torch.cuda.synchronize()
    for i, c in enumerate(cases):
        n = ncount[i]
        rcs, rci = O.grid_assign(c["kps"][:n], grid)
        assert np.array_equal(cs[i].cpu().numpy(), rcs), i
        assert np.array_equal(ci[i, :rcs[-1]].cpu().numpy(), rci), i
        if i < 3:
            nq = len(c["queries"])
            got = (int(nm[i]), q_idx[i, :nq].cpu().numpy(), q_dist[i, :nq].cpu().numpy(), owner[i, :n].cpu().numpy())
            _check(c, got)
        else:                                            # no keypoint in the grid: nothing accepted
            assert int(nm[i]) == 0 and bool((q_idx[i, :len(c["queries"])] == -1).all())
    # a problem with grid count -1 reads the grid the launch above wrote; the others build theirs again (same arrays)
    counts_mixed = counts.clone()
    counts_mixed[0] = -1
    nm.fill_(-9)
    owner.fill_(-1)
    m.proj_search_batch_device(cases[0]["params"], grid, dprobs, cap, nqmax, grid_counts=counts_mixed)
    torch.cuda.synchronize()
    for i, c in enumerate(cases[:3]):
        rcs, rci = O.grid_assign(c["kps"][:ncount[i]], grid)
        assert np.array_equal(cs[i].cpu().numpy(), rcs), i
        nq = len(c["queries"])
        _check(c, (int(nm[i]), q_idx[i, :nq].cpu().numpy(), q_dist[i, :nq].cpu().numpy(), owner[i, :ncount[i]].cpu().numpy()))
    # every problem above the launch's bound (max_n < n): not searched, and its grid is written empty
    cs.fill_(-7)
    m.proj_search_batch_device(cases[0]["params"], grid, dprobs, cap - 1, nqmax, grid_counts=counts)
    torch.cuda.synchronize()
    assert bool((cs == 0).all()) and bool((nm == -1).all())
    for i, c in enumerate(cases):
        assert bool((q_idx[i, :len(c["queries"])] == -1).all()), i
