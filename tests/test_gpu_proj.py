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
