"""CPU checks of the oracle's keypoint grid and projection / radius matchers (oracle/proj_oracle.cpp,
test infrastructure) against an independent pure-Python restatement of the reference's loops
(tests/proj_cases.py).  Parity status: the reference has no tests or fixtures for these matchers
(SURVEY §4, §8c); both restatements follow src/ORBmatcher.cc / src/Frame.cc line by line."""
import numpy as np
import pytest

from oracle import oracle as O
from proj_cases import MODES, make_case, py_features_in_area, py_grid, py_proj_search


def test_grid_assign_matches_python():
    c = make_case(1, MODES["mappoints"], n_target=500)
    cs, ci = O.grid_assign(c["kps"], c["grid"])
    cells = py_grid(c["kps"], c["grid"])
    assert cs[-1] == sum(len(x) for x in cells) < len(c["kps"])      # some keypoints fall outside the grid
    for cell, lst in enumerate(cells):
        assert ci[cs[cell]:cs[cell + 1]].tolist() == lst


def test_features_in_area_matches_python():
    c = make_case(2, MODES["mappoints"], n_target=600)
    k, g = c["kps"], c["grid"]
    cs, ci = O.grid_assign(k, g)
    cells = py_grid(k, g)
    rng = np.random.default_rng(0)
    for _ in range(300):
        x, y = rng.uniform(-30, 670), rng.uniform(-30, 510)
        r = float(rng.choice([2.5, 4.0, 7.0, 15.0, 40.0]))
        lo, hi = int(rng.integers(-1, 4)), int(rng.integers(-1, 8))
        got = O.features_in_area(k, cs, ci, g, x, y, r, lo, hi).tolist()
        assert got == py_features_in_area(k, cells, g, x, y, r, lo, hi)


@pytest.mark.parametrize("mode", sorted(MODES))
@pytest.mark.parametrize("dense", [False, True])
def test_proj_search_oracle_matches_python(mode, dense):
    for seed in (3, 4):
        c = make_case(seed, MODES[mode], n_target=240, n_query=200, dense=dense)
        got = O.proj_search(c["params"], c["grid"], c["queries"], c["qdesc"], c["kps"], c["desc"], c["uright"],
                            c["blocked"])
        ref = py_proj_search(c)
        assert got[0] == ref[0], (mode, seed)
        for g, r, name in zip(got[1:], ref[1:], ("q_idx", "q_dist", "owner")):
            assert np.array_equal(g, r), (mode, seed, name)


def test_proj_search_exercises_conflicts():
    """The dense cases really contain the sequential couplings the GPU has to reproduce."""
    c = make_case(5, MODES["keyframe"], n_target=240, n_query=200, dense=True)
    nm, qi, qd, own = O.proj_search(c["params"], c["grid"], c["queries"], c["qdesc"], c["kps"], c["desc"], None,
                                    c["blocked"])
    acc = qi[qi >= 0]
    assert len(acc) > 20 and len(np.unique(acc)) == len(acc)          # blocking: no keypoint assigned twice
    assert (own == -2).any()                                          # rotation filter removed some
    c = make_case(6, MODES["init"], n_target=240, n_query=200, dense=True)
    nm, qi, _, _ = O.proj_search(c["params"], c["grid"], c["queries"], c["qdesc"], c["kps"], c["desc"])
    assert nm == (qi >= 0).sum() and nm > 5


@pytest.mark.parametrize("seed", range(6))
def test_projection_oracle_matches_python(seed):
    """The projection step (orc_project: LASTFRAME :1363-1392, isInFrustum + the MAPPOINTS window, Fuse :854-893)
    equals the independent pure-Python restatement bit for bit, and every rejection branch occurs."""
    from multiagent_orb_slam2_amd.orbx import PROJ_FUSE, PROJ_LASTFRAME, PROJ_MAPPOINTS, PROJ_QUERY_DTYPE, QF_SKIP
    from proj_cases import make_projection_case, project_py
    p, v, sc, lsf = make_projection_case(seed)
    for mode in (PROJ_LASTFRAME, PROJ_MAPPOINTS, PROJ_FUSE):
        a = O.project(mode, p, v, sc, lsf)
        b = project_py(mode, p, v, sc, lsf).view(np.uint8).reshape(-1, 40)
        assert np.array_equal(a, b), f"mode {mode}: {int((a != b).any(1).sum())} queries differ"
        q = a.view(PROJ_QUERY_DTYPE).reshape(-1)
        kept = (q["flags"] & QF_SKIP) == 0
        assert 0.3 * len(p) < kept.sum() < 0.95 * len(p)          # both outcomes well represented
        if mode != PROJ_LASTFRAME:
            assert len(set(q["level"][kept].tolist())) >= 4        # PredictScale spreads the levels


@pytest.mark.parametrize("seed", range(3))
def test_stereo_mappoints_oracle_matches_python(seed):
    """MapPoints of a stereo frame (UnprojectStereo + the Frame form of the MapPoint constructor): the oracle equals the
    numpy-float32 restatement bit for bit; keypoints without depth (-1, 0) are skipped."""
    from multiagent_orb_slam2_amd.orbx import QF_BLOCKS, QF_SKIP
    from proj_cases import SCALE, stereo_frame_case, stereo_mappoints_py
    k, depth, twc, cam = stereo_frame_case(seed)
    a = O.stereo_mappoints(k, depth, twc, cam, SCALE, QF_BLOCKS)
    b = stereo_mappoints_py(k, depth, twc, cam, SCALE, QF_BLOCKS)
    assert np.array_equal(a.view(np.uint8), b.view(np.uint8))
    assert np.array_equal((a["flags"] & QF_SKIP) != 0, ~(depth > 0))
