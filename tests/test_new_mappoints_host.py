"""Host-side pieces of the batched CreateNewMapPoints stage (multiagent.NewMapPoints): the F12 / epipole geometry of
LocalMapping::ComputeF12 (src/LocalMapping.cc:542-557) and ORBmatcher.cc:666-672 against a float64 numpy restatement,
and the device observation-list builder against plain loops (torch on the CPU)."""
import numpy as np
import torch

from multiagent_orb_slam2_amd import multiagent as MA


def _rot(w):
    th = np.linalg.norm(w)
    if th == 0:
        return np.eye(3)
    k = w / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx


def test_triangulation_geometry_matches_numpy():
    rng = np.random.default_rng(4)
    K = np.array([[718.856, 0, 607.1928], [0, 718.856, 185.2157], [0, 0, 1]])
    N = 7
    R = np.stack([_rot(rng.normal(0, 0.1, 3)) for _ in range(N)])
    t = rng.normal(0, 1, (N, 3))
    pairs = np.array([[0, 1], [3, 2], [6, 0], [-1, 2], [5, 5]])
    g = MA.triangulation_geometry(torch.tensor(K), torch.tensor(R), torch.tensor(t), torch.tensor(pairs)).numpy()
    assert g.shape == (5, 12) and g.dtype == np.float32
    for p, (a, b) in enumerate(pairs):
        if a < 0:
            assert not g[p].any()
            continue
        R12 = R[a] @ R[b].T
        t12 = -R12 @ t[b] + t[a]
        tx = np.array([[0, -t12[2], t12[1]], [t12[2], 0, -t12[0]], [-t12[1], t12[0], 0]])
        F = np.linalg.inv(K).T @ tx @ R12 @ np.linalg.inv(K)
        if a == b:
            assert np.abs(g[p, :9]).max() < 1e-9                            # no baseline: F = 0, epipole undefined
            continue
        np.testing.assert_allclose(g[p, :9], F.reshape(-1), rtol=1e-4, atol=1e-7 * np.abs(F).max())
        C2 = R[b] @ (-R[a].T @ t[a]) + t[b]
        np.testing.assert_allclose(g[p, 9:11], [K[0, 0] * C2[0] / C2[2] + K[0, 2], K[1, 1] * C2[1] / C2[2] + K[1, 2]],
                                   rtol=1e-3)


def test_neighbour_observations_match_loops():
    rng = np.random.default_rng(2)
    n, nn, cap = 3, 4, 9
    new = torch.tensor([10, 11, 12], dtype=torch.int32)
    nb = torch.tensor([[1, 2, 3, -1], [10, 1, -1, -1], [0, 1, 2, 3]], dtype=torch.int32)
    m12 = torch.tensor(np.where(rng.random((n, nn, cap)) < 0.4, rng.integers(0, cap, (n, nn, cap)), -1), dtype=torch.int32)
    m12[nb.long() < 0] = -1
    obs, off = MA.neighbour_observations(new, nb, m12)
    exp, eoff = [], [0]
    for j in range(n):
        for i in range(cap):
            # the first neighbour with a match makes the MapPoint: [(neighbour, match), (new keyframe, i)]
            for k in range(nn):
                if nb[j, k] >= 0 and m12[j, k, i] >= 0:
                    exp += [[int(nb[j, k]), int(m12[j, k, i])], [int(new[j]), i]]
                    break
            eoff.append(len(exp))
    assert off.tolist() == eoff
    assert obs[:eoff[-1]].tolist() == exp
