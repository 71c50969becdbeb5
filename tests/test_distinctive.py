"""MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:246-311): the oracle against an independent numpy
restatement, and the HIP kernel (host, device and keyframe-store forms) against the oracle, index-exact."""
import numpy as np
import pytest
import torch

from multiagent_orb_slam2_amd import synthetic as S
from oracle import oracle as O


def numpy_distinctive(lists):
    out = []
    for d in lists:
        n = len(d)
        if n == 0:
            out.append(-1)
            continue
        bits = np.unpackbits(np.asarray(d, np.uint8), axis=1).astype(np.int32)
        D = (bits[:, None, :] != bits[None, :, :]).sum(-1)           # all-pairs Hamming, zero diagonal
        med = np.sort(D, axis=1)[:, int(0.5 * (n - 1))]
        out.append(int(np.argmin(med)))                               # first row with the smallest median
    return np.array(out, np.int32)


def mappoint_lists(seed, sizes):
    """Observed descriptors of MapPoints: a true descriptor seen in N keyframes with a few flipped bits each, plus
    exact duplicates and outliers so that medians tie."""
    rng = np.random.default_rng(seed)
    lists = []
    for n in sizes:
        base = rng.integers(0, 256, 32, dtype=np.uint8)
        d = np.repeat(base[None], n, 0)
        if n:
            flips = rng.random((n, 256)) < rng.uniform(0.0, 0.15)
            d = np.packbits(np.unpackbits(d, axis=1) ^ flips.astype(np.uint8), axis=1)
            if n > 3:
                d[rng.integers(0, n)] = d[rng.integers(0, n)]                       # duplicate
                d[rng.integers(0, n)] = rng.integers(0, 256, 32, dtype=np.uint8)    # outlier
        lists.append(d)
    return lists


SIZES = [0, 1, 2, 3, 4, 5, 8, 17, 31, 63, 64, 65, 100, 129, 300, 1, 2, 0, 7]


def test_oracle_matches_numpy():
    for seed in range(4):
        lists = mappoint_lists(seed, SIZES)
        assert np.array_equal(O.distinctive_descriptors(lists), numpy_distinctive(lists))


def test_oracle_ties_pick_first():
    d = S.random_descriptors(3, 1)
    assert O.distinctive_descriptors([np.repeat(d, 4, 0)]).tolist() == [0]    # all equal -> first
    a, b = S.random_descriptors(4, 2)
    assert O.distinctive_descriptors([np.stack([a, b])]).tolist() == [0]      # N=2: both medians 0 -> first


@pytest.mark.gpu
def test_gpu_distinctive_host_and_device(gpu):
    import multiagent_orb_slam2_amd as pkg
    m = pkg.ORBmatcher(0.75, True)
    for seed in range(6):
        lists = mappoint_lists(100 + seed, SIZES * 3)
        ref = O.distinctive_descriptors(lists)
        best, desc = m.ComputeDistinctiveDescriptors(lists)
        assert np.array_equal(best, ref), seed
        for p, d in enumerate(lists):
            if ref[p] >= 0:
                assert np.array_equal(desc[p], d[ref[p]])
        dev = torch.device("cuda", 0)
        off = np.zeros(len(lists) + 1, np.int32)
        off[1:] = np.cumsum([len(d) for d in lists])
        flat = torch.from_numpy(np.concatenate([d for d in lists if len(d)])).to(dev)
        b2, d2 = m.distinctive_descriptors_device(flat, torch.from_numpy(off).to(dev))
        assert np.array_equal(b2.cpu().numpy(), ref)


@pytest.mark.gpu
def test_gpu_distinctive_over_keyframe_store(gpu):
    """MapPoints observed in keyframes of a device store (MapFusion's packet ring layout): observation = (slot,
    keypoint index); the descriptor rows live in the packets."""
    import multiagent_orb_slam2_amd as pkg
    from multiagent_orb_slam2_amd import multiagent as MA
    dev = torch.device("cuda", 0)
    cap, slots = 64, 12
    st = MA.DeviceKeyframeStore(cap, slots, dev)
    rng = np.random.default_rng(9)
    desc = rng.integers(0, 256, (slots, cap, 32), dtype=np.uint8)
    # MapPoint p is keypoint p % cap seen in several keyframes with small perturbations
    M = 150
    obs, lists = [], []
    for p in range(M):
        n = int(rng.integers(0, slots + 1))
        ks = rng.choice(slots, n, replace=False)
        idx = p % cap
        base = desc[ks[0], idx] if n else None
        for k in ks:
            flips = rng.random(256) < 0.08
            desc[k, idx] = np.packbits(np.unpackbits(base) ^ flips.astype(np.uint8))
        obs.append(np.stack([ks, np.full(n, idx)], 1).astype(np.int32) if n else np.zeros((0, 2), np.int32))
    for p in range(M):
        lists.append(np.stack([desc[k, i] for k, i in obs[p]]) if len(obs[p]) else np.zeros((0, 32), np.uint8))
    lay = st.layout
    buf = st.buf.cpu().numpy()
    for k in range(slots):
        buf[k, lay.offsets["desc"]:lay.offsets["desc"] + cap * 32] = desc[k].reshape(-1)
    st.buf.copy_(torch.from_numpy(buf))
    off = np.zeros(M + 1, np.int32)
    off[1:] = np.cumsum([len(o) for o in obs])
    m = pkg.ORBmatcher(0.75, True)
    best, out = m.distinctive_descriptors_store_device(st.kf_store(), torch.from_numpy(np.concatenate(obs)).to(dev),
                                                       torch.from_numpy(off).to(dev))
    ref = O.distinctive_descriptors(lists)
    assert np.array_equal(best.cpu().numpy(), ref)
    outh = out.cpu().numpy()
    for p in range(M):
        if ref[p] >= 0:
            assert np.array_equal(outh[p], lists[p][ref[p]])
