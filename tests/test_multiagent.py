"""Multi-agent layer on CPU: sequence split, keyframe packets, and the N>1 exchange + sharded
cross-agent matching with world_size 2 over gloo (the GPU path uses the same code over RCCL)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from multiagent_orb_slam2_amd import multiagent as MA
from multiagent_orb_slam2_amd import synthetic as S
from multiagent_orb_slam2_amd.orbx import KP_DTYPE


def _reference_split(n, k):
    # generic_split_seq.cc:543-589 restated
    length, remain = n // k, n % k
    begin = end = 0
    out = []
    for _ in range(k):
        if remain > 0:
            end += length + 1
            remain -= 1
        else:
            end += length
        out.append((begin, end))
        begin = end
    return out


@pytest.mark.parametrize("n,k", [(10, 3), (4541, 8), (7, 7), (3, 4), (0, 2), (1101, 2)])
def test_split_sequence(n, k):
    got = [(r.start, r.stop) for r in MA.split_sequence(n, k)]
    assert got == _reference_split(n, k)
    assert sum(r.stop - r.start for r in MA.split_sequence(n, k)) == n


class OracleMatcher:
    """Test double: the oracle's SearchByBoW behind the ORBmatcher method name (CPU-only test)."""

    def SearchByBoW_KF_KF(self, d1, a1, v1, fv1, d2, a2, v2, fv2):
        from oracle import oracle as O
        return O.search_by_bow_kfkf(d1, a1, v1, fv1, d2, a2, v2, fv2, 0.75, True)


def _keyframes(agent, n_kf, cap):
    from oracle import oracle as O
    kps = np.zeros((n_kf, cap), KP_DTYPE)
    desc = np.zeros((n_kf, cap, 32), np.uint8)
    valid = np.zeros((n_kf, cap), np.uint8)
    counts = np.zeros(n_kf, np.int32)
    base = S.kitti_like_image(500, rows=160, cols=320)
    for i in range(n_kf):
        # agents revisit the same place: agent 1's keyframe i is a shifted view of agent 0's
        img = S.shifted_right_view(base, 10 * agent + i, max_disp=6) if agent else base
        r = O.extract(img, nfeatures=300)
        n = min(len(r["kps"]), cap)
        kps[i, :n], desc[i, :n], counts[i] = r["kps"][:n], r["desc"][:n], n
        valid[i, :n] = (np.arange(n) % 3 != 0)
    return kps, desc, valid, counts


def featvec_of(kv):
    # deterministic synthetic FeatureVector from the keypoint cell (vocabulary absent)
    cell = (kv.kps["x"] // 40).astype(np.int64) * 16 + (kv.kps["y"] // 40).astype(np.int64)
    ids = np.unique(cell).astype(np.uint32)
    order = np.argsort(cell, kind="stable").astype(np.int32)
    offs = np.concatenate([[0], np.cumsum([np.sum(cell == i) for i in ids])]).astype(np.int32)
    return ids, offs, order


def test_pack_unpack_roundtrip():
    cap = 320
    kps, desc, valid, counts = _keyframes(0, 2, cap)
    pk = MA.pack_keyframes(torch.from_numpy(kps.view(np.uint8).reshape(2, cap, 28)), torch.from_numpy(desc),
                           torch.from_numpy(counts), torch.from_numpy(valid), agent=3, frames=[10, 15], capacity=cap)
    assert pk.shape == (2, MA.packet_bytes(cap))
    views = MA.unpack_keyframes(pk, cap)
    for i, v in enumerate(views):
        assert v.agent == 3 and v.frame == [10, 15][i] and v.count == counts[i]
        assert np.array_equal(v.kps, kps[i, :counts[i]]) and np.array_equal(v.desc, desc[i, :counts[i]])
        assert np.array_equal(v.valid, valid[i, :counts[i]])


def _worker(rank, world, port, cap, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    kps, desc, valid, counts = _keyframes(rank, 2, cap)
    pk = MA.pack_keyframes(torch.from_numpy(kps.view(np.uint8).reshape(2, cap, 28)), torch.from_numpy(desc),
                           torch.from_numpy(counts), torch.from_numpy(valid), agent=rank, frames=[5 * rank, 5 * rank + 5],
                           capacity=cap)
    ex = MA.KeyframeExchange()
    gathered = ex.exchange(pk)
    store = MA.MapFusionStore()
    store.insert(MA.unpack_keyframes(gathered, cap))
    # sharded by query keyframe: this rank's own keyframes against every other agent's
    mine = [k for k in store.keyframes if k.agent == rank]
    results = []
    for qi, qkf in enumerate(mine):
        for ci, n, m12, ok in MA.cross_agent_match(OracleMatcher(), qkf, featvec_of(qkf), store.candidates_for(rank),
                                                   featvec_of):
            results.append((rank, qi, ci, int(n), m12.tolist()))
    objs = [None] * world
    dist.all_gather_object(objs, results)
    if rank == 0:
        q.put((gathered.numpy().copy(), objs))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_agent_exchange_and_sharded_matching_gloo():
    cap, world = 320, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cap, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered, objs = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    # the gathered store holds both agents' keyframes, rank-major
    views = MA.unpack_keyframes(torch.from_numpy(gathered), cap)
    assert [v.agent for v in views] == [0, 0, 1, 1]
    for a in range(world):
        kps, desc, valid, counts = _keyframes(a, 2, cap)
        for i in range(2):
            v = views[2 * a + i]
            assert np.array_equal(v.desc, desc[i, :counts[i]]) and np.array_equal(v.kps, kps[i, :counts[i]])
    # sharded results == a single-process computation of every (query, other-agent candidate) pair
    flat = sorted([tuple(r[:4]) for rr in objs for r in rr])
    exp = []
    m = OracleMatcher()
    for a in range(world):
        mine = [v for v in views if v.agent == a]
        cands = [v for v in views if v.agent != a]
        for qi, qkf in enumerate(mine):
            for ci, c in enumerate(cands):
                n, _ = m.SearchByBoW_KF_KF(qkf.desc, qkf.kps["angle"], qkf.valid, featvec_of(qkf), c.desc,
                                           c.kps["angle"], c.valid, featvec_of(c))
                exp.append((a, qi, ci, int(n)))
    assert flat == sorted(exp)
    assert max(r[3] for r in flat) >= 20   # the revisited place passes MapFusion's 20-match gate
