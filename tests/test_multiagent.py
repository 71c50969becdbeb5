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


def _fv_dict(views_fv, cap):
    n = len(views_fv)
    d = dict(fv_nodes=np.zeros((n, cap), np.int32), fv_offsets=np.zeros((n, cap + 1), np.int32),
             fv_indices=np.zeros((n, cap), np.int32), n_fv=np.zeros(n, np.int32))
    for i, (ids, offs, idx) in enumerate(views_fv):
        d["fv_nodes"][i, :len(ids)] = ids
        d["fv_offsets"][i, :len(offs)] = offs
        d["fv_indices"][i, :len(idx)] = idx
        d["n_fv"][i] = len(ids)
    return {k: torch.from_numpy(v) for k, v in d.items()}


def test_packet_layout_aligned_and_featvec_roundtrip():
    cap = 320
    lay = MA.PacketLayout(cap)
    assert lay.bytes % 16 == 0 and all(o % 16 == 0 for o in lay.offsets.values())
    kps, desc, valid, counts = _keyframes(0, 2, cap)
    fvs = [S.random_featvec(40 + i, int(counts[i]), n_nodes=30) for i in range(2)]
    pk = MA.pack_keyframes(torch.from_numpy(kps.view(np.uint8).reshape(2, cap, 28)), torch.from_numpy(desc),
                           torch.from_numpy(counts), torch.from_numpy(valid), agent=1, frames=[0, 5], capacity=cap,
                           fv=_fv_dict(fvs, cap))
    for i, v in enumerate(MA.unpack_keyframes(pk, cap)):
        assert v.count == counts[i] and np.array_equal(v.desc, desc[i, :counts[i]])
        for a, b in zip(v.featvec, fvs[i]):
            assert np.array_equal(a, b)


def test_store_ring_and_candidate_pairs():
    cap = 64
    st = MA.DeviceKeyframeStore(cap, slots=12, device="cpu")
    P = MA.packet_bytes(cap)
    for step in range(5):                                # ring wraps: 5 steps x 4 slots > 12
        pk = torch.full((4, P), step, dtype=torch.uint8)
        slots = st.insert(pk, agent=step % 2)
        assert len(slots) == 4 and (st.buf[slots.start:slots.stop] == step).all()
    assert list(slots) == [4, 5, 6, 7]                  # step 4 landed after step 3 (slots 0-3)
    # other-agent candidates: most recent first, never the querying agent
    pr = st.candidate_pairs([4, 5], agent=0, k=3)
    # step 3 (agent 1) wrapped into slots 0-3, so those are agent 1's most recent keyframes
    assert pr.tolist() == [[4, 3], [4, 2], [4, 1], [5, 3], [5, 2], [5, 1]]
    own = st.candidate_pairs([6], agent=0, k=2, other_agents_only=False)
    assert own.tolist() == [[6, 5], [6, 4]]


def _store_worker(rank, world, port, cap, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ex = MA.KeyframeExchange()
    st = MA.DeviceKeyframeStore(cap, slots=8, device="cpu")
    for step in range(3):
        kps, desc, valid, counts = _keyframes(rank, 2, cap)
        fvs = [S.random_featvec(100 * rank + 10 * step + i, int(counts[i]), n_nodes=20) for i in range(2)]
        pk = MA.pack_keyframes(torch.from_numpy(kps.view(np.uint8).reshape(2, cap, 28)), torch.from_numpy(desc),
                               torch.from_numpy(counts), torch.from_numpy(valid), agent=rank,
                               frames=[10 * step, 10 * step + 5], capacity=cap, fv=_fv_dict(fvs, cap))
        slots = st.exchange_into(ex, pk)
    pairs = st.candidate_pairs(slots[2 * rank:2 * rank + 2], rank, k=3)
    if rank == 0:
        q.put((st.buf.numpy().copy(), list(st.agent_of), list(st.stamp), list(slots), pairs.tolist()))
    dist.destroy_process_group()


def test_two_agent_store_exchange_gloo():
    cap, world = 320, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_store_worker, args=(r, world, port, cap, q)) for r in range(world)]
    for p in procs:
        p.start()
    buf, agent_of, stamp, slots, pairs = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert slots == [0, 1, 2, 3]                         # third step wrapped (3 x 4 > 8 slots)
    assert agent_of[:4] == [0, 0, 1, 1] and stamp[:4] == [8, 9, 10, 11]
    views = MA.unpack_keyframes(torch.from_numpy(buf[:4]), cap)
    assert [v.agent for v in views] == [0, 0, 1, 1] and [v.frame for v in views] == [20, 25, 20, 25]
    for v in views:
        fv_exp = S.random_featvec(100 * v.agent + 20 + (v.frame - 20) // 5, v.count, n_nodes=20)
        assert all(np.array_equal(a, b) for a, b in zip(v.featvec, fv_exp))
    # rank 0's queries (slots 0, 1) get agent 1's most recent keyframes: slots 3, 2 (this step), then 7 (step 1)
    assert pairs == [[0, 3], [0, 2], [0, 7], [1, 3], [1, 2], [1, 7]]


@pytest.mark.gpu
def test_gpu_keyframe_fusion_store_vs_oracle(gpu):
    """Extractor -> stereo valid flags -> vocabulary -> packets -> device store -> KeyFrameDatabase
    DetectLoopCandidates -> batched SearchByBoW: the candidates of every query checked against the oracle's
    database fed the same BowVectors in the same order, every (query, candidate) pair against the oracle's
    SearchByBoW on the unpacked host keyframes."""
    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    dev = torch.device("cuda", 0)
    voc = S.synthetic_vocabulary(31, k=10, L=4)
    v = pkg.ORBVocabulary.from_arrays(voc)
    ex = pkg.ORBextractor(1200, 1.2, 8, 20, 7)
    m = pkg.ORBmatcher(0.75, True)
    base = S.kitti_like_image(77)
    imgs = np.stack([base] + [S.shifted_right_view(base, 3 + i, max_disp=12) for i in range(8)])
    kps, desc, cnt = ex.extract_batch_device(torch.from_numpy(imgs).to(dev))
    cap = kps.shape[1]
    valid = (torch.arange(cap, device=dev)[None, :] < cnt[:, None]).to(torch.uint8)
    valid[:, ::4] = 0                                   # a quarter without MapPoints
    K = 2
    fus = MA.KeyframeFusion(m, v, cap, slots=6, device=dev, candidates=K, levelsup=2)
    odb = O.Kfdb(v.info()["n_words"], 6)
    total = n_real = 0
    qid = 1
    for step in range(3):                               # 3 keyframes per step into a 6-slot ring: wraps once
        r = slice(3 * step, 3 * step + 3)
        pr, m12, nm, passed = fus.step(kps[r], desc[r], cnt[r], valid[r], frames=[3 * step + i for i in range(3)])
        torch.cuda.synchronize()
        views = MA.unpack_keyframes(fus.store.buf, cap)
        new = list(range((3 * step) % 6, (3 * step) % 6 + 3))
        odb.erase(new)
        for k in new:
            odb.set_bow(k, *views[k].bow)
        expect = []
        for k in new:                                   # MapFusion: query, then add (src/MapFusion.cc:133, :149)
            c = odb.detect(0, k, qid, 0.0)[:K].tolist()
            qid += 1
            expect += [[k, x] for x in c] + [[k, -1]] * (K - len(c))
            odb.add([k])
        prh, m12h, nmh = pr.cpu().numpy(), m12.cpu().numpy(), nm.cpu().numpy()
        assert prh.tolist() == expect, step
        for p, (a, b) in enumerate(prh):
            if b < 0:
                assert nmh[p] == 0 and (m12h[p] == -1).all()
                continue
            A, B = views[a], views[b]
            rn, rm = O.search_by_bow_kfkf(A.desc, A.kps["angle"], A.valid, A.featvec, B.desc, B.kps["angle"], B.valid,
                                          B.featvec, 0.75, True)
            assert nmh[p] == rn and np.array_equal(m12h[p, :A.count], rm), (p, a, b)
            total += rn
            n_real += 1
        assert np.array_equal(passed.cpu().numpy(), nmh >= 20)
    assert fus.status.item() == 0
    assert n_real >= 6 and total > 100


class _FakeExchange:
    """One GPU standing in for two agents: exchange() writes every agent's packets of this step rank-major, as
    the RCCL all-gather would (the packets of all agents are prepared beforehand)."""

    def __init__(self, rank, world):
        self.rank, self.world = rank, world
        self.packets = None

    def exchange(self, packets, out=None):
        g = torch.cat([packets if r == self.rank else self.packets[r] for r in range(self.world)], 0)
        if out is None:
            return g
        out.copy_(g)
        return out


@pytest.mark.gpu
def test_gpu_keyframe_fusion_two_agents_one_gpu(gpu):
    """KeyframeFusion.step's multi-rank branch on the GPU, two agents emulated on one device: the exchanged ring,
    slot groups, orbx_kfdb_detect_sequential_device and orbx_kfdb_candidate_pairs_device with slot/query groups
    (the same-map discard of src/MapFusion.cc:136-144) and the batched SearchByBoW, against the oracle running
    MapFusion's loop over the same keyframes (every exchanged keyframe queried then added, in order)."""
    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    dev = torch.device("cuda", 0)
    voc = S.synthetic_vocabulary(31, k=10, L=4)
    v = pkg.ORBVocabulary.from_arrays(voc)
    ex = pkg.ORBextractor(1200, 1.2, 8, 20, 7)
    base = S.kitti_like_image(91)
    # agents 0 and 1 revisit the same place: 2 keyframes per agent per step, 3 steps
    imgs = np.stack([S.shifted_right_view(base, 5 + i, max_disp=10) for i in range(12)])
    kps, desc, cnt = ex.extract_batch_device(torch.from_numpy(imgs).to(dev))
    cap = kps.shape[1]
    valid = (torch.arange(cap, device=dev)[None, :] < cnt[:, None]).to(torch.uint8)
    valid[:, 1::3] = 0
    n, K, W, SLOTS = 2, 3, 2, 8
    fx = [_FakeExchange(r, W) for r in range(W)]
    fus = [MA.KeyframeFusion(pkg.ORBmatcher(0.75, True), v, cap, slots=SLOTS, device=dev, agent=r, exchange=fx[r],
                             candidates=K, levelsup=2) for r in range(W)]
    odb = O.Kfdb(v.info()["n_words"], SLOTS)
    kf_id, n_real, n_cross_same_step = 1, 0, 0
    for step in range(3):
        rows = [list(range(4 * step + 2 * r, 4 * step + 2 * r + 2)) for r in range(W)]
        pk = []
        for r in range(W):
            ix = torch.tensor(rows[r], device=dev)
            fv = v.transform_batch_device(desc[ix].contiguous(), cnt[ix].contiguous(), 2)
            pk.append(MA.pack_keyframes(kps[ix], desc[ix], cnt[ix], valid[ix], r, [10 * step + i for i in range(n)], cap,
                                        fv))
        for f in fx:
            f.packets = pk
        outs = []
        for r in range(W):
            ix = torch.tensor(rows[r], device=dev)
            outs.append(fus[r].step(kps[ix], desc[ix], cnt[ix], valid[ix], frames=[10 * step + i for i in range(n)]))
        torch.cuda.synchronize()
        views = MA.unpack_keyframes(fus[0].store.buf, cap)
        for a, b in zip(views, MA.unpack_keyframes(fus[1].store.buf, cap)):   # both rings hold the same keyframes
            assert (a.count, a.agent, a.frame) == (b.count, b.agent, b.frame)
            assert np.array_equal(a.desc, b.desc) and np.array_equal(a.kps, b.kps) and np.array_equal(a.valid, b.valid)
            assert (a.bow is None) == (b.bow is None) and (a.bow is None or all(np.array_equal(x, y) for x, y in zip(a.bow, b.bow)))
        new = list(range((4 * step) % SLOTS, (4 * step) % SLOTS + 4))
        agent = {k: views[k].agent for k in range(SLOTS) if views[k].count > 0}
        assert [agent[k] for k in new] == [0, 0, 1, 1]
        for r in range(W):
            assert fus[r].slot_group[new].tolist() == [0, 0, 1, 1]
        odb.erase(new)
        for k in new:
            odb.set_bow(k, *views[k].bow)
        expect = {0: [], 1: []}
        for k in new:
            a = agent[k]
            c = [x for x in odb.detect(0, k, kf_id, 0.0).tolist() if agent[x] != a][:K]
            kf_id += 1
            n_cross_same_step += sum(1 for x in c if x in new)
            expect[a] += [[k, x] for x in c] + [[k, -1]] * (K - len(c))
            odb.add([k])
        for r in range(W):
            pr, m12, nm, passed = outs[r]
            prh, m12h, nmh = pr.cpu().numpy(), m12.cpu().numpy(), nm.cpu().numpy()
            assert prh.tolist() == expect[r], (step, r)
            for p, (a, b) in enumerate(prh):
                if b < 0:
                    assert nmh[p] == 0 and (m12h[p] == -1).all()
                    continue
                A, B = views[a], views[b]
                rn, rm = O.search_by_bow_kfkf(A.desc, A.kps["angle"], A.valid, A.featvec, B.desc, B.kps["angle"],
                                              B.valid, B.featvec, 0.75, True)
                assert nmh[p] == rn and np.array_equal(m12h[p, :A.count], rm), (step, r, p)
                n_real += 1
            assert np.array_equal(passed.cpu().numpy(), nmh >= 20)
            fus[r].check()
    assert n_real >= 10 and n_cross_same_step >= 1


# ---- KeyframeFusion.step on CPU over gloo: ring, exchange, slot groups, query-then-add order ---------------
_FUS_CAP, _FUS_SLOTS, _FUS_K, _FUS_STEPS, _FUS_N = 320, 8, 3, 3, 2


def _fusion_inputs(rank, step):
    kps, desc, valid, counts = _keyframes(rank, 4, _FUS_CAP)
    # rotate the views per step so each step's keyframes differ
    sel = [(step + i) % 4 for i in range(_FUS_N)]
    return kps[sel], desc[sel], valid[sel], counts[sel]


def _fusion_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from fusion_doubles import OracleKfdb, OracleMatcher, OracleVocab
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    voc = S.synthetic_vocabulary(31, k=10, L=4)
    vocab = OracleVocab(voc)
    m = OracleMatcher(0.75, True)
    fus = MA.KeyframeFusion(m, vocab, _FUS_CAP, slots=_FUS_SLOTS, device=torch.device("cpu"), agent=rank,
                            exchange=MA.KeyframeExchange(), candidates=_FUS_K, levelsup=2,
                            db=OracleKfdb(vocab.n_words, _FUS_SLOTS))
    m.fusion = fus
    outs = []
    for step in range(_FUS_STEPS):
        kps, desc, valid, counts = _fusion_inputs(rank, step)
        pr, m12, nm, passed = fus.step(torch.from_numpy(kps.view(np.uint8).reshape(_FUS_N, _FUS_CAP, 28)),
                                       torch.from_numpy(desc), torch.from_numpy(counts), torch.from_numpy(valid),
                                       frames=[10 * step + i for i in range(_FUS_N)])
        outs.append((pr.tolist(), nm.tolist(), m12.tolist(), passed.tolist(), fus.slot_group.tolist()))
    fus.check()
    objs = [None] * world
    dist.all_gather_object(objs, outs)
    if rank == 0:
        q.put(objs)
    dist.destroy_process_group()


def _fusion_expected(world):
    """MapFusion's server loop (src/MapFusion.cc:51-81) over the same keyframes in processing order: every
    exchanged keyframe in turn is queried (DetectLoopCandidates, :133), its first K other-map candidates
    (:136-144) are matched (SearchByBoW, :275), then it joins the database (:149 / :222)."""
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from oracle import oracle as O
    voc = S.synthetic_vocabulary(31, k=10, L=4)
    vocab = O.Vocabulary(voc)
    db = O.Kfdb(int(np.sum(voc["is_leaf"])), _FUS_SLOTS)
    ring = {}
    expect = {r: [] for r in range(world)}
    pos, kf_id = 0, 1
    for step in range(_FUS_STEPS):
        n_new = world * _FUS_N
        if pos + n_new > _FUS_SLOTS:
            pos = 0
        slots = list(range(pos, pos + n_new))
        pos += n_new
        db.erase(slots)
        for r in range(world):
            kps, desc, valid, counts = _fusion_inputs(r, step)
            for i in range(_FUS_N):
                s = slots[r * _FUS_N + i]
                c = counts[i]
                bow = vocab.transform(desc[i, :c], 2)
                ring[s] = dict(agent=r, desc=desc[i, :c], angle=kps[i, :c]["angle"], valid=valid[i, :c],
                               fv=(bow["fv_nodes"], bow["fv_offsets"], bow["fv_indices"]))
                db.set_bow(s, bow["bow_words"], bow["bow_values"])
        step_out = {r: ([], [], []) for r in range(world)}
        for s in slots:
            r = ring[s]["agent"]
            cands = [c for c in db.detect(0, s, kf_id, 0.0).tolist() if ring[c]["agent"] != r][:_FUS_K]
            kf_id += 1
            for c in cands + [-1] * (_FUS_K - len(cands)):
                step_out[r][0].append([s, c])
                if c < 0:
                    step_out[r][1].append(0)
                    step_out[r][2].append(None)
                    continue
                A, B = ring[s], ring[c]
                nm, m12 = O.search_by_bow_kfkf(A["desc"], A["angle"], A["valid"], A["fv"], B["desc"], B["angle"],
                                               B["valid"], B["fv"], 0.75, True)
                step_out[r][1].append(int(nm))
                step_out[r][2].append(np.asarray(m12).tolist())
            db.add([s])
        for r in range(world):
            expect[r].append(step_out[r])
    return expect


def test_keyframe_fusion_step_two_agents_gloo():
    """KeyframeFusion.step's multi-rank branch on CPU (gloo, world 2) with oracle-backed vocabulary, database and
    matcher: the exchanged ring, the slot groups, the sequential query-then-add order and the same-map discard
    must give exactly MapFusion's single-server results, split by the agent that owns each query."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fusion_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    objs = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    expect = _fusion_expected(world)
    n_real = 0
    for r in range(world):
        for step in range(_FUS_STEPS):
            pr, nm, m12, passed, groups = objs[r][step]
            epr, enm, em12 = expect[r][step]
            assert pr == epr, (r, step)
            assert nm == enm, (r, step)
            for p, e in enumerate(em12):
                if e is None:
                    assert all(v == -1 for v in m12[p])
                else:
                    assert m12[p][:len(e)] == e
                    n_real += 1
            assert passed == [v >= 20 for v in nm]
            # ring slots of this step carry their agent
            assert sorted(set(g for g in groups if g >= 0)) == [0, 1]
    assert n_real >= 6
    # sequential adds: in the first step (empty ring before it) agent 1's keyframes (slots 2, 3) already see agent
    # 0's keyframes of the same exchange (slots 0, 1), which MapFusion added before them
    assert any(c in (0, 1) for _, c in objs[1][0][0])
    assert max(v for r in range(world) for st in objs[r] for v in st[1]) >= 20


# ---- configs C4 / C5 at their agent counts, emulated on one GPU ------------------------------------------------
# C4: 4 agents on EuRoC MH01-MH04 (752x480, 1200 kpts, Examples/Stereo/EuRoC.yaml:88) -- one sequence per agent;
# C5: 8 agents on KITTI seq 00 (1242x375, 2000 kpts) split 8-way (generic_split_seq.cc:543-589, 4541 frames).
AGENT_CONFIGS = {
    "C4": dict(W=4, rows=480, cols=752, nfeat=1200, chunks=[range(0, 3682), range(0, 3040), range(0, 2700), range(0, 2033)]),
    "C5": dict(W=8, rows=375, cols=1242, nfeat=2000, chunks=MA.split_sequence(4541, 8)),
}


def agent_images(cfg, steps, n, places=3, seed=700):
    """Keyframe j of agent r at step s shows place (r + s + j) % places, shifted: every agent revisits the places
    the others see, so MapFusion finds cross-agent candidates.  Returns (images [steps][W][n], frame ids)."""
    bases = [S.kitti_like_image(seed + p, rows=cfg["rows"], cols=cfg["cols"]) for p in range(places)]
    imgs, frames = [], []
    for s in range(steps):
        imgs.append([[S.shifted_right_view(bases[(r + s + j) % places], 3 + 5 * r + j, max_disp=10) for j in range(n)]
                     for r in range(cfg["W"])])
        frames.append([[cfg["chunks"][r].start + 5 * (s * n + j) for j in range(n)] for r in range(cfg["W"])])
    return imgs, frames


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["C4", "C5"])
def test_gpu_keyframe_fusion_agents_one_gpu(gpu, config):
    """KeyframeFusion.step's multi-rank branch at C4's / C5's agent count on one GPU: every agent's packets
    exchanged rank-major (the RCCL all-gather's order), W replicas of the ring, slot groups, the sequential
    DetectLoopCandidates, the same-map discard (src/MapFusion.cc:136-144) and SearchByBoW, against the oracle running
    MapFusion's single-server loop over the same keyframes."""
    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    cfg = AGENT_CONFIGS[config]
    W, n, K, STEPS = cfg["W"], 2, 3, 3
    SLOTS = 2 * W * n
    dev = torch.device("cuda", 0)
    voc = S.synthetic_vocabulary(31, k=10, L=5)
    v = pkg.ORBVocabulary.from_arrays(voc)
    ex = pkg.ORBextractor(cfg["nfeat"], 1.2, 8, 20, 7)
    imgs, frames = agent_images(cfg, STEPS, n)
    flat = np.stack([im for st in imgs for ag in st for im in ag])
    kps, desc, cnt = ex.extract_batch_device(torch.from_numpy(flat).to(dev))
    cap = kps.shape[1]
    valid = (torch.arange(cap, device=dev)[None, :] < cnt[:, None]).to(torch.uint8)
    valid[:, 2::5] = 0
    fx = [_FakeExchange(r, W) for r in range(W)]
    fus = [MA.KeyframeFusion(pkg.ORBmatcher(0.75, True), v, cap, slots=SLOTS, device=dev, agent=r, exchange=fx[r],
                             candidates=K, levelsup=3) for r in range(W)]
    odb = O.Kfdb(v.info()["n_words"], SLOTS)
    kf_id, n_real, n_cross, n_gate = 1, 0, 0, 0
    for step in range(STEPS):
        rows = [[(step * W + r) * n + j for j in range(n)] for r in range(W)]
        pk = []
        for r in range(W):
            ix = torch.tensor(rows[r], device=dev)
            fv = v.transform_batch_device(desc[ix].contiguous(), cnt[ix].contiguous(), 3)
            pk.append(MA.pack_keyframes(kps[ix], desc[ix], cnt[ix], valid[ix], r, frames[step][r], cap, fv))
        for f in fx:
            f.packets = pk
        outs = []
        for r in range(W):
            ix = torch.tensor(rows[r], device=dev)
            outs.append(fus[r].step(kps[ix], desc[ix], cnt[ix], valid[ix], frames=frames[step][r]))
        torch.cuda.synchronize()
        views = MA.unpack_keyframes(fus[0].store.buf, cap)
        for r in range(1, W):   # every rank's ring holds the same keyframes
            for a, b in zip(views, MA.unpack_keyframes(fus[r].store.buf, cap)):
                assert (a.count, a.agent, a.frame) == (b.count, b.agent, b.frame)
                assert np.array_equal(a.desc, b.desc) and np.array_equal(a.valid, b.valid)
        base = (step * W * n) % SLOTS
        new = list(range(base, base + W * n))
        agent = {k: views[k].agent for k in range(SLOTS) if views[k].count > 0}
        assert [agent[k] for k in new] == [r for r in range(W) for _ in range(n)]
        assert [views[k].frame for k in new] == [f for r in range(W) for f in frames[step][r]]
        for r in range(W):
            assert fus[r].slot_group[new].tolist() == [r for r in range(W) for _ in range(n)]
        odb.erase(new)
        for k in new:
            odb.set_bow(k, *views[k].bow)
        expect = {r: [] for r in range(W)}
        for k in new:   # MapFusion's loop: query, drop same-map candidates, first K, then add
            a = agent[k]
            c = [x for x in odb.detect(0, k, kf_id, 0.0).tolist() if agent[x] != a][:K]
            kf_id += 1
            n_cross += sum(1 for x in c if x in new)
            expect[a] += [[k, x] for x in c] + [[k, -1]] * (K - len(c))
            odb.add([k])
        for r in range(W):
            pr, m12, nm, passed = outs[r]
            prh, m12h, nmh = pr.cpu().numpy(), m12.cpu().numpy(), nm.cpu().numpy()
            assert prh.tolist() == expect[r], (step, r)
            for p, (a, b) in enumerate(prh):
                if b < 0:
                    assert nmh[p] == 0 and (m12h[p] == -1).all()
                    continue
                assert agent[b] != r                                   # same-map discard
                A, B = views[a], views[b]
                rn, rm = O.search_by_bow_kfkf(A.desc, A.kps["angle"], A.valid, A.featvec, B.desc, B.kps["angle"],
                                              B.valid, B.featvec, 0.75, True)
                assert nmh[p] == rn and np.array_equal(m12h[p, :A.count], rm), (step, r, p)
                n_real += 1
                n_gate += int(rn >= 20)
            assert np.array_equal(passed.cpu().numpy(), nmh >= 20)
            fus[r].check()
    assert n_real >= W * n and n_cross >= 1 and n_gate >= 1


def test_keyframe_fusion_agent_must_be_rank():
    """the same-map discard compares slot groups (rank-major) with the query group (the agent)."""
    class X:
        world, rank = 4, 2
    with pytest.raises(ValueError):
        MA.KeyframeFusion(None, None, 64, slots=8, device=torch.device("cpu"), agent=1, exchange=X())
