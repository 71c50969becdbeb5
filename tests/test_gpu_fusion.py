"""The native keyframe path (orbx_fusion: BoW, packets, ring, sequential DetectLoopCandidates, other-map candidate
pairs, batched SearchByBoW) against the oracle running MapFusion's loop, for one agent and for two agents emulated
on one GPU (two-phase API with the all-gather done by the test), and the native RCCL exchange at world 1."""
import numpy as np
import pytest
import torch

from multiagent_orb_slam2_amd import multiagent as MA
from multiagent_orb_slam2_amd import synthetic as S

pytestmark = pytest.mark.gpu


def _inputs(seed, n_img, nfeat=1200):
    import multiagent_orb_slam2_amd as pkg
    dev = torch.device("cuda", 0)
    ex = pkg.ORBextractor(nfeat, 1.2, 8, 20, 7)
    base = S.kitti_like_image(seed)
    imgs = np.stack([S.shifted_right_view(base, 3 + i, max_disp=12) for i in range(n_img)])
    kps, desc, cnt = ex.extract_batch_device(torch.from_numpy(imgs).to(dev))
    cap = kps.shape[1]
    depth = torch.rand((n_img, cap), device=dev) - 0.3           # stands in for mvDepth: > 0 on ~70 %
    return kps, desc, cnt, depth, cap


def _check_step(views, agent_of, new, queries, K, kf_id, odb, pr, m12, nm):
    """MapFusion's loop over the new slots in order (query, then add); returns the next keyframe id."""
    from oracle import oracle as O
    odb.erase(new)
    for k in new:
        odb.set_bow(k, *views[k].bow)
    expect = {}
    for k in new:
        c = [x for x in odb.detect(0, k, kf_id, 0.0).tolist() if agent_of[x] != agent_of[k] or len(set(agent_of.values())) == 1]
        kf_id += 1
        expect[k] = c[:K] + [-1] * (K - len(c[:K]))
        odb.add([k])
    prh, m12h, nmh = pr.cpu().numpy(), m12.cpu().numpy(), nm.cpu().numpy()
    exp_pairs = [[q, c] for q in queries for c in expect[q]]
    assert prh.tolist() == exp_pairs
    n_real = 0
    for p, (a, b) in enumerate(prh):
        if b < 0:
            assert nmh[p] == 0 and (m12h[p] == -1).all()
            continue
        A, B = views[a], views[b]
        rn, rm = O.search_by_bow_kfkf(A.desc, A.kps["angle"], A.valid, A.featvec, B.desc, B.kps["angle"], B.valid,
                                      B.featvec, 0.75, True)
        assert nmh[p] == rn and np.array_equal(m12h[p, :A.count], rm), (p, a, b)
        n_real += 1
    return kf_id, n_real


def test_native_fusion_single_agent_vs_oracle(gpu):
    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    kps, desc, cnt, depth, cap = _inputs(77, 20)
    voc = S.synthetic_vocabulary(31, k=10, L=4)
    v = pkg.ORBVocabulary.from_arrays(voc)
    K, SLOTS, n = 3, 8, 3
    eng = pkg.KeyframeFusionEngine(v, pkg.ORBmatcher(0.75, True), cap, SLOTS, max_keyframes=n, candidates=K, levelsup=2)
    odb = O.Kfdb(v.info()["n_words"], SLOTS)
    kf_id, total_real = 1, 0
    for step in range(4):                                         # 3 keyframes a step, every 2nd row: the ring wraps
        rows = range(5 * step, 5 * step + 2 * n, 2)
        out = eng.new_outputs(n)
        eng.step(kps, desc, cnt, rows, frame_base=100 * step, frame_step=2, depth=depth, outputs=out)
        torch.cuda.synchronize()
        ring = eng.read_ring()
        views = MA.unpack_keyframes(ring, cap)
        new, queries = eng.last_step()
        for j, k in enumerate(new):                               # packets hold exactly the chosen rows
            r = rows[j]
            c = int(cnt[r])
            assert views[k].count == c and views[k].frame == 100 * step + 2 * j and views[k].agent == 0
            assert np.array_equal(views[k].desc, desc[r, :c].cpu().numpy())
            assert np.array_equal(views[k].valid, (depth[r, :c] > 0).to(torch.uint8).cpu().numpy())
        agent_of = {k: 0 for k in range(SLOTS)}
        kf_id, nr = _check_step(views, agent_of, list(new), list(queries), K, kf_id, odb, *out)
        total_real += nr
    eng.check()
    assert total_real >= 10


def test_native_fusion_two_agents_one_gpu(gpu):
    """Two engines (agents 0 and 1, world 2) on one GPU; the test all-gathers their packets (rank-major) and hands
    them to phase 2, as the bench does with torch.distributed at N > 1: engine 0 takes them from a separate buffer
    (commit copies them into its ring), engine 1 has them written straight into the ring slots its pack reserved
    (exchange_view, a zero-copy view) and commits in place -- the two rings must agree."""
    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    kps, desc, cnt, depth, cap = _inputs(91, 16)
    voc = S.synthetic_vocabulary(31, k=10, L=4)
    v = pkg.ORBVocabulary.from_arrays(voc)
    K, SLOTS, n, W = 3, 8, 2, 2
    eng = [pkg.KeyframeFusionEngine(v, pkg.ORBmatcher(0.75, True), cap, SLOTS, max_keyframes=n, candidates=K, levelsup=2,
                                    agent=r, world=W) for r in range(W)]
    odb = O.Kfdb(v.info()["n_words"], SLOTS)
    kf_id, total_real, cross = 1, 0, 0
    with pytest.raises(pkg.OrbxError):
        eng[1].exchange_view()                   # nothing reserved before the first pack()
    for step in range(3):
        sends = []
        for r in range(W):
            send = torch.empty((n, eng[r].packet_bytes), dtype=torch.uint8, device=kps.device)
            eng[r].pack(kps, desc, cnt, range(4 * step + 2 * r, 4 * step + 2 * r + n), frame_base=10 * step, depth=depth,
                        send=send)
            sends.append(send)
        gathered = torch.cat(sends, 0)
        outs = []
        for r in range(W):
            o = eng[r].new_outputs(n)
            if r == 0:
                eng[r].commit(gathered, o)
            else:
                view = eng[r].exchange_view()
                assert view.shape == gathered.shape and view.data_ptr() != gathered.data_ptr()
                view.copy_(gathered)
                eng[r].commit(None, o)
            outs.append(o)
        torch.cuda.synchronize()
        rings = [e.read_ring() for e in eng]
        new, _ = eng[0].last_step()
        assert np.array_equal(rings[0][new.start:new.stop], rings[1][new.start:new.stop])
        views = MA.unpack_keyframes(rings[0], cap)
        agent_of = {k: views[k].agent for k in range(SLOTS)}
        assert [agent_of[k] for k in new] == [0, 0, 1, 1]
        # one oracle loop over the step's slots; each engine answers its own agent's queries
        odb.erase(list(new))
        for k in new:
            odb.set_bow(k, *views[k].bow)
        expect = {}
        for k in new:
            c = [x for x in odb.detect(0, k, kf_id, 0.0).tolist() if agent_of[x] != agent_of[k]][:K]
            cross += sum(1 for x in c if x in new)
            kf_id += 1
            expect[k] = c + [-1] * (K - len(c))
            odb.add([k])
        for r in range(W):
            _, queries = eng[r].last_step()
            pr, m12, nm = outs[r]
            assert pr.cpu().numpy().tolist() == [[q, c] for q in queries for c in expect[q]], (step, r)
            for p, (a, b) in enumerate(pr.cpu().numpy()):
                if b < 0:
                    continue
                A, B = views[a], views[b]
                rn, rm = O.search_by_bow_kfkf(A.desc, A.kps["angle"], A.valid, A.featvec, B.desc, B.kps["angle"],
                                              B.valid, B.featvec, 0.75, True)
                assert int(nm[p]) == rn and np.array_equal(m12[p, :A.count].cpu().numpy(), rm)
                total_real += 1
    for e in eng:
        e.check()
    assert total_real >= 8 and cross >= 1


def test_native_rccl_exchange_world1(gpu):
    """orbx_exchange at world 1 (one GPU on this box): unique id, communicator, all-gather = copy."""
    import multiagent_orb_slam2_amd as pkg
    uid = pkg.KeyframeExchangeRCCL.unique_id()
    assert len(uid) == 128
    x = pkg.KeyframeExchangeRCCL(uid, 1, 0, 0)
    send = torch.randint(0, 256, (3, 4096), dtype=torch.uint8, device="cuda:0")
    recv = torch.zeros_like(send)
    x.allgather(send, recv)
    torch.cuda.synchronize()
    assert torch.equal(send, recv)
    x.close()


@pytest.mark.parametrize("config", ["C4", "C5"])
def test_native_fusion_agents_one_gpu(gpu, config):
    """The native engine (orbx_fusion) at C4's (4 agents, 752x480 / 1200) and C5's (8 agents, KITTI 1242x375 / 2000,
    seq 00 split 8-way) agent counts on one GPU: W engines, the test all-gathers their packets rank-major and hands them
    to phase 2 -- ring replicas, slot groups, the sequential DetectLoopCandidates, the same-map discard and the batched
    SearchByBoW against the oracle's MapFusion loop."""
    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    from test_multiagent import AGENT_CONFIGS, agent_images
    cfg = AGENT_CONFIGS[config]
    W, n, K, STEPS = cfg["W"], 2, 3, 3
    SLOTS = 2 * W * n
    dev = torch.device("cuda", 0)
    voc = S.synthetic_vocabulary(37, k=10, L=5)
    v = pkg.ORBVocabulary.from_arrays(voc)
    ex = pkg.ORBextractor(cfg["nfeat"], 1.2, 8, 20, 7)
    imgs, frames = agent_images(cfg, STEPS, n, seed=760)
    flat = np.stack([im for st in imgs for ag in st for im in ag])
    kps, desc, cnt = ex.extract_batch_device(torch.from_numpy(flat).to(dev))
    cap = kps.shape[1]
    depth = torch.rand((len(flat), cap), device=dev) - 0.3
    eng = [pkg.KeyframeFusionEngine(v, pkg.ORBmatcher(0.75, True), cap, SLOTS, max_keyframes=n, candidates=K, levelsup=3,
                                    agent=r, world=W) for r in range(W)]
    odb = O.Kfdb(v.info()["n_words"], SLOTS)
    kf_id, total_real, cross = 1, 0, 0
    for step in range(STEPS):
        sends = []
        for r in range(W):
            send = torch.empty((n, eng[r].packet_bytes), dtype=torch.uint8, device=dev)
            first = (step * W + r) * n
            eng[r].pack(kps, desc, cnt, range(first, first + n), frame_base=frames[step][r][0], frame_step=5, depth=depth,
                        send=send)
            sends.append(send)
        gathered = torch.cat(sends, 0)
        outs = []
        for r in range(W):
            o = eng[r].new_outputs(n)
            eng[r].commit(gathered, o)
            outs.append(o)
        torch.cuda.synchronize()
        rings = [e.read_ring() for e in eng]
        new, _ = eng[0].last_step()
        for r in range(1, W):
            assert np.array_equal(rings[0][new.start:new.stop], rings[r][new.start:new.stop])
        views = MA.unpack_keyframes(rings[0], cap)
        agent_of = {k: views[k].agent for k in range(SLOTS)}
        assert [agent_of[k] for k in new] == [r for r in range(W) for _ in range(n)]
        assert [views[k].frame for k in new] == [f for r in range(W) for f in frames[step][r]]
        odb.erase(list(new))
        for k in new:
            odb.set_bow(k, *views[k].bow)
        expect = {}
        for k in new:
            c = [x for x in odb.detect(0, k, kf_id, 0.0).tolist() if agent_of[x] != agent_of[k]][:K]
            cross += sum(1 for x in c if x in new)
            kf_id += 1
            expect[k] = c + [-1] * (K - len(c))
            odb.add([k])
        for r in range(W):
            _, queries = eng[r].last_step()
            assert list(queries) == list(range(new.start + r * n, new.start + (r + 1) * n))
            pr, m12, nm = outs[r]
            assert pr.cpu().numpy().tolist() == [[q, c] for q in queries for c in expect[q]], (step, r)
            for p, (a, b) in enumerate(pr.cpu().numpy()):
                if b < 0:
                    continue
                assert agent_of[b] != r
                A, B = views[a], views[b]
                rn, rm = O.search_by_bow_kfkf(A.desc, A.kps["angle"], A.valid, A.featvec, B.desc, B.kps["angle"],
                                              B.valid, B.featvec, 0.75, True)
                assert int(nm[p]) == rn and np.array_equal(m12[p, :A.count].cpu().numpy(), rm)
                total_real += 1
    for e in eng:
        e.check()
    assert total_real >= W * n and cross >= 1
