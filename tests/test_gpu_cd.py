"""MapFusion::CovisibilityDiscovery's detection and matching (src/MapFusion.cc:774-885) on the device
(multiagent.CovisibilityDiscovery) against the oracle running the reference's loop: per absorbed-map keyframe, minScore
from its covisible keyframes (:801-816), DetectCovisibilityCandidates ignoring the absorbed map (:819-820), SearchByBoW
with every candidate and the 15-match gate (:840-856)."""
import numpy as np
import pytest
import torch

from multiagent_orb_slam2_amd import multiagent as MA
from multiagent_orb_slam2_amd import synthetic as S

pytestmark = pytest.mark.gpu


def _maps(n, seed, nfeat=1000, rows=240, cols=480):
    """Matched map = left views of n scenes (slots 0..n-1), absorbed map = right views (slots n..2n-1)."""
    import multiagent_orb_slam2_amd as pkg
    left = [S.kitti_like_image(seed + i, rows=rows, cols=cols) for i in range(n)]
    right = [S.shifted_right_view(l, seed + i, max_disp=16) for i, l in enumerate(left)]
    ex = pkg.ORBextractor(nfeat, 1.2, 8, 20, 7)
    return ex.extract_batch_device(torch.from_numpy(np.stack(left + right)).cuda())


@pytest.mark.parametrize("strategy", [1, 2, 3])
def test_covisibility_discovery_vs_oracle(gpu, strategy):
    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    n = 12
    kps, desc, cnt = _maps(n, 40)
    cap = kps.shape[1]
    dev = kps.device
    voc = S.synthetic_vocabulary(13, k=10, L=4)
    v = pkg.ORBVocabulary.from_arrays(voc)
    fv = v.transform_batch_device(desc, cnt, 2)
    valid = (torch.arange(cap, device=dev)[None, :] < cnt[:, None]).to(torch.uint8)
    valid[:, 3::4] = 0
    store = pkg.KfStore.from_fields(cap, desc=(desc, cap * 32), kps=(kps, cap * 28), valid=(valid, cap),
                                    fv_nodes=(fv["fv_nodes"], cap * 4), fv_offsets=(fv["fv_offsets"], (cap + 1) * 4),
                                    fv_indices=(fv["fv_indices"], cap * 4), n_fv=(fv["n_fv"], 4))
    db = pkg.KeyFrameDatabase(v.info()["n_words"], 2 * n, max_words=cap)
    db.set_strategy(strategy)
    db.set_bow_device(torch.arange(2 * n, dtype=torch.int32, device=dev), fv["bow_words"], fv["bow_values"], fv["n_words"])
    db.add(list(range(n)))
    queries = list(range(n, 2 * n))
    covis = [[c for c in (q - 2, q - 1, q + 1, q + 2) if n <= c < 2 * n] for q in queries]
    cd = MA.CovisibilityDiscovery(pkg.ORBmatcher(0.75, True), db, store, max_fv_nodes=cap)
    pr, m12, nm, passed, n_cand = cd.run(queries, [5000 + i for i in range(n)], covis, queries)
    torch.cuda.synchronize()

    # the oracle: the reference's loop, one keyframe at a time
    kh, dh, ch = kps.cpu().numpy(), desc.cpu().numpy(), cnt.cpu().numpy()
    vh = valid.cpu().numpy()
    fvh = {k: t.cpu().numpy() for k, t in fv.items()}
    odb = O.Kfdb(v.info()["n_words"], 2 * n)
    for s in range(2 * n):
        nw = int(fvh["n_words"][s])
        odb.set_bow(s, fvh["bow_words"][s, :nw].astype(np.uint32), fvh["bow_values"][s, :nw])
    odb.add(list(range(n)))

    def view(s):
        c = int(ch[s])
        k = kh[s, :c].copy().view(pkg.KP_DTYPE).reshape(-1)
        nf = int(fvh["n_fv"][s])
        offs = fvh["fv_offsets"][s, :nf + 1]
        f = (fvh["fv_nodes"][s, :nf].astype(np.uint32), offs, fvh["fv_indices"][s, :offs[-1]])
        return dh[s, :c], k["angle"], vh[s, :c], f

    k_launch = max(1, int(n_cand.max()))
    exp_pairs, n_gate, n_real = [], 0, 0
    prh, nmh, m12h = pr.cpu().numpy(), nm.cpu().numpy(), m12.cpu().numpy()
    for i, q in enumerate(queries):
        ms = np.float32(1.0)
        for c in covis[i]:
            sc = np.float32(odb.score(q, c))
            if sc < ms:
                ms = sc
        cands = odb.detect(1, q, 5000 + i, float(ms), queries).tolist()
        assert n_cand[i] == len(cands), (i, n_cand[i], cands)
        exp_pairs += [[q, c] for c in cands] + [[q, -1]] * (k_launch - len(cands))
        for j, c in enumerate(cands):
            p = i * k_launch + j
            rn, rm = O.search_by_bow_kfkf(*view(q), *view(c), 0.75, True)
            assert nmh[p] == rn and np.array_equal(m12h[p, :int(ch[q])], rm), (q, c)
            n_real += 1
            n_gate += int(rn >= 15)
    assert prh.tolist() == exp_pairs
    assert np.array_equal(passed.cpu().numpy(), nmh >= 15)
    assert n_real >= n and n_gate >= 1
