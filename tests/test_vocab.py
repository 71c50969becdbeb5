"""DBoW2 vocabulary transform (BowVector + FeatureVector): oracle checks on CPU, GPU parity (bit-exact
doubles, identical CSR) with -m gpu.  The ORB vocabulary (ORBvoc.txt) is absent, so the
vocabularies are synthetic, in DBoW2's text format."""
import numpy as np
import pytest

from multiagent_orb_slam2_amd import synthetic as S
from oracle import oracle as O


def _py_transform(voc, feats, levelsup):
    """Pure-Python restatement of TemplatedVocabulary::transform (small cases only)."""
    n_lines = len(voc["parent"])
    children = [[] for _ in range(n_lines + 1)]
    word, wid = {}, 0
    for i, p in enumerate(voc["parent"]):
        children[p].append(i + 1)
        if voc["is_leaf"][i]:
            word[i + 1] = wid
            wid += 1
    desc = {i + 1: voc["desc"][i] for i in range(n_lines)}
    wt = {i + 1: voc["weight"][i] for i in range(n_lines)}
    bow, fv = {}, {}
    for f, x in enumerate(feats):
        cur, level, nid = 0, 0, 0
        while children[cur]:
            level += 1
            best, bd = None, None
            for c in children[cur]:
                d = int(np.unpackbits(x ^ desc[c]).sum())
                if bd is None or d < bd:
                    best, bd = c, d
            cur = best
            if level == voc["L"] - levelsup:
                nid = cur
        w = wt[cur]
        if w > 0:
            if voc["weighting"] in (0, 1):
                bow[word[cur]] = bow[word[cur]] + w if word[cur] in bow else w
            else:
                bow.setdefault(word[cur], w)
            fv.setdefault(nid, []).append(f)
    keys = sorted(bow)
    if voc["scoring"] == 0:
        norm = 0.0
        for k in keys:
            norm += abs(bow[k])
    else:
        norm = 0.0
        for k in keys:
            norm += bow[k] * bow[k]
        norm = norm ** 0.5
    vals = [bow[k] / norm for k in keys] if norm > 0 else [bow[k] for k in keys]
    return keys, vals, fv


@pytest.mark.parametrize("weighting,scoring,levelsup", [(0, 0, 1), (1, 0, 2), (2, 0, 0), (3, 1, 3), (0, 1, 2)])
def test_oracle_vocab_matches_python(weighting, scoring, levelsup):
    voc = S.synthetic_vocabulary(3, k=4, L=3, weighting=weighting, scoring=scoring, stop_frac=0.1)
    feats = S.random_descriptors(4, 150)
    r = O.vocab_transform(voc, feats, levelsup)
    keys, vals, fv = _py_transform(voc, feats, levelsup)
    assert r["bow_words"].tolist() == keys
    assert r["bow_values"].tolist() == vals
    assert r["fv_nodes"].tolist() == sorted(fv)
    assert [r["fv_indices"][a:b].tolist() for a, b in zip(r["fv_offsets"][:-1], r["fv_offsets"][1:])] == \
        [fv[k] for k in sorted(fv)]


def test_vocabulary_text_format_roundtrip(tmp_path):
    voc = S.synthetic_vocabulary(5, k=3, L=2)
    path = tmp_path / "voc.txt"
    S.write_vocabulary_text(voc, str(path))
    lines = path.read_text().split("\n")
    assert lines[0] == "3 2 0 0" and len(lines) == 1 + len(voc["parent"])
    parts = lines[1].split()
    assert len(parts) == 2 + 32 + 1
    assert float(parts[-1]) == voc["weight"][0]


@pytest.mark.gpu
@pytest.mark.parametrize("weighting,scoring,levelsup", [(0, 0, 2), (0, 0, 4), (1, 1, 1), (2, 0, 0), (3, 0, 2)])
def test_gpu_vocab_transform_bit_exact(gpu, weighting, scoring, levelsup):
    import multiagent_orb_slam2_amd as pkg
    voc = S.synthetic_vocabulary(7, k=10, L=4, weighting=weighting, scoring=scoring)
    v = pkg.ORBVocabulary.from_arrays(voc)
    assert v.info()["n_words"] == int(voc["is_leaf"].sum())
    feats = O.extract(S.kitti_like_image(17))["desc"]
    g = v.transform(feats, levelsup)
    r = O.vocab_transform(voc, feats, levelsup)
    assert np.array_equal(g.bow_words, r["bow_words"])
    assert g.bow_values.tobytes() == r["bow_values"].tobytes()      # bit-exact doubles
    assert np.array_equal(g.featvec[0], r["fv_nodes"]) and np.array_equal(g.featvec[1], r["fv_offsets"])
    assert np.array_equal(g.featvec[2], r["fv_indices"])


@pytest.mark.gpu
def test_gpu_vocab_load_text_and_batch(gpu, tmp_path):
    import torch

    import multiagent_orb_slam2_amd as pkg
    voc = S.synthetic_vocabulary(9, k=10, L=4)
    path = tmp_path / "voc.txt"
    S.write_vocabulary_text(voc, str(path))
    v = pkg.ORBVocabulary.load_text(str(path))
    imgs = np.stack([S.kitti_like_image(40 + i) for i in range(3)])
    ex = pkg.ORBextractor(2000, 1.2, 8, 20, 7)
    kps, desc, cnt = ex.extract_batch_device(torch.from_numpy(imgs).cuda())
    out = v.transform_batch_device(desc, cnt, levelsup=2)
    torch.cuda.synchronize()
    desc_h, cnt_h = desc.cpu().numpy(), cnt.cpu().numpy()
    o = {k: t.cpu().numpy() for k, t in out.items()}
    for i in range(3):
        feats = desc_h[i, :cnt_h[i]]
        r = O.vocab_transform(voc, feats, 2)
        nw, nf = o["n_words"][i], o["n_fv"][i]
        assert np.array_equal(o["bow_words"][i, :nw].astype(np.uint32), r["bow_words"])
        assert o["bow_values"][i, :nw].tobytes() == r["bow_values"].tobytes()
        assert np.array_equal(o["fv_nodes"][i, :nf].astype(np.uint32), r["fv_nodes"])
        assert np.array_equal(o["fv_offsets"][i, :nf + 1], r["fv_offsets"])
        assert np.array_equal(o["fv_indices"][i, :r["fv_offsets"][-1]], r["fv_indices"])


@pytest.mark.gpu
@pytest.mark.parametrize("check_ori", [True, False])
def test_gpu_bow_pairs_over_keyframe_store(gpu, check_ori):
    """Extractor -> vocabulary -> batched SearchByBoW(KF, KF) over a device keyframe store, every pair
    checked against the oracle's single-pair SearchByBoW on the host copies (MapFusion.cc:275 call shape)."""
    import torch

    import multiagent_orb_slam2_amd as pkg
    voc = S.synthetic_vocabulary(21, k=10, L=4)
    v = pkg.ORBVocabulary.from_arrays(voc)
    base = [S.kitti_like_image(60 + i) for i in range(3)]
    imgs = np.stack(base + [S.shifted_right_view(b, 9) for b in base])      # overlapping views -> real matches
    ex = pkg.ORBextractor(1500, 1.2, 8, 20, 7)
    kps, desc, cnt = ex.extract_batch_device(torch.from_numpy(imgs).cuda())
    out = v.transform_batch_device(desc, cnt, levelsup=4)
    B, cap = desc.shape[0], desc.shape[1]
    rng = np.random.default_rng(5)
    valid_h = (rng.random((B, cap)) < 0.85).astype(np.uint8)
    valid_h[np.arange(cap)[None, :] >= cnt.cpu().numpy()[:, None]] = 0
    valid = torch.from_numpy(valid_h).cuda()
    pairs_h = np.array([(i, j) for i in range(B) for j in range(B) if i != j] + [(2, 2)], np.int32)
    pairs = torch.from_numpy(pairs_h).cuda()
    m = pkg.ORBmatcher(0.75, check_ori)
    n_fv = out["n_fv"]
    store = pkg.orbx.KfStore.from_fields(
        cap, desc=(desc, cap * 32), kps=(kps, cap * 28), valid=(valid, cap), fv_nodes=(out["fv_nodes"], cap * 4),
        fv_offsets=(out["fv_offsets"], (cap + 1) * 4), fv_indices=(out["fv_indices"], cap * 4), n_fv=(n_fv, 4))
    m12, nm = m.SearchByBoW_pairs_device(store, pairs, int(n_fv.max().item()))
    torch.cuda.synchronize()
    kh, dh, ch = kps.cpu().numpy(), desc.cpu().numpy(), cnt.cpu().numpy()
    o = {k: out[k].cpu().numpy() for k in ("fv_nodes", "fv_offsets", "fv_indices", "n_fv")}
    m12h, nmh = m12.cpu().numpy(), nm.cpu().numpy()

    def kf(k):
        n, nf = ch[k], o["n_fv"][k]
        fv = (o["fv_nodes"][k, :nf].astype(np.uint32), o["fv_offsets"][k, :nf + 1], o["fv_indices"][k, :o["fv_offsets"][k, nf]])
        ang = np.ascontiguousarray(kh[k, :n]).view(pkg.KP_DTYPE).reshape(-1)["angle"]
        return dh[k, :n], ang, valid_h[k, :n], fv

    total = 0
    for p, (a, b) in enumerate(pairs_h):
        d1, a1, v1, f1 = kf(a)
        d2, a2, v2, f2 = kf(b)
        rn, rm = O.search_by_bow_kfkf(d1, a1, v1, f1, d2, a2, v2, f2, 0.75, check_ori)
        assert nmh[p] == rn, (p, a, b)
        assert np.array_equal(m12h[p, :ch[a]], rm), (p, a, b)
        assert (m12h[p, ch[a]:] == -1).all()
        total += rn
    assert total > 200
