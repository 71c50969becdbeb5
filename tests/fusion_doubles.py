"""Oracle-backed test doubles for KeyframeFusion's library objects (vocabulary, keyframe database, matcher), so that
KeyframeFusion.step itself -- ring, exchange, slot groups, query-then-add order, candidate pairs -- runs on CPU
tensors (gloo tests) with the oracle's restatements doing the per-keyframe work.  Test infrastructure only.

The database double runs MapFusion's loop literally (src/MapFusion.cc:133 detect, :149/:222 add): adds are queued
in processing order and a sequential detect walks the queue, answering each query keyframe before adding it."""
import numpy as np
import torch

from multiagent_orb_slam2_amd import multiagent as MA
from oracle import oracle as O


class OracleVocab:
    def __init__(self, voc):
        self.voc = voc
        self.v = O.Vocabulary(voc)
        self.n_words = int(np.sum(voc["is_leaf"]))

    def info(self):
        return dict(k=self.voc["k"], L=self.voc["L"], n_nodes=len(self.voc["parent"]) + 1, n_words=self.n_words)

    def transform_batch_device(self, desc, counts, levelsup=4, stream=None):
        B, cap = desc.shape[0], desc.shape[1]
        z = lambda *shape, dt=np.int32: np.zeros(shape, dt)
        out = dict(fv_nodes=z(B, cap), fv_offsets=z(B, cap + 1), fv_indices=z(B, cap), n_fv=z(B),
                   bow_words=z(B, cap), bow_values=z(B, cap, dt=np.float64), n_words=z(B))
        d, c = desc.numpy(), counts.numpy()
        for i in range(B):
            r = self.v.transform(d[i, :c[i]], levelsup)
            nf, nw = len(r["fv_nodes"]), len(r["bow_words"])
            out["fv_nodes"][i, :nf] = r["fv_nodes"]
            out["fv_offsets"][i, :nf + 1] = r["fv_offsets"]
            out["fv_indices"][i, :len(r["fv_indices"])] = r["fv_indices"]
            out["n_fv"][i] = nf
            out["bow_words"][i, :nw] = r["bow_words"]
            out["bow_values"][i, :nw] = r["bow_values"]
            out["n_words"][i] = nw
        return {k: torch.from_numpy(v) for k, v in out.items()}


class OracleKfdb:
    def __init__(self, n_words, slots):
        self.db = O.Kfdb(n_words, slots)
        self.S = slots
        self.pending = []

    def _flush(self):
        self.db.add(self.pending)
        self.pending = []

    def erase(self, slots):
        self._flush()
        self.db.erase(list(slots))

    def add(self, slots):
        self.pending += list(slots)

    def set_bow_device(self, slots, words, values, n_words, strides=None, stream=None):
        # rows of a packet ring: byte views starting at each field (strides in elements are the packet size)
        w8, v8, n8 = words.contiguous().numpy(), values.contiguous().numpy(), n_words.contiguous().numpy()
        for i, k in enumerate(slots.tolist()):
            nw = int(n8[i, :4].view(np.int32)[0])
            self.db.set_bow(k, w8[i, :4 * nw].copy().view(np.uint32), v8[i, :8 * nw].copy().view(np.float64))

    def detect_device(self, kind, query_slots, query_ids, min_scores=None, status=None, stream=None, sequential=False):
        qs, ids = query_slots.tolist(), query_ids.tolist()
        ms = [0.0] * len(qs) if min_scores is None else min_scores.tolist()
        res = {}
        if sequential:
            for k in self.pending:
                if k in qs:
                    i = qs.index(k)
                    res[i] = self.db.detect(kind, k, ids[i], ms[i])
                self.db.add([k])
            self.pending = []
        self._flush()
        for i in range(len(qs)):
            if i not in res:
                res[i] = self.db.detect(kind, qs[i], ids[i], ms[i])
        out = torch.full((len(qs), self.S), -1, dtype=torch.int32)
        n = torch.zeros(len(qs), dtype=torch.int32)
        for i, c in res.items():
            out[i, :len(c)] = torch.from_numpy(c.astype(np.int32))
            n[i] = len(c)
        return out, n, status

    @staticmethod
    def candidate_pairs_device(cand, n_cand, query_slots, k, slot_group=None, query_group=None, out=None, stream=None):
        pairs = []
        for q, qs in enumerate(query_slots.tolist()):
            c = cand[q, :int(n_cand[q])].tolist()
            if slot_group is not None and query_group is not None:
                c = [x for x in c if int(slot_group[x]) != int(query_group[q])]
            c = c[:k]
            pairs += [[qs, x] for x in c] + [[qs, -1]] * (k - len(c))
        return torch.tensor(pairs, dtype=torch.int32).reshape(-1, 2)


class OracleMatcher:
    """SearchByBoW(KF, KF) over the fusion's packet ring (the KfStore argument only names it)."""

    def __init__(self, nnratio=0.75, check_ori=True):
        self.nnratio, self.check_ori = nnratio, check_ori
        self.fusion = None

    def SearchByBoW_pairs_device(self, store, pairs, max_fv_nodes, stream=None):
        st = self.fusion.store
        views = MA.unpack_keyframes(st.buf, st.capacity)
        P = pairs.shape[0]
        m12 = torch.full((P, st.capacity), -1, dtype=torch.int32)
        nm = torch.zeros(P, dtype=torch.int32)
        for p, (a, b) in enumerate(pairs.tolist()):
            if a < 0 or b < 0:
                continue
            A, B = views[a], views[b]
            n, m = O.search_by_bow_kfkf(A.desc, A.kps["angle"], A.valid, A.featvec, B.desc, B.kps["angle"], B.valid,
                                        B.featvec, self.nnratio, self.check_ori)
            nm[p] = int(n)
            m12[p, :A.count] = torch.from_numpy(np.asarray(m, np.int32))
        return m12, nm
