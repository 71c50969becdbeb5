"""Synthetic keyframe databases and query sequences for the KeyFrameDatabase tests, plus a pure-Python
restatement of the reference's queries (src/KeyFrameDatabase.cc:76-420, DBoW2 L1Scoring
ScoringObject.cpp:23-66) used to check the C++ oracle on small cases.

A case models places: keyframes of one place draw most of their words from the place's pool (so they
share many words and are covisible), the rest from a Zipf-like global distribution (common words shared
by everyone).  BowVectors are L1-normalised like DBoW2's TF-IDF + L1_NORM vectors."""
from __future__ import annotations

import numpy as np

LOOP, COVIS, RELOC = 0, 1, 2


def make_kfdb_case(seed: int, n_slots: int = 120, n_vocab: int = 4000, n_places: int = 8, words_lo: int = 30,
                   words_hi: int = 260, n_queries: int = 40, repeat_ids: bool = True, max_words: int = 4096):
    rng = np.random.default_rng(seed)
    zipf = 1.0 / np.arange(1, n_vocab + 1) ** 1.1
    cdf = np.cumsum(zipf / zipf.sum())
    pools = [rng.choice(n_vocab, size=min(n_vocab, 500), replace=False) for _ in range(n_places)]
    place = rng.integers(0, n_places, n_slots)
    bows = []
    for k in range(n_slots):
        m = int(rng.integers(words_lo, words_hi + 1))
        m = min(m, max_words)
        own = rng.choice(pools[place[k]], size=min(len(pools[place[k]]), int(m * 0.7)), replace=False)
        common = np.minimum(np.searchsorted(cdf, rng.random(m)), n_vocab - 1)
        words = np.unique(np.concatenate([own, common]))[:m]
        vals = rng.gamma(1.0, 1.0, len(words))
        vals = vals / vals.sum()
        if rng.random() < 0.1:                          # a few exactly-equal values (term = -2 min(v, w))
            vals[:] = 1.0 / len(words)
        bows.append((words.astype(np.uint32), vals.astype(np.float64)))
    covis = {}
    for k in range(n_slots):
        same = np.flatnonzero(place == place[k])
        same = same[same != k]
        other = rng.choice(n_slots, size=3, replace=False)
        cand = np.concatenate([rng.permutation(same), other])
        cand = [int(c) for c in dict.fromkeys(cand.tolist()) if c != k]
        covis[k] = cand[:int(rng.integers(0, 11))]
    # operations: adds (random order), some erases / re-adds, queries
    ops = []
    order = rng.permutation(n_slots)
    n_add = int(n_slots * 0.8)
    ops.append(("add", order[:n_add // 2].tolist()))
    ops.append(("erase", order[:max(1, n_add // 10)].tolist()))
    ops.append(("add", order[n_add // 2:n_add].tolist()))
    ops.append(("add", order[:max(1, n_add // 20)].tolist()))   # re-added: go to the end of every list
    next_id = 1000
    used = []
    batch = []
    for qi in range(n_queries):
        kind = int(rng.integers(0, 3))
        # mostly keyframes not in the database yet (LoopClosing / MapFusion add the query after detection)
        slot = int(rng.choice(order[n_add:])) if rng.random() < 0.8 else int(rng.integers(0, n_slots))
        if repeat_ids and used and rng.random() < 0.15:
            qid = int(rng.choice(used))                  # a repeated query id: stale scratch fields
        else:
            qid = next_id
            next_id += int(rng.integers(1, 4))
            used.append(qid)
        ms = float(rng.choice([0.0, 0.005, 0.01, 0.02, 0.05]))
        if kind == LOOP:
            excl = [c for c in covis[slot]] + rng.choice(n_slots, size=int(rng.integers(0, 4))).tolist()
        elif kind == COVIS:
            excl = rng.choice(n_slots, size=int(rng.integers(0, n_slots // 3))).tolist()
        else:
            excl = []
        batch.append((kind, slot, qid, ms, sorted(set(int(e) for e in excl))))
        if rng.random() < 0.25 or qi == n_queries - 1:
            ops.append(("query", batch))
            batch = []
    init_scores = [rng.uniform(0, 0.1, n_slots).astype(np.float32) for _ in range(3)]
    return dict(n_slots=n_slots, n_vocab=n_vocab, bows=bows, covis=covis, ops=ops, init_scores=init_scores)


# --------------------------------------------------------------------------------------------------
# pure-Python restatement (small cases only)
# --------------------------------------------------------------------------------------------------
f32 = np.float32


def l1_score(a, b) -> float:
    """DBoW2 L1Scoring::score(v1 = a, v2 = b): common words ascending, |v-w| - |v| - |w|, then -s/2."""
    (aw, av), (bw, bv) = a, b
    i = j = 0
    s = 0.0
    while i < len(aw) and j < len(bw):
        if aw[i] == bw[j]:
            vi, wi = float(av[i]), float(bv[j])
            s += abs(vi - wi) - abs(vi) - abs(wi)
            i += 1
            j += 1
        elif aw[i] < bw[j]:
            i += 1
        else:
            j += 1
    return -s / 2.0


class PyKfdb:
    def __init__(self, n_vocab, n_slots):
        self.inv = [[] for _ in range(n_vocab)]
        self.bow = [(np.zeros(0, np.uint32), np.zeros(0))] * n_slots
        self.covis = [[] for _ in range(n_slots)]
        self.q = np.zeros((3, n_slots), np.uint64)
        self.w = np.zeros((3, n_slots), np.int64)
        self.s = np.zeros((3, n_slots), np.float32)

    def add(self, k):
        for w in self.bow[k][0]:
            self.inv[int(w)].append(k)

    def erase(self, k):
        for w in self.bow[k][0]:
            lst = self.inv[int(w)]
            if k in lst:
                lst.remove(k)

    def detect(self, kind, qs, qid, min_score, excl):
        excl = set(excl)
        q, w, s = self.q[kind], self.w[kind], self.s[kind]
        sharing = []
        for word in self.bow[qs][0]:
            for k in self.inv[int(word)]:
                if kind == COVIS and k in excl:
                    continue
                if q[k] != qid:
                    w[k] = 0
                    if kind != LOOP or k not in excl:
                        q[k] = qid
                        sharing.append(k)
                w[k] += 1
        if not sharing:
            return []
        max_common = max(int(w[k]) for k in sharing)
        min_common = int(f32(max_common) * f32(0.8))
        scored = []
        for k in sharing:
            if w[k] > min_common:
                si = f32(l1_score(self.bow[qs], self.bow[k]))
                if kind != COVIS:
                    s[k] = si
                if kind == RELOC or si >= f32(min_score):
                    scored.append((si, k))
        if not scored:
            return []
        acc_list = []
        best_acc = f32(0.0) if kind == RELOC else f32(min_score)
        for si, k in scored:
            best, acc, bk = si, si, k
            for n in self.covis[k]:
                if q[n] != qid:
                    continue
                if kind != RELOC and not (w[n] > min_common):
                    continue
                acc = f32(acc + s[n])
                if s[n] > best:
                    bk, best = n, s[n]
            acc_list.append((acc, bk))
            if acc > best_acc:
                best_acc = acc
        retain = f32(0.75) * best_acc
        out, seen = [], set()
        for acc, bk in acc_list:
            if acc > retain and bk not in seen:
                out.append(bk)
                seen.add(bk)
        return out


def run_case(case, db, py_style: bool = False):
    """Apply a case's operations to a database object (the oracle Kfdb, PyKfdb or the GPU
    KeyFrameDatabase); returns the candidate lists of every query in order."""
    results = []
    for op, arg in case["ops"]:
        if op == "add":
            for k in arg:
                db.add(k) if py_style else db.add([k])
        elif op == "erase":
            for k in arg:
                db.erase(k) if py_style else db.erase([k])
        else:
            for kind, slot, qid, ms, excl in arg:
                results.append(list(db.detect(kind, slot, qid, ms, excl)))
    return results


def setup_db(case, db, py_style: bool = False):
    for k, (w, v) in enumerate(case["bows"]):
        if py_style:
            db.bow[k] = (w, v)
        else:
            db.set_bow(k, w, v)
    if py_style:
        for k, lst in case["covis"].items():
            db.covis[k] = list(lst)[:10]
        for kind in range(3):
            db.s[kind] = case["init_scores"][kind]
    else:
        db.set_covisibility(case["covis"])
        n = case["n_slots"]
        for kind in range(3):
            db.set_state(kind, np.zeros(n, np.uint64), np.zeros(n, np.int32), case["init_scores"][kind])


# --------------------------------------------------------------------------------------------------
# numpy model of the GPU's batched reformulation (orbx_kfdb.hip): every query of a batch computed from
# the scratch fields at batch start, list order from the (first shared word, add sequence) key, scores
# written by earlier queries of the batch looked up (score_before), plus the interaction flag that
# sends a batch back to one-query-at-a-time evaluation.  Must equal the sequential restatement on every
# batch it does not flag.
# --------------------------------------------------------------------------------------------------
def batch_model(db: PyKfdb, kind, queries, seqs, members):
    S = len(db.covis)
    q0, w0, s0 = db.q[kind].copy(), db.w[kind].copy(), db.s[kind].copy()
    sets = [set(db.bow[k][0].tolist()) if members[k] else set() for k in range(S)]
    outs, hist = [], []
    for qs, qid, ms, excl in queries:
        ex = np.zeros(S, bool)
        ex[list(excl)] = True
        qwords = db.bow[qs][0].tolist()
        pos = {w: p for p, w in enumerate(qwords)}
        cnt = np.zeros(S, np.int64)
        first = np.full(S, 1 << 30)
        for k in range(S):
            if kind == COVIS and ex[k]:
                continue
            common = sets[k].intersection(pos)
            if common:
                cnt[k] = len(common)
                first[k] = min(pos[w] for w in common)
        pushed = (cnt > 0) & (q0 != qid) & ~((kind == LOOP) & ex)
        mx = int(cnt[pushed].max()) if pushed.any() else 0
        mc = int(f32(mx) * f32(0.8))
        cand = np.flatnonzero(pushed & (cnt > mc))
        si = np.zeros(S, np.float32)
        for k in cand:
            si[k] = f32(l1_score(db.bow[qs], db.bow[k]))

        def score_before(n):
            if kind != COVIS:
                for pc, pp, pm, ps in reversed(hist):
                    if pp[n] and pc[n] > pm:
                        return ps[n]
            return s0[n]

        def post(n):
            if q0[n] == qid:
                return True, w0[n] + cnt[n], s0[n]
            if pushed[n]:
                return True, cnt[n], (si[n] if kind != COVIS and cnt[n] > mc else score_before(n))
            return False, 0, 0

        best_acc = f32(0) if kind == RELOC else f32(ms)
        accs = []
        for k in cand:
            if kind != RELOC and not (si[k] >= f32(ms)):
                continue
            acc, best, bk = si[k], si[k], int(k)
            for n in db.covis[k]:
                is_q, wp, sp = post(n)
                if not is_q or (kind != RELOC and not wp > mc):
                    continue
                acc = f32(acc + sp)
                if sp > best:
                    bk, best = n, sp
            accs.append(((first[k], seqs[k]), acc, bk))
            if acc > best_acc:
                best_acc = acc
        retain = f32(0.75) * best_acc
        out, seen = [], set()
        for _, bk in sorted((key, bk) for key, acc, bk in accs if acc > retain):
            if bk not in seen:
                out.append(bk)
                seen.add(bk)
        outs.append(out)
        hist.append((cnt, pushed, mc, si))
    # interaction flag (k_kfdb_state)
    flag = False
    for k in range(S):
        qf, touched = q0[k], False
        for j, (qs, qid, ms, excl) in enumerate(queries):
            if touched and (q0[k] == qid or qf == qid):
                flag = True
            c = hist[j][0][k]
            if c == 0:
                continue
            touched = True
            if qf != qid and not (kind == LOOP and k in set(excl)):
                qf = qid
    return outs, flag
