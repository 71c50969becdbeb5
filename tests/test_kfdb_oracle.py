"""CPU checks of the oracle's keyframe database queries (oracle/kfdb_oracle.cpp, test infrastructure)
against an independent pure-Python restatement (tests/kfdb_cases.py).  Parity status: the reference has
no tests or fixtures for KeyFrameDatabase; both restatements follow
src/KeyFrameDatabase.cc and DBoW2's L1Scoring line by line, including the stale KeyFrame scratch fields
read when a query id repeats."""
import numpy as np
import pytest

from kfdb_cases import LOOP, COVIS, RELOC, PyKfdb, l1_score, make_kfdb_case, run_case, setup_db
from oracle import oracle as O


def _pair(case):
    o = O.Kfdb(case["n_vocab"], case["n_slots"])
    setup_db(case, o)
    p = PyKfdb(case["n_vocab"], case["n_slots"])
    setup_db(case, p, py_style=True)
    return o, p


@pytest.mark.parametrize("seed", range(6))
def test_detect_sequences_match_python(seed):
    case = make_kfdb_case(seed, n_slots=90, n_queries=36)
    o, p = _pair(case)
    ro = run_case(case, o)
    rp = run_case(case, p, py_style=True)
    assert ro == rp
    assert sum(len(r) for r in ro) > 0
    for kind in (LOOP, COVIS, RELOC):
        q, w, s = o.get_state(kind)
        assert np.array_equal(q, p.q[kind]) and np.array_equal(w, p.w[kind]) and np.array_equal(s, p.s[kind])


def test_scores_match_python():
    case = make_kfdb_case(7, n_slots=40)
    o, p = _pair(case)
    rng = np.random.default_rng(1)
    for a, b in rng.integers(0, 40, (200, 2)):
        assert o.score(a, b) == l1_score(case["bows"][a], case["bows"][b])
    assert o.score(3, 3) == pytest.approx(1.0)                        # identical normalised vectors


def test_known_small_database():
    """Hand-computed: query {1:.2, 5:.3, 9:.5}; slot 1 shares 1,5 (score .5), slot 2 shares 5,9 (.8)."""
    o = O.Kfdb(16, 4)
    o.set_bow(0, [1, 5, 9], [0.2, 0.3, 0.5])
    o.set_bow(1, [1, 5, 10], [0.4, 0.4, 0.2])
    o.set_bow(2, [5, 9], [0.5, 0.5])
    o.add([1, 2])
    assert o.score(0, 1) == 0.5 and o.score(0, 2) == 0.8
    assert o.detect(RELOC, 0, 7).tolist() == [2]                      # retain > 0.75 * 0.8
    assert o.detect(LOOP, 0, 8, 0.0).tolist() == [2]
    assert o.detect(LOOP, 0, 9, 0.0, [2]).tolist() == [1]             # slot 2 connected to the query
    assert o.detect(COVIS, 0, 10, 0.9).tolist() == []                 # nothing reaches minScore
    o.set_covisibility({1: [2]})
    # slot 1's neighbour 2 adds its score: acc(1) = .5 + .8 > acc(2) = .8, best keyframe of 1 is 2
    assert o.detect(RELOC, 0, 11).tolist() == [2]
    o.erase([2])
    assert o.detect(RELOC, 0, 12).tolist() == [1]
    o.clear()
    assert o.detect(RELOC, 0, 13).tolist() == []


@pytest.mark.parametrize("seed", range(100, 106))
def test_batched_reformulation_matches_sequential(seed):
    """The GPU's batched form (tests/kfdb_cases.batch_model) equals the sequential queries on every batch
    it does not flag; flagged batches (repeated / stale ids) are re-run one by one by orbx_kfdb_detect."""
    import copy

    from kfdb_cases import batch_model
    case = make_kfdb_case(seed, n_slots=150, n_queries=48, words_hi=400)
    p = PyKfdb(case["n_vocab"], case["n_slots"])
    setup_db(case, p, py_style=True)
    members, seqs, nxt = [False] * case["n_slots"], [None] * case["n_slots"], 0
    n_unflagged = 0
    for op, arg in case["ops"]:
        for k in (arg if op != "query" else []):
            if op == "add":
                p.add(k)
                members[k], seqs[k], nxt = True, nxt, nxt + 1
            else:
                p.erase(k)
                members[k], seqs[k] = False, None
        if op != "query":
            continue
        for kind in (LOOP, COVIS, RELOC):
            qsel = [a for a in arg if a[0] == kind]
            if not qsel:
                continue
            model, flag = batch_model(copy.deepcopy(p), kind, [a[1:] for a in qsel], seqs, members)
            ref = [p.detect(*a) for a in qsel]
            if not flag:
                assert model == ref
                n_unflagged += 1
    assert n_unflagged > 5
