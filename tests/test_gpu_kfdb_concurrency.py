"""One KeyFrameDatabase shared by the reference's threads, on the device API, against the oracle.

The reference's KeyFrameDatabase locks mMutex in add / erase and every Detect* (src/KeyFrameDatabase.cc:42,50,84,210,
316) because Tracking (relocalisation, Tracking.cc:1366), LoopClosing (DetectLoopCandidates then add,
LoopClosing.cc:164,169) and KeyFrame::SetBadFlag (erase, KeyFrame.cc:564) reach it from different threads.  Here the
three run on three host threads, each issuing its device queries on its own HIP stream without synchronising; a
test-side ticket lock records the order in which the calls reached the library.  liborbx orders each operation's
stream after the previous operation (orbx_kfdb's last_op event), so replaying the log on the oracle must give every
candidate list.  A fourth thread reads (n_members, scores) without the ticket lock: the database's own lock orders it."""
import threading

import numpy as np
import pytest

from kfdb_cases import LOOP, RELOC, make_kfdb_case, setup_db

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("strategy", [1, 2, 3])
def test_three_threads_one_database(gpu, strategy):
    import torch

    import multiagent_orb_slam2_amd as pkg
    from oracle import oracle as O
    case = make_kfdb_case(900 + strategy, n_slots=160, n_queries=4, words_hi=300)
    g = pkg.KeyFrameDatabase(case["n_vocab"], case["n_slots"], max_words=2048)
    g.set_strategy(strategy)
    setup_db(case, g)
    g.add(list(range(80)))
    dev = torch.device("cuda", 0)
    ticket = threading.Lock()
    log = []          # (op, slot, id, min_score, excl, (out, out_n, status) or None) in library order
    errors = []

    def call(op, slot, qid=0, ms=0.0, excl=(), stream=None):
        with ticket:
            try:
                if op == "add":
                    g.add([slot])
                    res = None
                elif op == "erase":
                    g.erase([slot])
                    res = None
                else:
                    kind = LOOP if op == "loop" else RELOC
                    qs = torch.tensor([slot], dtype=torch.int32, device=dev)
                    ids = torch.tensor([qid], dtype=torch.int64, device=dev)
                    msd = torch.tensor([ms], dtype=torch.float32, device=dev) if kind == LOOP else None
                    eo = es = None
                    if kind == LOOP:
                        eo = torch.tensor([0, len(excl)], dtype=torch.int32, device=dev)
                        es = torch.tensor(list(excl) or [0], dtype=torch.int32, device=dev)
                    res = g.detect_device(kind, qs, ids, msd, eo, es, stream=stream)
                log.append((op, slot, qid, ms, list(excl), res))
            except Exception as e:   # noqa: BLE001
                errors.append(repr(e))

    def tracking():
        s = torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            for r in range(40):
                call("reloc", 150 + r % 10, 1_000_000 + r, stream=s)

    def loop_closing():
        s = torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            for i in range(40):
                slot = 80 + i
                call("loop", slot, 2_000_000 + i, 0.01, case["covis"][slot], stream=s)
                call("add", slot)

    def set_bad():
        for i in range(30):
            call("erase", i)

    pairs = np.array([[i, (7 * i + 3) % 160] for i in range(64)], np.int32)
    sref = g.score(pairs)
    stop = threading.Event()
    reader_bad = []

    def reader():
        while not stop.is_set():
            n = g.n_members()
            if not 0 <= n <= 160:
                reader_bad.append(n)
            if not np.array_equal(g.score(pairs).view(np.uint64), sref.view(np.uint64)):
                reader_bad.append("score")

    ths = [threading.Thread(target=f) for f in (tracking, loop_closing, set_bad)]
    rd = threading.Thread(target=reader)
    rd.start()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    stop.set()
    rd.join()
    torch.cuda.synchronize()
    assert errors == [] and reader_bad == []

    o = O.Kfdb(case["n_vocab"], case["n_slots"])
    setup_db(case, o)
    o.add(list(range(80)))
    n_cand = 0
    for op, slot, qid, ms, excl, res in log:
        if op in ("add", "erase"):
            getattr(o, op)([slot])
            continue
        kind = LOOP if op == "loop" else RELOC
        ref = list(o.detect(kind, slot, qid, ms, excl))
        out, out_n, status = res
        pkg.KeyFrameDatabase.check_status(status)
        got = out[0, :int(out_n[0].item())].cpu().tolist()
        assert got == ref, (op, slot, qid)
        n_cand += len(ref)
    assert len(log) == 40 + 80 + 30 and n_cand > 0
    for kind in (LOOP, RELOC):
        gq, gw, gs = g.get_state(kind)
        oq, ow, os_ = o.get_state(kind)
        assert np.array_equal(gq, oq) and np.array_equal(gw, ow)
        assert np.array_equal(gs.view(np.uint32), os_.view(np.uint32))
