"""Multi-agent layer: one SLAM agent per GPU, keyframe packets exchanged over RCCL.

Reference behaviour being replaced:
* agents are ``System`` objects in one process fed by one loop; one sequence is split into contiguous
  chunks, the remainder going to the first agents (Examples/MultiAgent/generic_split_seq.cc:543-589);
* every keyframe an agent's LoopClosing processes is handed to the server by pointer
  (src/LoopClosing.cc:83-94 -> MultiAgentServer::InsertKeyFrame -> MapFusion::InsertKeyFrame,
  src/MapFusion.cc:83-88), where MapFusion matches it against other agents' keyframes with
  ORBmatcher::SearchByBoW (src/MapFusion.cc:275, :849).

Here each agent is one process/GPU (rank r = agent r).  A keyframe is a fixed-size packet (header,
keypoints 28 B/slot, descriptors 32 B/slot, MapPoint-valid flag 1 B/slot); packets of all ranks are
all-gathered once per exchange (RCCL on GPUs, gloo on CPU), and cross-agent matching is sharded by
query keyframe: every rank matches its own new keyframes against the gathered keyframes of the other
agents.
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass

import os

import numpy as np

HEADER = 32        # int32 count, agent, frame, n_fv (FeatureVector nodes), n_words (BowVector entries), 3 x pad
KP_BYTES = 28
DESC_BYTES = 32


def split_sequence(n_frames: int, n_agents: int) -> list[range]:
    """Contiguous per-agent chunks, remainder to the first agents (generic_split_seq.cc:543-589)."""
    if n_agents <= 0:
        raise ValueError("n_agents must be positive")
    length, remain = divmod(n_frames, n_agents)
    out, begin = [], 0
    for _ in range(n_agents):
        end = begin + length + (1 if remain > 0 else 0)
        remain = max(remain - 1, 0)
        out.append(range(begin, end))
        begin = end
    return out


def _a16(x: int) -> int:
    return (x + 15) & ~15


class PacketLayout:
    """Byte layout of one keyframe packet (every field 16-byte aligned, so a packet array is directly an
    orbx_kf_store with all strides = packet bytes):

        header 32 | kps cap*28 | desc cap*32 | fv_nodes cap*4 | fv_offsets (cap+1)*4 | fv_indices cap*4 | valid cap
        | bow_words cap*4 | bow_values cap*8

    i.e. what KeyFrame carries into MapFusion: keypoints (angle), descriptors, the BoW FeatureVector
    (KeyFrame::mFeatVec) and MapPoint-valid flags for SearchByBoW (KeyFrame.h:171-185), and the BowVector
    (KeyFrame::mBowVec) for the KeyFrameDatabase query that picks the candidates (src/MapFusion.cc:133)."""

    def __init__(self, capacity: int):
        self.capacity = capacity
        o = HEADER
        self.offsets = {}
        for name, size in (("kps", capacity * KP_BYTES), ("desc", capacity * DESC_BYTES), ("fv_nodes", capacity * 4),
                           ("fv_offsets", (capacity + 1) * 4), ("fv_indices", capacity * 4), ("valid", capacity),
                           ("bow_words", capacity * 4), ("bow_values", capacity * 8)):
            self.offsets[name] = o
            o = _a16(o + size)
        self.bytes = o


def packet_bytes(capacity: int) -> int:
    return PacketLayout(capacity).bytes


def pack_keyframes(kps, desc, counts, valid, agent: int, frames, capacity: int, fv=None):
    """Pack n keyframes into a (n, packet_bytes) uint8 tensor on the same device.

    kps: (n, capacity, 28) uint8, desc: (n, capacity, 32) uint8, counts: (n,) int32,
    valid: (n, capacity) uint8 (keypoint has a MapPoint), frames: (n,) frame ids (device tensor or host list),
    fv: optional dict of the vocabulary batch outputs (fv_nodes (n, cap), fv_offsets (n, cap+1),
    fv_indices (n, cap), n_fv (n,), bow_words / bow_values (n, cap), n_words (n,)), as
    ORBVocabulary.transform_batch_device returns them."""
    import torch
    n = kps.shape[0]
    dev = kps.device
    lay = PacketLayout(capacity)
    out = torch.zeros((n, lay.bytes), dtype=torch.uint8, device=dev)
    n_fv = fv["n_fv"].to(torch.int32) if fv is not None else torch.zeros_like(counts, dtype=torch.int32)
    n_words = fv["n_words"].to(torch.int32) if fv is not None and "n_words" in fv else torch.zeros_like(n_fv)
    if not torch.is_tensor(frames):   # a host list goes through pinned memory on a GPU (a pageable copy stalls)
        f = torch.as_tensor(frames, dtype=torch.int32)
        frames = f.pin_memory().to(dev, non_blocking=True) if dev.type == "cuda" else f.to(dev)
    z = torch.zeros_like(n_fv)
    hdr = torch.stack([counts.to(torch.int32), torch.full_like(counts, agent, dtype=torch.int32),
                       frames.to(torch.int32), n_fv, n_words, z, z, z], 1)
    out[:, :HEADER] = hdr.contiguous().view(torch.uint8).view(n, HEADER)

    def put(name, t, nbytes):
        o = lay.offsets[name]
        out[:, o:o + nbytes] = t.contiguous().view(torch.uint8).reshape(n, -1)

    put("kps", kps, capacity * KP_BYTES)
    put("desc", desc, capacity * DESC_BYTES)
    put("valid", valid, capacity)
    if fv is not None:
        put("fv_nodes", fv["fv_nodes"], capacity * 4)
        put("fv_offsets", fv["fv_offsets"], (capacity + 1) * 4)
        put("fv_indices", fv["fv_indices"], capacity * 4)
        if "bow_words" in fv:
            put("bow_words", fv["bow_words"], capacity * 4)
            put("bow_values", fv["bow_values"], capacity * 8)
    return out


@dataclass
class KeyframeView:
    count: int
    agent: int
    frame: int
    kps: np.ndarray      # structured KP_DTYPE (count,)
    desc: np.ndarray     # (count, 32) uint8
    valid: np.ndarray    # (count,) uint8
    featvec: tuple = None  # (node ids uint32, offsets int32, indices int32) or None
    bow: tuple = None      # BowVector (word ids uint32 ascending, values float64) or None


def unpack_keyframes(packets, capacity: int) -> list[KeyframeView]:
    from .orbx import KP_DTYPE
    p = packets.cpu().numpy() if hasattr(packets, "cpu") else np.asarray(packets)
    lay = PacketLayout(capacity)
    o = lay.offsets
    out = []
    for row in p:
        cnt, agent, frame, n_fv, n_words = row[:HEADER].view(np.int32)[:5]
        kp = row[o["kps"]:o["kps"] + capacity * KP_BYTES].view(KP_DTYPE)[:cnt].copy()
        d = row[o["desc"]:o["desc"] + capacity * DESC_BYTES].reshape(capacity, DESC_BYTES)[:cnt].copy()
        v = row[o["valid"]:o["valid"] + capacity][:cnt].copy()
        fv = None
        if n_fv > 0:
            nodes = row[o["fv_nodes"]:o["fv_nodes"] + 4 * capacity].view(np.uint32)[:n_fv].copy()
            offs = row[o["fv_offsets"]:o["fv_offsets"] + 4 * (capacity + 1)].view(np.int32)[:n_fv + 1].copy()
            idx = row[o["fv_indices"]:o["fv_indices"] + 4 * capacity].view(np.int32)[:offs[-1]].copy()
            fv = (nodes, offs, idx)
        bow = None
        if n_words > 0:
            bow = (row[o["bow_words"]:o["bow_words"] + 4 * capacity].view(np.uint32)[:n_words].copy(),
                   row[o["bow_values"]:o["bow_values"] + 8 * capacity].view(np.float64)[:n_words].copy())
        out.append(KeyframeView(int(cnt), int(agent), int(frame), kp, d, v, fv, bow))
    return out


class KeyframeExchange:
    """All-gather of keyframe packets: the MapFusion ingress (src/MapFusion.cc:83-88) as one collective.

    Works with the ``nccl`` (RCCL over xGMI) and ``gloo`` backends.  With timed=True (GPU tensors) every call is
    bracketed by HIP events on the current stream, so stats() reports the time from the stream reaching the
    collective to its completion, per call, and the rate at which each rank receives the other ranks' bytes."""

    def __init__(self, group=None, timed: bool = False):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.bytes_moved = 0
        self.calls = 0
        self.timed = timed
        self._events = []

    def exchange(self, packets, out=None):
        """packets: (n, P) uint8 on this rank (same n and P on every rank) -> (world*n, P), rank-major
        (written into `out` when given, e.g. a slice of a DeviceKeyframeStore ring)."""
        import torch
        n, P = packets.shape
        if out is None:
            out = torch.empty((self.world * n, P), dtype=torch.uint8, device=packets.device)
        ev = None
        if self.timed and packets.is_cuda:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        if packets.is_cuda and self.dist.get_backend(self.group) == "gloo":
            # gloo gathers host tensors only: stage through host memory (rehearsal of the N>1 path on one GPU)
            host = [torch.empty((n, P), dtype=torch.uint8) for _ in range(self.world)]
            self.dist.all_gather(host, packets.cpu(), group=self.group)
            out.copy_(torch.cat(host, 0).to(out.device))
        elif hasattr(self.dist, "all_gather_into_tensor") and packets.is_cuda:
            self.dist.all_gather_into_tensor(out, packets.contiguous(), group=self.group)
        else:
            parts = list(out.chunk(self.world, 0))
            self.dist.all_gather(parts, packets.contiguous(), group=self.group)
        if ev is not None:
            ev[1].record()
            self._events.append((ev, out.numel()))
        self.bytes_moved += out.numel()
        self.calls += 1
        return out

    def reset_stats(self):
        self._events = []

    def stats(self):
        """Timed calls since reset_stats(): mean microseconds per all-gather, bytes gathered per call (all ranks'
        packets), bytes received per rank per call ((world-1)/world of them) and that received rate in GB/s."""
        if not self._events:
            return None
        us = [a.elapsed_time(b) * 1e3 for (a, b), _ in self._events]
        nbytes = float(np.mean([nb for _, nb in self._events]))
        recv = nbytes * (self.world - 1) / self.world
        mean_us = float(np.mean(us))
        return {"calls": len(us), "us_per_allgather": round(mean_us, 2), "us_min": round(float(np.min(us)), 2),
                "bytes_per_allgather": int(nbytes), "bytes_received_per_rank": int(recv),
                "recv_GBps": round(recv / (mean_us * 1e-6) / 1e9, 3) if mean_us > 0 else None}


class NativeKeyframeExchange(KeyframeExchange):
    """The same all-gather through liborbx's own RCCL communicator (orbx_exchange, KeyframeExchangeRCCL): what a C++
    MultiAgentServer without torch would call.  The communicator's unique id is made on rank 0 and handed to the others
    over the torch process group (broadcast_object_list), then every call is stream-ordered on the current stream."""

    def __init__(self, group=None, timed: bool = False, device: int = 0):
        super().__init__(group, timed)
        from .orbx import KeyframeExchangeRCCL
        uid = [KeyframeExchangeRCCL.unique_id() if self.rank == 0 else None]
        self.dist.broadcast_object_list(uid, src=0, group=group)
        self.x = KeyframeExchangeRCCL(uid[0], self.world, self.rank, device)

    def exchange(self, packets, out=None):
        import torch
        n, P = packets.shape
        if out is None:
            out = torch.empty((self.world * n, P), dtype=torch.uint8, device=packets.device)
        stream = torch.cuda.current_stream(packets.device)
        ev = None
        if self.timed:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record(stream)
        self.x.allgather(packets.contiguous(), out, stream=stream)
        if ev is not None:
            ev[1].record(stream)
            self._events.append((ev, out.numel()))
        self.bytes_moved += out.numel()
        self.calls += 1
        return out

    def close(self):
        self.x.close()


def allgather_sweep(exchange: KeyframeExchange, device, sizes_mb, reps: int = 10, warmup: int = 3):
    """All-gather bandwidth over the exchange's collective at several per-rank payloads: mean microseconds per call
    (HIP events on the current stream), the bytes each rank receives ((world-1) x payload) per second, and the
    ring-algorithm bus bandwidth (payload x (world-1) / time = the bytes each rank receives per second), the algorithm
    bandwidth (world x payload / time) beside it; data_ok checks every rank's block arrived."""
    import torch
    out = []
    w = exchange.world
    for mb in sizes_mb:
        nbytes = max(16, int(mb * 1e6) // 16 * 16)
        send = torch.full((1, nbytes), exchange.rank & 0xFF, dtype=torch.uint8, device=device)
        recv = torch.empty((w, nbytes), dtype=torch.uint8, device=device)
        for _ in range(warmup):
            exchange.exchange(send, out=recv)
        s = torch.cuda.current_stream(device)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        saved = exchange.timed
        exchange.timed = False
        e0.record(s)
        for _ in range(reps):
            exchange.exchange(send, out=recv)
        e1.record(s)
        e1.synchronize()
        exchange.timed = saved
        us = e0.elapsed_time(e1) * 1e3 / reps
        ok = bool(all(int(recv[r, 0].item()) == (r & 0xFF) and int(recv[r, -1].item()) == (r & 0xFF) for r in range(w)))
        recv_b = nbytes * (w - 1)
        out.append({"bytes_per_rank": nbytes, "us_per_allgather": round(us, 2),
                    "algbw_GBps": round(w * nbytes / (us * 1e-6) / 1e9, 2),
                    "busbw_GBps": round(recv_b / (us * 1e-6) / 1e9, 2), "data_ok": ok})
    return out


class MapFusionStore:
    """Every agent's keyframes as seen by this rank's fusion matcher."""

    def __init__(self):
        self.keyframes: list[KeyframeView] = []

    def insert(self, kfs: list[KeyframeView]):
        self.keyframes.extend(kfs)

    def candidates_for(self, agent: int) -> list[KeyframeView]:
        """Keyframes of the other agents (MapFusion drops same-map candidates, src/MapFusion.cc:136-144)."""
        return [k for k in self.keyframes if k.agent != agent]


def cross_agent_match(matcher, query: KeyframeView, query_fv, candidates: list[KeyframeView], featvec_of,
                      min_matches: int = 20):
    """MapFusion::ComputeSim3's first gate (src/MapFusion.cc:275-281): SearchByBoW(curKF, candKF) for every
    candidate; candidates with >= min_matches (20 in the reference) go on to Sim3 RANSAC (out of scope).
    Returns [(candidate index, nmatches, match12)]."""
    out = []
    for ci, c in enumerate(candidates):
        n, m12 = matcher.SearchByBoW_KF_KF(query.desc, query.kps["angle"], query.valid, query_fv,
                                           c.desc, c.kps["angle"], c.valid, featvec_of(c))
        out.append((ci, n, m12, n >= min_matches))
    return out


class DeviceKeyframeStore:
    """MapFusion's keyframe store on the GPU: a ring of `slots` keyframe packets (PacketLayout) that the
    exchange all-gathers into directly, seen by the matcher as one orbx_kf_store (all strides = packet
    bytes).  Host-side bookkeeping records which agent owns each slot and the insertion order."""

    def __init__(self, capacity: int, slots: int, device):
        import torch
        self.layout = PacketLayout(capacity)
        self.capacity = capacity
        self.slots = slots
        self.buf = torch.zeros((slots, self.layout.bytes), dtype=torch.uint8, device=device)
        self.agent_of = [-1] * slots
        self.stamp = [-1] * slots        # insertion sequence number per slot
        self.pos = 0
        self.seq = 0
        self._store = None

    def _reserve(self, n: int) -> int:
        if n > self.slots:
            raise ValueError(f"{n} keyframes do not fit a store of {self.slots} slots")
        if self.pos + n > self.slots:
            self.pos = 0
        base = self.pos
        self.pos += n
        return base

    def _record(self, base: int, agents):
        for i, a in enumerate(agents):
            self.agent_of[base + i] = int(a)
            self.stamp[base + i] = self.seq
            self.seq += 1

    def insert(self, packets, agent: int) -> range:
        """Local insert (single agent): copy packets into the ring; returns their slots."""
        n = packets.shape[0]
        base = self._reserve(n)
        self.buf[base:base + n].copy_(packets)
        self._record(base, [agent] * n)
        return range(base, base + n)

    def exchange_into(self, exchange: "KeyframeExchange", packets) -> range:
        """All-gather every rank's packets straight into the ring (rank-major); returns the new slots."""
        n = packets.shape[0]
        w = exchange.world
        base = self._reserve(w * n)
        exchange.exchange(packets, out=self.buf[base:base + w * n])
        self._record(base, [r for r in range(w) for _ in range(n)])
        return range(base, base + w * n)

    def ingest(self, packets, agent: int, exchange: "KeyframeExchange" = None):
        """This step's keyframes into the ring: all-gathered from every rank when an exchange with world > 1 is
        given (rank-major), else inserted locally.  Returns (new slots, this agent's slots among them, the agent
        of every new slot).  The slot order is the order MapFusion processes them in (query, then add)."""
        n = packets.shape[0]
        if exchange is not None and exchange.world > 1:
            new = self.exchange_into(exchange, packets)
            mine = range(new.start + exchange.rank * n, new.start + (exchange.rank + 1) * n)
        else:
            new = self.insert(packets, agent)
            mine = new
        return new, mine, [self.agent_of[s] for s in new]

    def kf_store(self):
        """orbx_kf_store over the ring (pointers are fixed for the store's lifetime)."""
        if self._store is None:
            from .orbx import KfStore
            P, o, b = self.layout.bytes, self.layout.offsets, self.buf
            f = lambda name: (b[0, o[name]:], P)
            self._store = KfStore.from_fields(self.capacity, desc=f("desc"), kps=f("kps"), valid=f("valid"),
                                              fv_nodes=f("fv_nodes"), fv_offsets=f("fv_offsets"),
                                              fv_indices=f("fv_indices"), n_fv=(b[0, 12:], P))
        return self._store

    def candidate_pairs(self, query_slots, agent: int, k: int, other_agents_only: bool = True) -> np.ndarray:
        """(query, candidate) slot pairs: for every query, the k most recently inserted keyframes of the
        other agents (MapFusion drops same-map candidates, src/MapFusion.cc:136-144) -- or, with
        other_agents_only=False (single agent: LoopClosing's own-map candidates), the k keyframes inserted
        most recently before it.  Stands in for KeyFrameDatabase::DetectMapFusionCandidates's BoW scoring
        (src/KeyFrameDatabase.cc:199-308)."""
        filled = [s for s in range(self.slots) if self.stamp[s] >= 0]
        by_recency = sorted(filled, key=lambda s: -self.stamp[s])
        pairs = []
        for q in query_slots:
            if other_agents_only:
                c = [s for s in by_recency if self.agent_of[s] != agent]
            else:
                c = [s for s in by_recency if self.stamp[s] < self.stamp[q]]
            pairs.extend((q, s) for s in c[:k])
        return np.array(pairs, np.int32).reshape(-1, 2)


class KeyframeFusion:
    """The per-agent keyframe path after the front-end, all on the device:

        new keyframes (extractor batch rows) -> ORBVocabulary::transform (BowVector + FeatureVector at level
        L-4, src/KeyFrame.cc ComputeBoW) -> packets -> all-gather into every rank's DeviceKeyframeStore
        (MapFusion ingress, src/MapFusion.cc:83-88) -> for every exchanged keyframe in order: DetectLoopCandidates
        (src/MapFusion.cc:133), then the keyframe joins the database (:149 / :222) -- queries sharded by keyframe:
        each rank answers its own keyframes' queries on its replica of the database -> first k candidates of
        another map (:136-144) -> SearchByBoW(new KF, candidate) (:275) -> the 20-match gate (:275-281).

    The database covers the store ring: a slot leaves it when the ring overwrites it.  The query-then-add order
    is one sequential detect per step (orbx_kfdb_detect_sequential_device): the step's slots are added in
    processing order (rank-major) and each query sees only what was added before it, so a later keyframe of
    the step -- also another agent's -- can be a candidate of the next one, exactly as in MapFusion's loop.
    Query ids are global keyframe sequence numbers (KeyFrame::mnId), fresh per keyframe.  There is no
    covisibility graph in this front-end-only pipeline, so queries exclude nothing and use minScore 0 (the
    reference bounds it by the scores of the query's covisible keyframes, :100-131).  With one agent (no
    exchange) candidates may come from the agent's own map, as LoopClosing's (src/LoopClosing.cc:164).

    vocab / matcher / db are the library objects (ORBVocabulary, ORBmatcher, KeyFrameDatabase); tests on CPU
    pass oracle-backed doubles with the same methods."""

    def __init__(self, matcher, vocab, capacity: int, slots: int, device, agent: int = 0, exchange=None,
                 candidates: int = 16, levelsup: int = 4, min_matches: int = 20, db=None):
        import torch

        if exchange is not None and getattr(exchange, "world", 1) > 1 and agent != exchange.rank:
            # the slot groups of a step are rank-major (rank r's packets are group r) and the query group is the
            # agent: they must be one number, or the same-map discard (MapFusion.cc:136-144) compares different ids
            raise ValueError(f"agent {agent} != exchange rank {exchange.rank}: one agent per rank")
        self.matcher, self.vocab, self.capacity = matcher, vocab, capacity
        self.store = DeviceKeyframeStore(capacity, slots, device)
        self.agent, self.exchange = agent, exchange
        self.k, self.levelsup, self.min_matches = candidates, levelsup, min_matches
        info = vocab.info()
        self.max_fv_nodes = min(capacity, info["k"] ** max(info["L"] - levelsup, 0) + 1)   # launch width hint
        if db is None:
            from .orbx import KeyFrameDatabase
            dev_index = device.index if getattr(device, "index", None) is not None else 0
            db = KeyFrameDatabase(info["n_words"], slots, max_words=min(capacity, 4096), device=dev_index)
        self.db = db
        self.device = device
        self._slot_tensors = {}
        self._next_id = 1
        self.slot_group = torch.full((slots,), -1, dtype=torch.int32, device=device)   # map (agent) of each slot
        self.status = torch.zeros((1,), dtype=torch.int32, device=device)             # orbx_kfdb_detect_device flags

    def _cached(self, key, make):
        t = self._slot_tensors.get(key)
        if t is None:
            t = make()
            self._slot_tensors[key] = t
        return t

    def _slots(self, r: range):
        import torch
        return self._cached((r.start, r.stop), lambda: torch.arange(r.start, r.stop, dtype=torch.int32, device=self.device))

    def step(self, kps, desc, counts, valid, frames, stream=None):
        """kps (n, cap, 28) u8, desc (n, cap, 32) u8, counts (n,), valid (n, cap) u8: this agent's new
        keyframes.  Returns (pairs (n*k, 2) device, match12 (n*k, cap), nmatches (n*k,), passed (n*k,) bool);
        pairs (query, -1) are padding (fewer than k candidates) with no matches."""
        import torch
        n = kps.shape[0]
        fv = self.vocab.transform_batch_device(desc.contiguous(), counts.contiguous(), self.levelsup, stream=stream)
        pk = pack_keyframes(kps, desc, counts, valid, self.agent, frames, self.capacity, fv)
        new, mine, agents = self.store.ingest(pk, self.agent, self.exchange)
        multi = len(new) != len(mine)
        w = len(new) // max(n, 1)
        grp = self._cached(("group", w, n), lambda: torch.arange(w * n, dtype=torch.int32, device=self.device) // n)
        if multi:
            self.slot_group[new.start:new.stop].copy_(grp)
        else:
            self.slot_group[new.start:new.stop].fill_(self.agent)
        # the ring overwrote these slots: they leave the database and take the new BowVectors; then they join it
        # in processing order, and the sequential detect answers each query as if it ran before its own add
        self.db.erase(list(new))
        P, o = self.store.layout.bytes, self.store.layout.offsets
        rows = self.store.buf[new.start:new.stop]
        self.db.set_bow_device(self._slots(new), rows[:, o["bow_words"]:], rows[:, o["bow_values"]:], rows[:, 16:],
                               strides=(P // 4, P // 8, P // 4), stream=stream)
        self.db.add(list(new))
        q = self._slots(mine)
        first = self._next_id + (mine.start - new.start)       # global keyframe ids in processing order
        ids = torch.arange(first, first + n, dtype=torch.int64, device=self.device)
        self._next_id += len(new)
        zeros = self._cached(("zeros", n), lambda: torch.zeros((n,), dtype=torch.float32, device=self.device))
        cand, n_cand, _ = self.db.detect_device(0, q, ids, zeros, status=self.status, stream=stream, sequential=True)
        if multi:
            qg = self._cached(("qgroup", n), lambda: torch.full((n,), self.agent, dtype=torch.int32, device=self.device))
            pr = self.db.candidate_pairs_device(cand, n_cand, q, self.k, self.slot_group, qg, stream=stream)
        else:
            pr = self.db.candidate_pairs_device(cand, n_cand, q, self.k, stream=stream)
        m12, nm = self.matcher.SearchByBoW_pairs_device(self.store.kf_store(), pr, self.max_fv_nodes, stream=stream)
        return pr, m12, nm, nm >= self.min_matches

    def check(self):
        """Raise if any detect so far reported interacting queries or exceeded capacity (synchronises)."""
        from .orbx import KeyFrameDatabase
        KeyFrameDatabase.check_status(self.status)


class CovisibilityDiscovery:
    """MapFusion::CovisibilityDiscovery's detection and matching (src/MapFusion.cc:774-885) over device keyframes.

    For every keyframe of the absorbed map (query slots, processed in order as the reference's loop does): minScore =
    the smallest ORBVocabulary::score against its covisible keyframes, starting at 1 and kept in a float (:801-816);
    DetectCovisibilityCandidates(KF, minScore, vpCurrentMapKFs) on the matched map's database (:819-820, the whole
    absorbed map ignored); SearchByBoW(KF, candidate) with ORBmatcher(0.75, true) for every candidate (:840-856), a
    candidate kept with >= 15 matches.  The queries use fresh keyframe ids and the COVIS scratch fields only, so the
    batch equals the sequential loop (the database reports any interaction in its status word).  The Fuse step that
    follows (:903-910: projection search and map edits on the CPU's map) is outside the hot path.

    db: KeyFrameDatabase holding the matched map's keyframes as members; store: orbx_kf_store (KfStore) over every
    slot (both maps); matcher: ORBmatcher(0.75, True).  Runs on the current torch stream."""

    def __init__(self, matcher, db, store, max_fv_nodes: int, min_matches: int = 15):
        self.matcher, self.db, self.store = matcher, db, store
        self.max_fv_nodes, self.min_matches = max_fv_nodes, min_matches

    def run(self, query_slots, query_ids, covisible, ignore):
        """query_slots / query_ids: the absorbed map's keyframes (lists); covisible[i]: slots of query i's covisible
        keyframes (GetVectorCovisibleKeyFrames); ignore: vpCurrentMapKFs.  Returns (pairs (P, 2), match12 (P, cap),
        nmatches (P,), passed (P,)) device tensors and the per-query candidate counts (host; one synchronisation)."""
        import torch

        from .orbx import KFDB_COVIS, KeyFrameDatabase
        dev = self.store._keep[0].device
        nq = len(query_slots)
        q = torch.tensor(query_slots, dtype=torch.int32, device=dev)
        ids = torch.tensor(query_ids, dtype=torch.int64, device=dev)
        ms = torch.ones((nq,), dtype=torch.float32, device=dev)          # float minScore = 1 (:805)
        sp = [(query_slots[i], c) for i in range(nq) for c in covisible[i]]
        if sp:
            sc = self.db.score_device(torch.tensor(sp, dtype=torch.int32, device=dev))
            owner = torch.tensor([i for i in range(nq) for _ in covisible[i]], dtype=torch.int64, device=dev)
            ms.scatter_reduce_(0, owner, sc.to(torch.float32), reduce="amin", include_self=True)
        n_ign = len(ignore)
        excl_slots = torch.tensor(list(ignore) * nq if n_ign else [0], dtype=torch.int32, device=dev)
        excl_off = torch.arange(0, nq + 1, dtype=torch.int32, device=dev) * n_ign
        cand, n_cand, status = self.db.detect_device(KFDB_COVIS, q, ids, ms, excl_off, excl_slots)
        n_host = n_cand.cpu().numpy()
        KeyFrameDatabase.check_status(status)
        k = max(1, int(n_host.max()) if nq else 1)
        pr = KeyFrameDatabase.candidate_pairs_device(cand, n_cand, q, k)
        m12, nm = self.matcher.SearchByBoW_pairs_device(self.store, pr, self.max_fv_nodes)
        return pr, m12, nm, nm >= self.min_matches, n_host


def triangulation_geometry(K, Rcw, tcw, pairs):
    """F12 = K1^-T [t12]x R12 K2^-1 with R12 = R1w R2w^T, t12 = -R12 t2w + t1w (LocalMapping::ComputeF12,
    src/LocalMapping.cc:542-557) and the epipole of KF1's centre in KF2 (ORBmatcher.cc:666-672) for (kf1, kf2) index
    pairs into per-keyframe poses.  K (3, 3), Rcw (N, 3, 3), tcw (N, 3), pairs (P, 2) integer tensors (any device, one
    intrinsics for all keyframes); float32 arithmetic.  Returns (P, 12) rows [F12 row-major, ex, ey, 0] for
    ORBmatcher.SearchForTriangulation_pairs_device; rows of pairs with a negative index are zero."""
    import torch
    K = K.to(torch.float32)
    p = pairs.long().clamp(min=0)
    R1, t1 = Rcw[p[:, 0]].float(), tcw[p[:, 0]].float()
    R2, t2 = Rcw[p[:, 1]].float(), tcw[p[:, 1]].float()
    R12 = R1 @ R2.transpose(1, 2)
    t12 = -(R12 @ t2[:, :, None])[:, :, 0] + t1
    z = torch.zeros_like(t12[:, 0])
    tx = torch.stack([z, -t12[:, 2], t12[:, 1], t12[:, 2], z, -t12[:, 0], -t12[:, 1], t12[:, 0], z], 1).view(-1, 3, 3)
    Kinv = torch.linalg.inv(K)
    F = Kinv.T[None] @ tx @ R12 @ Kinv[None]
    C1 = -(R1.transpose(1, 2) @ t1[:, :, None])[:, :, 0]                   # Ow1 = -R1w^T t1w
    C2 = (R2 @ C1[:, :, None])[:, :, 0] + t2
    iz = 1.0 / C2[:, 2]
    ex = K[0, 0] * C2[:, 0] * iz + K[0, 2]
    ey = K[1, 1] * C2[:, 1] * iz + K[1, 2]
    g = torch.cat([F.reshape(-1, 9), ex[:, None], ey[:, None], z[:, None]], 1).contiguous()
    return torch.where((pairs.long() >= 0).all(1)[:, None], g, torch.zeros_like(g))


def neighbour_observations(new_slots, neighbours, match12):
    """Observation lists of the MapPoints CreateNewMapPoints makes, built on the device without a host round trip
    (LocalMapping.cc:244-448): keypoint i of new keyframe j becomes a MapPoint at most once, with the first neighbour k
    (in order) whose match match12[j, k, i] >= 0, observed [(neighbour k, its match), (new keyframe j, i)] -- creation
    order, the pin of mObservations' KeyFrame* order; no match, no MapPoint (an empty list).  new_slots
    (n,), neighbours (n, nn) slots (-1 = none), match12 (n, nn, capacity).  Returns (obs (n*capacity*2, 2) int32 --
    the first offsets[-1] rows used, offsets (n*capacity + 1,) int32) for ORBmatcher.distinctive_descriptors_store_device."""
    import torch
    n, nn, cap = match12.shape
    dev = match12.device
    hit = (match12 >= 0) & (neighbours.view(n, nn, 1) >= 0)                 # (n, nn, cap)
    has = hit.any(1)                                                        # (n, cap)
    first = torch.argmax(hit.int(), 1)                                      # first neighbour with a match
    nb_slot = torch.gather(neighbours.int(), 1, first)                      # (n, cap)
    nb_kp = torch.gather(match12.int(), 1, first.view(n, 1, cap)).view(n, cap)
    cnt = has.view(-1).int() * 2
    offsets = torch.zeros((n * cap + 1,), dtype=torch.int32, device=dev)
    offsets[1:] = torch.cumsum(cnt, 0)
    pair = torch.stack([torch.stack([nb_slot, nb_kp], 2),
                        torch.stack([new_slots.view(n, 1).expand(n, cap).int(),
                                     torch.arange(cap, dtype=torch.int32, device=dev).view(1, cap).expand(n, cap)], 2)],
                       2).view(n * cap, 2, 2)
    obs = pair[has.view(-1)].reshape(-1, 2)
    full = torch.zeros((n * cap * 2, 2), dtype=torch.int32, device=dev)
    full[:obs.shape[0]] = obs
    return full, offsets


class NewMapPoints:
    """LocalMapping::CreateNewMapPoints' matching for a batch of new keyframes (src/LocalMapping.cc:213-274): every new
    keyframe against its best covisible neighbours with ORBmatcher(0.6, false).SearchForTriangulation, all pairs in
    one launch, then ComputeDistinctiveDescriptors of the MapPoints it creates (:440-448: a keypoint with its first
    matching neighbour, two observations -- neighbour_observations' lists), read from the match table in place
    (orbx_distinctive_descriptors_neighbours_device).

    The reference visits the neighbours of one keyframe in turn and a keypoint triangulated with neighbour k is
    skipped for neighbours k' > k; here every pair reads the MapPoint flags given (has_mp) and the pair results are
    exactly those of SearchForTriangulation on that state -- the pose checks, SVD triangulation and map insertion
    that decide which matches become MapPoints run on the map side (out of the hot path)."""

    def __init__(self, store, max_fv_nodes: int, sigma2, scale, matcher=None, only_stereo: bool = False):
        from .orbx import ORBmatcher
        self.store, self.max_fv_nodes = store, max_fv_nodes
        self.sigma2 = np.ascontiguousarray(sigma2, np.float32)
        self.scale = np.ascontiguousarray(scale, np.float32)
        self.matcher = matcher if matcher is not None else ORBmatcher(0.6, False)
        self.only_stereo = only_stereo

    def run(self, new_slots, neighbours, geom, has_mp=None, uright=None):
        """new_slots (n,), neighbours (n, nn) int32 device tensors (-1 = no neighbour), geom (n, nn, 12) rows from
        triangulation_geometry.  Returns (match12 (n, nn, cap), nmatches (n, nn), best, descriptors): best[j*cap + i] =
        index in neighbour_observations' list of MapPoint (j, i), descriptors its distinctive descriptor."""
        import torch
        n, nn = neighbours.shape
        cap = self.store.capacity
        k1 = new_slots.view(n, 1).expand(n, nn).int()
        pairs = torch.stack([torch.where(neighbours >= 0, k1, torch.full_like(k1, -1)), neighbours.int()], 2)
        m12, nm = self.matcher.SearchForTriangulation_pairs_device(
            self.store, pairs.view(-1, 2).contiguous(), geom.reshape(-1, 12).contiguous(), self.sigma2, self.scale,
            self.max_fv_nodes, has_mp=has_mp, uright=uright, bOnlyStereo=self.only_stereo)
        m12 = m12.view(n, nn, cap)
        best, desc = self.matcher.distinctive_descriptors_neighbours_device(self.store, new_slots.int().contiguous(),
                                                                           neighbours.int().contiguous(), m12)
        return m12, nm.view(n, nn), best, desc


# ---------------------------------------------------------------------------------------------------------------------
# Per-frame tracking matches and LocalMapping's Fuse on the device: the reference's callers of the
# projection matchers, batched.  The poses are the caller's (the reference's motion model and optimisation are out of
# scope); these classes run the matching work a Tracking / LocalMapping thread issues for them.
# ---------------------------------------------------------------------------------------------------------------------
def problem_table(rows, **cols):
    """ProjProblem structs (include/orbx.h orbx_proj_problem, 112 B) as a (rows, 14) int64 array: each keyword is a
    field name with an int (the same for every row) or a (rows,) int array; pointer fields hold addresses, nq / n their
    counts (the little-endian low half of the 8-byte slot, the padding zero)."""
    order = ["queries", "qdesc", "nq", "kps", "desc", "uright", "blocked", "n", "cell_start", "cell_idx", "q_idx",
             "q_dist", "owner", "nmatches"]
    t = np.zeros((rows, 14), np.int64)
    for k, v in cols.items():
        t[:, order.index(k)] = v
    return t


class FrameTracker:
    """Tracking's matching for a batch of stereo frames (src/Tracking.cc), each against its last frame:
    TrackWithMotionModel (:882-904): the last frame's MapPoints (UpdateLastFrame's stereo points, :823-880 -- made here
    by orbx_stereo_mappoints from its depths and pose) projected into the current frame (orbx_proj_project, LASTFRAME)
    and SearchByProjection(CurrentFrame, LastFrame, th=7) with ORBmatcher(0.9, true); then TrackLocalMap's
    SearchLocalPoints (:1160-1205): the MapPoints not matched yet through isInFrustum(0.5) and
    SearchByProjection(F, vpLocalMapPoints, th=1) with ORBmatcher(0.8), keypoints that got a MapPoint in the first search
    excluded (:92-93 Observations() > 0).  The current frame's grid is Frame::AssignFeaturesToGrid (orbx_grid_build).
    One launch per stage over the whole batch; buffers per output set (n_sets), problem tables built once per set.
    For the bench the last frame of frame i is frame i itself seen from pose 'last' (its keypoints as the MapPoints'
    observations), and the current pose is 'last' moved by a residual motion -- the motion model's prediction error.
    The last frame holds the MapPoints of the even keypoints; the local map holds all of them."""

    def __init__(self, matcher, batch: int, capacity: int, grid, camera, bf: float, scale, log_sf: float, device,
                 n_sets: int, twc_last, view_last_frame, view_local_map, inv_sigma2):
        import torch
        from .orbx import PROJ_LASTFRAME, PROJ_MAPPOINTS, ProjParams
        self.m, self.B, self.cap, self.grid = matcher, batch, capacity, grid
        self.camera = np.ascontiguousarray(camera, np.float32)
        self.scale = np.ascontiguousarray(scale, np.float32)
        self.log_sf = float(log_sf)
        dev = torch.device("cuda", device) if isinstance(device, int) else device
        self.dev = dev
        B, cap = batch, capacity
        ncell = grid.cols * grid.rows
        self.twc = torch.from_numpy(np.tile(np.asarray(twc_last, np.float32).reshape(1, 12), (B, 1))).to(dev)
        self.v_lf = torch.from_numpy(np.tile(_view_bytes(view_last_frame), (B, 1))).to(dev)
        self.v_mp = torch.from_numpy(np.tile(_view_bytes(view_local_map), (B, 1))).to(dev)
        self.p_lf = ProjParams.make(PROJ_LASTFRAME, 100, 0.9, True, inv_sigma2)          # ORBmatcher(0.9, true), TH_HIGH
        self.p_mp = ProjParams.make(PROJ_MAPPOINTS, 100, 0.8, False, inv_sigma2)         # ORBmatcher(0.8), TH_HIGH
        # the last frame holds the MapPoints of every second keypoint (its tracked points); the local map holds all of
        # them, so SearchLocalPoints has the other half plus the motion-model misses to find (found >= 0: skipped)
        self.lf_skip = torch.tensor([-1, 0], dtype=torch.int32).repeat(B, (cap + 1) // 2)[:, :cap].contiguous().to(dev)
        self.sets = []
        for _ in range(n_sets):
            z = dict(pts=torch.empty((B, cap, 48), dtype=torch.uint8, device=dev),
                     q1=torch.empty((B, cap, 40), dtype=torch.uint8, device=dev),
                     q2=torch.empty((B, cap, 40), dtype=torch.uint8, device=dev),
                     cs=torch.empty((B, ncell + 1), dtype=torch.int32, device=dev),
                     ci=torch.empty((B, cap), dtype=torch.int32, device=dev),
                     ur=torch.empty((B, cap), dtype=torch.float32, device=dev),
                     depth=torch.empty((B, cap), dtype=torch.float32, device=dev),
                     blk=torch.empty((B, cap), dtype=torch.bool, device=dev))
            for k in ("qi1", "qd1", "qi2", "qd2"):
                z[k] = torch.empty((B, cap), dtype=torch.int32, device=dev)
            for k in ("own1", "own2", "fnd"):
                z[k] = torch.empty((B, cap), dtype=torch.int32, device=dev)
            for k in ("nm1", "nm2"):
                z[k] = torch.empty((B,), dtype=torch.int32, device=dev)
            z["probs"] = {}
            self.sets.append(z)

    def stereo_out(self, s: int):
        """(uright, depth) buffers of set s, for ORBmatcher.stereo_refine_batch_device(out=...)."""
        return self.sets[s]["ur"], self.sets[s]["depth"]

    def _problems(self, z, kps, desc):
        import torch
        key = (kps.data_ptr(), desc.data_ptr())
        if key not in z["probs"]:
            B, cap = self.B, self.cap
            i = np.arange(B, dtype=np.int64)
            common = dict(nq=cap, kps=kps.data_ptr() + i * cap * 28, desc=desc.data_ptr() + i * cap * 32,
                          qdesc=desc.data_ptr() + i * cap * 32, uright=z["ur"].data_ptr() + i * cap * 4, n=cap,
                          cell_start=z["cs"].data_ptr() + i * z["cs"].shape[1] * 4, cell_idx=z["ci"].data_ptr() + i * cap * 4)
            t1 = problem_table(B, queries=z["q1"].data_ptr() + i * cap * 40, q_idx=z["qi1"].data_ptr() + i * cap * 4,
                               q_dist=z["qd1"].data_ptr() + i * cap * 4, owner=z["own1"].data_ptr() + i * cap * 4,
                               nmatches=z["nm1"].data_ptr() + i * 4, **common)
            t2 = problem_table(B, queries=z["q2"].data_ptr() + i * cap * 40, q_idx=z["qi2"].data_ptr() + i * cap * 4,
                               q_dist=z["qd2"].data_ptr() + i * cap * 4, owner=z["own2"].data_ptr() + i * cap * 4,
                               nmatches=z["nm2"].data_ptr() + i * 4, blocked=z["blk"].data_ptr() + i * cap, **common)
            z["probs"][key] = (torch.from_numpy(t1.view(np.uint8)).to(self.dev), torch.from_numpy(t2.view(np.uint8)).to(self.dev))
        return z["probs"][key]

    def run(self, s: int, kps, desc, counts, stream=None):
        """Frames kps / desc / counts (B, cap, 28) / (B, cap, 32) / (B,) with the stereo results already in set s's
        (uright, depth).  Returns (q_idx motion model, nmatches, q_idx local map, nmatches) tensors of set s."""
        from .orbx import PROJ_LASTFRAME, PROJ_MAPPOINTS, QF_BLOCKS
        z, m, cap = self.sets[s], self.m, self.cap
        p1, p2 = self._problems(z, kps, desc)
        m.stereo_mappoints_device(kps, z["depth"], counts, self.twc, self.camera, self.scale, QF_BLOCKS, out=z["pts"],
                                  stream=stream)
        m.proj_project_device(PROJ_LASTFRAME, z["pts"], counts, self.v_lf, self.scale, self.log_sf, out=z["q1"],
                              found=self.lf_skip, stream=stream)
        if os.environ.get("ORBX_TRACK_GRID_LAUNCH"):               # A/B only: Frame::AssignFeaturesToGrid as its own launch
            m.grid_build_device(self.grid, kps, counts, stream=stream, out=(z["cs"], z["ci"]))
            m.proj_search_batch_device(self.p_lf, self.grid, p1, cap, cap, stream=stream)
        else:
            # the frame's grid (Frame::AssignFeaturesToGrid) built inside the motion-model search, which writes it out
            # for the local-map search: one 1024-thread workgroup per frame to place beside the front end instead of two
            m.proj_search_batch_device(self.p_lf, self.grid, p1, cap, cap, stream=stream, grid_counts=counts)
        # SearchLocalPoints skips the MapPoints that are in mCurrentFrame.mvpMapPoints (Tracking.cc:1163-1177): query
        # q's match stands only if the keypoint's owner is still q -- the rotation filter sets the entries it drops back
        # to NULL (ORBmatcher.cc:1456-1466; owner -2), and those MapPoints are searched again; the keypoints that now
        # hold a MapPoint are blocked for the second search.  One launch (orbx_proj_found_device) instead of eight
        # elementwise torch kernels on the stereo queue.
        m.proj_found_device(z["qi1"], z["own1"], z["fnd"], blocked=z["blk"], stream=stream)
        m.proj_project_device(PROJ_MAPPOINTS, z["pts"], counts, self.v_mp, self.scale, self.log_sf, out=z["q2"],
                              found=z["fnd"], stream=stream)
        m.proj_search_batch_device(self.p_mp, self.grid, p2, cap, cap, stream=stream)
        return z["qi1"], z["nm1"], z["qi2"], z["nm2"]


def found_in_frame(q_idx, owner):
    """Host form of FrameTracker's rule: MapPoint q is in the current frame after SearchByProjection(F, LastF) iff it
    was assigned a keypoint (q_idx[q] >= 0) and that keypoint still holds it (owner[q_idx[q]] == q; the rotation
    filter resets dropped entries, owner -2).  Returns the boolean mask over queries."""
    q_idx = np.asarray(q_idx)
    owner = np.asarray(owner)
    at = owner[np.maximum(q_idx, 0)] if len(owner) else np.full(q_idx.shape, -1)
    return (q_idx >= 0) & (at == np.arange(len(q_idx)))


def _view_bytes(v):
    """One VIEW_DTYPE record (array element or 1-element array) as a (1, 112) uint8 array."""
    from .orbx import VIEW_DTYPE
    return np.frombuffer(np.asarray(v, VIEW_DTYPE).reshape(1).tobytes(), np.uint8).reshape(1, 112)


class _nullcontext:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


def circle_trajectory(n: int, step: float = 0.8):
    """n keyframe poses 'step' metres apart on a closed circle, heading along it (a periodic synthetic trajectory, so a
    keyframe ring of n slots has no seam).  Returns (Rwc (n, 3, 3), Ow (n, 3)) float64."""
    R_ = n * step / (2 * np.pi)
    th = 2 * np.pi * np.arange(n) / n
    c, s = np.cos(th), np.sin(th)
    Rwc = np.zeros((n, 3, 3))
    Rwc[:, 0, 0], Rwc[:, 0, 2], Rwc[:, 1, 1], Rwc[:, 2, 0], Rwc[:, 2, 2] = c, s, 1, -s, c
    Ow = np.stack([R_ * (1 - c), np.zeros(n), R_ * s], 1)
    return Rwc, Ow


def make_view(Rwc, Ow, camera, bf, bounds, th, view_cos_limit=0.5, level_mode=0):
    """orbx_view (VIEW_DTYPE) of a camera with pose (Rwc, Ow): Rcw = Rwc^T, tcw = -Rcw Ow."""
    from .orbx import VIEW_DTYPE
    v = np.zeros(1, VIEW_DTYPE)[0]
    Rcw = np.asarray(Rwc, np.float64).T
    v["R"] = Rcw.reshape(9)
    v["t"] = -Rcw @ np.asarray(Ow, np.float64)
    v["Ow"] = Ow
    v["fx"], v["fy"], v["cx"], v["cy"] = camera
    v["bf"] = bf
    v["min_x"], v["max_x"], v["min_y"], v["max_y"] = bounds
    v["th"], v["view_cos_limit"], v["level_mode"] = th, view_cos_limit, level_mode
    return v


class LocalFuse:
    """LocalMapping::SearchInNeighbors' Fuse calls for a batch of new keyframes (src/LocalMapping.cc:460-520): each
    new keyframe's MapPoints fused into each of its neighbours (Fuse(pKFi, vpMapPointMatches), :486-496) and the
    neighbours' MapPoints fused into it (Fuse(mpCurrentKeyFrame, vpFuseCandidates), :499-520), the search part of
    ORBmatcher::Fuse (:830-951: the projection by orbx_proj_project FUSE, th = 3, then the window search with the
    stereo / mono reprojection tests and TH_LOW).  The replace / add-observation bookkeeping after each search is map
    work (out of scope).  A keyframe's MapPoints come from its stereo depths (orbx_stereo_mappoints) at
    creation and live in per-slot rings beside the keyframe store with its right coordinates and grid; the poses are
    the caller's (here: a periodic trajectory, one pose per slot).  Fuse's candidates are deduplicated in the reference
    (mnFuseCandidateForKF); here each neighbour's MapPoints are separate problems, as each is a separate view."""

    def __init__(self, matcher, store, slots: int, capacity: int, grid, camera, bf: float, scale, log_sf: float,
                 inv_sigma2, twc_slots, views_slots, device):
        import torch
        from .orbx import PROJ_FUSE, ProjParams
        self.m, self.store, self.slots, self.cap, self.grid = matcher, store, slots, capacity, grid
        self.camera = np.ascontiguousarray(camera, np.float32)
        self.scale = np.ascontiguousarray(scale, np.float32)
        self.log_sf = float(log_sf)
        dev = torch.device("cuda", device) if isinstance(device, int) else device
        self.dev = dev
        ncell = grid.cols * grid.rows
        self.pts = torch.zeros((slots, capacity, 48), dtype=torch.uint8, device=dev)
        self.ur = torch.full((slots, capacity), -1.0, dtype=torch.float32, device=dev)
        self.cnt = torch.zeros((slots,), dtype=torch.int32, device=dev)
        self.cs = torch.zeros((slots, ncell + 1), dtype=torch.int32, device=dev)
        self.ci = torch.zeros((slots, capacity), dtype=torch.int32, device=dev)
        self.twc = torch.from_numpy(np.ascontiguousarray(twc_slots, np.float32).reshape(slots, 12)).to(dev)
        self.views = torch.from_numpy(np.frombuffer(np.ascontiguousarray(views_slots).tobytes(), np.uint8)
                                      .reshape(slots, 112).copy()).to(dev)
        self.params = ProjParams.make(PROJ_FUSE, 50, 0.6, False, inv_sigma2)             # TH_LOW
        # plans per (new slots, neighbours) pattern, least recently used evicted: the bench's ring repeats a few
        # patterns, real covisibility would not (2 directions x P x cap x ~56 B of device buffers per plan)
        self.cache = OrderedDict()
        self.cache_max = 8

    def add_keyframes(self, slots: range, kps, desc, counts, uright, depth, rows, stream=None):
        """The new keyframes (rows of the extractor outputs) into the rings at 'slots' (a contiguous range)."""
        import torch
        from .orbx import QF_BLOCKS
        a, b = slots.start, slots.stop
        with torch.cuda.stream(stream) if stream is not None else _nullcontext():
            torch.index_select(counts, 0, rows, out=self.cnt[a:b])
            torch.index_select(uright, 0, rows, out=self.ur[a:b])
            kk = torch.index_select(kps, 0, rows)
            dk = torch.index_select(depth, 0, rows)
        if os.environ.get("ORBX_KF_PREP_SPLIT"):                  # A/B only: the MapPoints and the grid as two launches
            self.m.stereo_mappoints_device(kk, dk, self.cnt[a:b], self.twc[a:b], self.camera, self.scale, QF_BLOCKS,
                                           out=self.pts[a:b], stream=stream)
            self.m.grid_build_device(self.grid, kk, self.cnt[a:b], stream=stream, out=(self.cs[a:b], self.ci[a:b]))
        else:
            # the keyframes' MapPoints and grids in one launch of one workgroup per keyframe
            self.m.keyframe_prep_device(self.grid, kk, dk, self.cnt[a:b], self.twc[a:b], self.camera, self.scale, QF_BLOCKS,
                                        self.pts[a:b], self.cs[a:b], self.ci[a:b], stream=stream)

    def _plan(self, new_slots, neighbours):
        """Per (new keyframe j, neighbour k): the two directions' views, point sets and problem tables (cached per
        pattern: the ring's slot patterns repeat).  Both directions are one problem array of 2P problems (direction 0
        first), searched by one projection launch and one search launch."""
        import torch
        key = (tuple(new_slots), tuple(map(tuple, neighbours)))
        if key in self.cache:
            self.cache.move_to_end(key)
            return self.cache[key]
        while len(self.cache) >= self.cache_max:
            self.cache.popitem(last=False)     # its tensors were record_stream'ed on the streams that used them
        n, nn = neighbours.shape
        P, cap, st = n * nn, self.cap, self.store
        ns = np.repeat(np.asarray(new_slots, np.int64), nn)
        nb = np.asarray(neighbours, np.int64).reshape(-1)
        ok = np.concatenate([nb >= 0, nb >= 0])
        nbc = np.where(nb >= 0, nb, 0)
        tgt, src = np.concatenate([nbc, ns]), np.concatenate([ns, nbc])   # 0: current MPs into neighbour; 1: the reverse
        dev = self.dev
        q = torch.empty((2 * P, cap, 40), dtype=torch.uint8, device=dev)
        qi, qd = torch.empty((2 * P, cap), dtype=torch.int32, device=dev), torch.empty((2 * P, cap), dtype=torch.int32, device=dev)
        own, nm = torch.empty((2 * P, cap), dtype=torch.int32, device=dev), torch.empty((2 * P,), dtype=torch.int32, device=dev)
        i = np.arange(2 * P, dtype=np.int64)
        t = problem_table(2 * P, queries=q.data_ptr() + i * cap * 40, qdesc=st.desc + src * st.desc_stride,
                          nq=np.where(ok, cap, 0), kps=st.kps + tgt * st.kps_stride, desc=st.desc + tgt * st.desc_stride,
                          uright=self.ur.data_ptr() + tgt * cap * 4, n=cap,
                          cell_start=self.cs.data_ptr() + tgt * self.cs.shape[1] * 4,
                          cell_idx=self.ci.data_ptr() + tgt * cap * 4, q_idx=qi.data_ptr() + i * cap * 4,
                          q_dist=qd.data_ptr() + i * cap * 4, owner=own.data_ptr() + i * cap * 4,
                          nmatches=nm.data_ptr() + i * 4)
        views = self.views[torch.from_numpy(tgt).to(dev)].contiguous()
        vpts = torch.from_numpy(src.astype(np.int32)).to(dev)
        # every buffer the problem table points at stays referenced here (q_dist and owner too: a freed block would be
        # handed to another tensor while the searches still write it)
        out = dict(q=q, qi=qi, qd=qd, own=own, nm=nm, probs=torch.from_numpy(t.view(np.uint8)).to(dev), views=views,
                   vpts=vpts)
        self.cache[key] = out
        return out

    def run(self, new_slots, neighbours, stream=None):
        """new_slots (n,) and neighbours (n, nn) as host int arrays (-1 = none).  Returns ((q_idx, nmatches) of the
        current-into-neighbour searches, (q_idx, nmatches) of the neighbour-into-current ones), (n*nn, cap) / (n*nn,)."""
        from .orbx import PROJ_FUSE
        nb = np.asarray(neighbours)
        p = self._plan(np.asarray(new_slots), nb)
        P = nb.shape[0] * nb.shape[1]
        # one projection + one search launch over both directions (r5b: keyframe_fuse 0.73 -> 0.49 ms live)
        self.m.proj_project_device(PROJ_FUSE, self.pts, self.cnt, p["views"], self.scale, self.log_sf, out=p["q"],
                                   view_points=p["vpts"], stream=stream)
        self.m.proj_search_batch_device(self.params, self.grid, p["probs"], self.cap, self.cap, stream=stream)
        if stream is not None:
            # the kernels read / write these through raw pointers on 'stream': an evicted plan's memory must not be
            # handed out again before that stream's work is done
            for t in p.values():
                t.record_stream(stream)
        return [(p["qi"][:P], p["nm"][:P]), (p["qi"][P:], p["nm"][P:])]
