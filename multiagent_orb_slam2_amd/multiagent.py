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

from dataclasses import dataclass

import numpy as np

HEADER = 16        # int32 count, int32 agent, int32 frame, int32 reserved
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


def packet_bytes(capacity: int) -> int:
    return HEADER + capacity * (KP_BYTES + DESC_BYTES + 1)


def pack_keyframes(kps, desc, counts, valid, agent: int, frames, capacity: int):
    """Pack n keyframes into a (n, packet_bytes) uint8 tensor on the same device.

    kps: (n, capacity, 28) uint8, desc: (n, capacity, 32) uint8, counts: (n,) int32,
    valid: (n, capacity) uint8 (keypoint has a MapPoint), frames: (n,) frame ids."""
    import torch
    n = kps.shape[0]
    dev = kps.device
    out = torch.zeros((n, packet_bytes(capacity)), dtype=torch.uint8, device=dev)
    hdr = torch.stack([counts.to(torch.int32), torch.full_like(counts, agent, dtype=torch.int32),
                       torch.as_tensor(frames, dtype=torch.int32, device=dev), torch.zeros_like(counts, dtype=torch.int32)], 1)
    out[:, :HEADER] = hdr.contiguous().view(torch.uint8).view(n, HEADER)
    o = HEADER
    out[:, o:o + capacity * KP_BYTES] = kps.reshape(n, -1)
    o += capacity * KP_BYTES
    out[:, o:o + capacity * DESC_BYTES] = desc.reshape(n, -1)
    o += capacity * DESC_BYTES
    out[:, o:o + capacity] = valid.reshape(n, -1)
    return out


@dataclass
class KeyframeView:
    count: int
    agent: int
    frame: int
    kps: np.ndarray      # structured KP_DTYPE (count,)
    desc: np.ndarray     # (count, 32) uint8
    valid: np.ndarray    # (count,) uint8


def unpack_keyframes(packets, capacity: int) -> list[KeyframeView]:
    from .orbx import KP_DTYPE
    p = packets.cpu().numpy() if hasattr(packets, "cpu") else np.asarray(packets)
    out = []
    for row in p:
        cnt, agent, frame, _ = row[:HEADER].view(np.int32)
        o = HEADER
        kp = row[o:o + capacity * KP_BYTES].view(KP_DTYPE)[:cnt].copy()
        o += capacity * KP_BYTES
        d = row[o:o + capacity * DESC_BYTES].reshape(capacity, DESC_BYTES)[:cnt].copy()
        o += capacity * DESC_BYTES
        v = row[o:o + capacity][:cnt].copy()
        out.append(KeyframeView(int(cnt), int(agent), int(frame), kp, d, v))
    return out


class KeyframeExchange:
    """All-gather of keyframe packets: the MapFusion ingress (src/MapFusion.cc:83-88) as one collective.

    Works with the ``nccl`` (RCCL over xGMI) and ``gloo`` backends."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.bytes_moved = 0
        self.calls = 0

    def exchange(self, packets):
        """packets: (n, P) uint8 on this rank (same n and P on every rank) -> (world*n, P), rank-major."""
        import torch
        n, P = packets.shape
        out = torch.empty((self.world * n, P), dtype=torch.uint8, device=packets.device)
        if hasattr(self.dist, "all_gather_into_tensor") and packets.is_cuda:
            self.dist.all_gather_into_tensor(out, packets.contiguous(), group=self.group)
        else:
            parts = list(out.chunk(self.world, 0))
            self.dist.all_gather(parts, packets.contiguous(), group=self.group)
        self.bytes_moved += out.numel()
        self.calls += 1
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
