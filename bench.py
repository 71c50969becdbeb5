#!/usr/bin/env python3
"""bench.py — frames/s of the ORB stereo front-end (extract L + extract R + stereo L<->R Hamming match)
at KITTI size 1242x375, 8 levels, 2000 keypoints, on 1..N MI355X (one agent per GPU).

A "step" = one batch of --batch synthetic stereo frames per GPU through the hot path:
  ORBextractor on 2*batch images (src/ORBextractor.cc:1043-1105)  +  Frame::ComputeStereoMatches on
  batch pairs (descriptor band search, SAD sub-pixel refinement, median rejection; src/Frame.cc:466-639)
and the keyframe path: every 5th left frame becomes a keyframe (MapPoint-valid = stereo-matched, as
Tracking::CreateNewKeyFrame makes stereo MapPoints), its DBoW2 FeatureVector is computed on the GPU
(KeyFrame::ComputeBoW, synthetic k=10 L=6 vocabulary of ORBvoc's shape), the keyframe packets are
all-gathered over RCCL into every rank's MapFusion store (src/MapFusion.cc:83-88 replaced by
ncclAllGather; a local insert at N=1), each exchanged keyframe in turn queries the KeyFrameDatabase over
the store (DetectLoopCandidates, src/MapFusion.cc:133) and then joins it (:149 / :222) -- each rank answers
its own keyframes' queries -- and is matched with SearchByBoW against its first 16 candidates (other
agents' at N>1 -- MapFusion.cc:136-144, :275; the agent's own earlier ones at N=1 -- LoopClosing.cc:164,
:288), so every rank does the same work at every N.  Inputs are resident in HBM before the timed region;
weak scaling.  Rank r's frames are its contiguous chunk of one synthetic sequence, split as the reference's
multi-agent driver splits a sequence (Examples/MultiAgent/generic_split_seq.cc:543-589).

--config kitti (C2/C5: 1242x375, 2000 kpts, KITTI00-02.yaml) or euroc (C4: 752x480, 1200 kpts, EuRoC.yaml:88).

Prints ONE JSON line on rank 0 (driver contract).  Run: python bench.py [--gpus N --steps K --warmup W]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# Hardware queues per process: HIP's default (4 on the box).  r5a: 4 and 8 queues measured equal (73,954 / 74,196
# stereo frames/s in one call, profiles/r5a_hwq*.log); ORBX_HW_QUEUES overrides (read by the HIP runtime
# at init, before any GPU call).
if os.environ.get("ORBX_HW_QUEUES"):
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ["ORBX_HW_QUEUES"]

METRIC = "frames/sec ORB extract+match, KITTI 1242×375 @2000 kpts, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0                         # MI355X HBM3E peak (MI355X_MICROARCH.md)
VALU_PEAK_TOPS = 256 * 128 * 2.4e9 / 1e12     # 256 CU x 4 SIMD-32 x 2.4 GHz lane-ops (MI355X_MICROARCH.md)
NLEV, SCALE, INI, MINTH = 8, 1.2, 20, 7
KF_EVERY = 5
KF_CANDIDATES = 16
TRI_NEIGHBOURS = 10                           # CreateNewMapPoints' neighbours of a stereo keyframe (LocalMapping.cc:216)
STORE_STEPS = 3                               # keyframe store ring = 3 steps of every agent's keyframes
# Camera.bf and Camera.fx of the reference's stereo settings (baseline b = bf / fx, Frame.cc mb)
CONFIGS = {
    "kitti": dict(rows=375, cols=1242, nfeatures=2000, bf=386.1448, fx=718.856, seq_frames=4541,
                  source="Examples/Stereo/KITTI00-02.yaml (1242x375 synthetic, BASELINE C2/C5)"),
    "euroc": dict(rows=480, cols=752, nfeatures=1200, bf=47.90639384423901, fx=435.2046959714599, seq_frames=3682,
                  source="Examples/Stereo/EuRoC.yaml:18-19,25,88 (752x480, 1200 kpts, BASELINE C4)"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="kitti")
    ap.add_argument("--batch", type=int, default=256, help="stereo frames per GPU per step (512 images per extractor launch; "
                                                          "r6zv/r6zw: 128 / 192 / 256 / 384 / 512 frames -> 75.4k / 78.0k / 78.6k / 76.8k / 76.6k frames/s)")
    ap.add_argument("--desc-stream", type=int, default=int(os.environ.get("ORBX_BENCH_DESC_STREAM", "1")),
                    help="1: the extractor's descriptor stage on the stereo stream (orbx_extract_batch_device_split), "
                         "so step k+1's front end overlaps step k's descriptor stage; 2: on a stream of its own; 0: on "
                         "the launch stream")
    ap.add_argument("--sets", type=int, default=3,
                    help="output / pyramid sets in flight: step k's stereo and keyframe path read set k %% sets while later "
                         "steps' front ends write the others (2: the front end of step k+2 waits for keyframe path k)")
    ap.add_argument("--pyr-sets", type=int, default=0,
                    help="pyramid sets of the extractor ring (0 = --sets): step k's stereo SAD reads set k %% pyr-sets; "
                         "the front end of step k + pyr-sets waits for that stereo step")
    ap.add_argument("--inflight", type=int, default=1,
                    help="extractor contexts used in turn (step k on context k %% n, each on its own queue), so step k+1's "
                         "extraction can start while step k's tail runs")
    ap.add_argument("--cu-exclude", type=int, default=int(os.environ.get("ORBX_CU_EXCLUDE", "0")),
                    help="front-end and stereo streams leave this many CUs out of their CU mask (the keyframe stream keeps "
                         "every CU), so the keyframe path's small kernels are not starved; 0 = plain streams")
    ap.add_argument("--kf-cus", type=int, default=0,
                    help="diagnostics: the keyframe stream keeps only this many CUs in its CU mask (0 = every CU)")
    ap.add_argument("--distinct", type=int, default=0,
                    help="distinct synthetic stereo pairs per rank, tiled to the batch (0: the largest multiple of 5 <= the "
                         "batch -- 255 at 256 -- so every agent's keyframes show the same scenes, see main())")
    ap.add_argument("--input-sets", type=int, default=3,
                    help="resident input batches read in turn (set k = the batch rolled by 3k rows / 11k columns): 3 x 119 MB "
                         "exceeds the 256 MB Infinity Cache, so every step's level-0 reads come from HBM (1 = one batch "
                         "re-read every step)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget (0 = skip)")
    ap.add_argument("--host-api-frames", type=int, default=200, help="stereo frames through the host C-ABI (0 = skip)")
    ap.add_argument("--alone-reps", type=int, default=5,
                    help="calls of the roofline_alone block (the extraction alone, one stream); 0 skips it")
    ap.add_argument("--host-fed-steps", type=int, default=10,
                    help="steps of the host-fed block: the batch's images copied H2D from pinned host memory every step on a "
                         "copy stream, overlapped with the previous step (0 = skip)")
    ap.add_argument("--no-timing", action="store_true", help="skip per-stage event timing")
    ap.add_argument("--no-c3", dest="c3", action="store_false", help="skip the C3 2000x2000 all-pairs block")
    ap.add_argument("--no-tri", dest="tri", action="store_false",
                    help="leave CreateNewMapPoints' matching (SearchForTriangulation vs 10 neighbours + distinctive "
                         "descriptors) out of the keyframe path")
    ap.add_argument("--no-tracking", dest="tracking", action="store_false",
                    help="leave the tracking matches (SearchByProjection motion model + local map) out of the step")
    ap.add_argument("--track-stream", choices=["stereo", "kf", "own"],
                    default=os.environ.get("ORBX_BENCH_TRACK_STREAM", "stereo"),
                    help="queue of the tracking matches: after the stereo step on the stereo queue, at the head of "
                         "the keyframe queue, or on a queue of its own after the stereo step (diagnostics; with "
                         "ORBX_HW_QUEUES > 4 so it gets a hardware queue)")
    ap.add_argument("--no-fuse", dest="fuse", action="store_false",
                    help="leave SearchInNeighbors' Fuse (both ways with 10 neighbours) out of the keyframe path")
    ap.add_argument("--no-cd", dest="cd", action="store_false", help="skip the CovisibilityDiscovery-shaped block")
    ap.add_argument("--diag-skip", default="", help="diagnostics only (not the metric): comma list of stereo,keyframes "
                                                     "to leave out of the step")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N>1 process group: nccl (RCCL over xGMI, the measured path) or gloo (rehearsal: several ranks "
                         "sharing one GPU, packets staged through host memory)")
    ap.add_argument("--exchange", default="torch", choices=["torch", "native"],
                    help="N>1 keyframe all-gather in the step: torch (torch.distributed all_gather_into_tensor; RCCL under "
                         "the nccl backend) or native (liborbx's orbx_exchange: its own RCCL communicator, the path a C++ "
                         "MultiAgentServer without torch takes; nccl backend only)")
    ap.add_argument("--exchange-copy", action="store_true",
                    help="A/B only: all-gather into a separate buffer that the MapFusion commit copies into the ring "
                         "(round 5's form) instead of straight into the ring slots")
    ap.add_argument("--emulate-agents", type=int, default=0,
                    help="diagnostics, N=1 only: the keyframe path as rank 0 of this many agents -- this rank's packets stand "
                         "in for every agent's (copied rank-major into the ring as if all-gathered), so the KeyFrameDatabase "
                         "and ring carry an N-agent load on one GPU (not a scaling figure: no collective, one front end)")
    ap.add_argument("--xgmi-mb", default="0.17,2,16,64",
                    help="N>1: per-rank payloads (MB) of the all-gather bandwidth sweep after the timed steps (empty = skip)")
    ap.add_argument("--sync-each", action="store_true",
                    help="diagnostics: synchronise after every timed step (host_enqueue_* = pure host cost, no back-pressure)")
    return ap.parse_args()


def rank_env(base: dict, rank: int, world: int, port: int) -> dict:
    """The environment torch.distributed.run gives rank `rank` of a one-node job of `world` ranks (one per GPU,
    LOCAL_RANK = RANK), rendezvous on 127.0.0.1 (the container hostname may not resolve)."""
    env = dict(base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", ROLE_RANK=str(rank), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
               ORBX_LAUNCHER="bench.py --gpus")
    return env


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(world: int, cmd: list, poll_s: float = 0.2, grace_s: float = 20.0) -> int:
    """`bench.py --gpus N` without a launcher: start N fresh child processes (rank r on GPU r) before this process
    makes any GPU call, rank 0's stdout passed through (its one JSON line), the other ranks' stdout sent to stderr so
    that stdout holds that line only.  When a rank fails, the others are stopped (SIGTERM, then SIGKILL after
    grace_s: a rank blocked in a collective whose peer died never returns).  Returns the first non-zero exit status
    (or 0).  The children are started as subprocesses, never exec'd into this process."""
    import signal
    import subprocess
    port = free_port()
    procs = []
    for r in range(world):
        procs.append(subprocess.Popen(cmd, env=rank_env(os.environ, r, world, port),
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno()))

    def forward(pipe):
        # rank 0's JSON line to stdout; anything else it prints there (gloo's "[Gloo] Rank 0 is connected ..." banner,
        # library chatter) to stderr
        for raw in iter(pipe.readline, b""):
            line = raw.decode(errors="replace")
            dst = sys.stdout if line.lstrip().startswith("{") else sys.stderr
            dst.write(line)
            dst.flush()
    fwd = threading.Thread(target=forward, args=(procs[0].stdout,), daemon=True)
    fwd.start()

    def stop_all(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                try:
                    p.send_signal(sig)
                except OSError:
                    pass

    prev = {s: signal.getsignal(s) for s in (signal.SIGTERM, signal.SIGINT)}

    def on_signal(signum, _frame):
        stop_all(signal.SIGTERM)
        raise SystemExit(128 + signum)
    for s in prev:
        signal.signal(s, on_signal)
    rc, failed_at = 0, None
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad and rc == 0:
                rc, failed_at = bad[0], time.monotonic()
                stop_all(signal.SIGTERM)
            if all(c is not None for c in codes):
                break
            if failed_at is not None and time.monotonic() - failed_at > grace_s:
                stop_all(signal.SIGKILL)
            time.sleep(poll_s)
    finally:
        for s, h in prev.items():
            signal.signal(s, h)
    fwd.join(timeout=10.0)
    return rc


def compulsory_bytes(cfg):
    """SURVEY §8(d) algorithmic bytes: one extraction reads the image once and writes nfeatures x (28 B keypoint +
    32 B descriptor); one stereo descriptor match reads both descriptor sets and writes (index, distance)."""
    img = cfg["rows"] * cfg["cols"]
    n = cfg["nfeatures"]
    return {"extraction": img + n * (28 + 32), "stereo_match": 2 * n * 32 + n * 8}


class Geometry:
    """The synthetic camera motion the matching stages need (the reference's poses come from tracking and optimisation,
    which are out of scope): KITTI intrinsics with the principal point at the image centre, no distortion (bounds =
    the image); keyframes of an agent on a closed circle (multiagent.circle_trajectory: 0.8 m apart, heading along it),
    one pose per keyframe-ring position, so the ring has no seam; for the tracking stage, frame i's last frame at the
    origin and the current frame moved by the motion model's residual (6 cm forward, 1 cm sideways, 0.2 deg of yaw)."""

    def __init__(self, cfg, ring_kf: int):
        from multiagent_orb_slam2_amd import multiagent as MA
        self.cfg = cfg
        self.fx = cfg["fx"]
        self.camera = np.array([cfg["fx"], cfg["fx"], cfg["cols"] / 2, cfg["rows"] / 2], np.float32)
        self.bf = cfg["bf"]
        self.bounds = (0.0, float(cfg["cols"]), 0.0, float(cfg["rows"]))
        self.ring_kf = max(ring_kf, TRI_NEIGHBOURS + 2)
        self.Rwc, self.Ow = MA.circle_trajectory(self.ring_kf)
        a = 0.0035
        self.R_cur = np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]])
        self.O_cur = np.array([0.01, 0.0, 0.06])
        tlc = self.O_cur                                    # the current camera centre in the last frame (:1344-1352)
        mb = self.bf / self.fx
        self.level_mode = 1 if tlc[2] > mb else (-1 if -tlc[2] > mb else 0)

    def K(self):
        c = self.camera
        return np.array([[c[0], 0, c[2]], [0, c[1], c[3]], [0, 0, 1]], np.float64)

    def tracking_views(self):
        from multiagent_orb_slam2_amd import multiagent as MA
        lf = MA.make_view(self.R_cur, self.O_cur, self.camera, self.bf, self.bounds, 7.0, level_mode=self.level_mode)
        mp = MA.make_view(self.R_cur, self.O_cur, self.camera, self.bf, self.bounds, 1.0, view_cos_limit=0.5)
        twc_last = np.concatenate([np.eye(3).reshape(9), np.zeros(3)]).astype(np.float32)
        return twc_last, lf, mp

    def slot_tables(self, slots: int, world: int, n_kf: int):
        """Per keyframe-store slot: Twc (12 floats) and the Fuse view (th = 3) of the keyframe held there; slot s holds
        keyframe c(s) of its agent (slots are rank-major per step: multiagent KeyframeFusion)."""
        from multiagent_orb_slam2_amd import multiagent as MA
        from multiagent_orb_slam2_amd.orbx import VIEW_DTYPE
        per = world * n_kf
        twc = np.zeros((slots, 12), np.float32)
        views = np.zeros(slots, VIEW_DTYPE)
        for s in range(slots):
            c = ((s // per) * n_kf + (s % per) % n_kf) % self.ring_kf
            twc[s, :9], twc[s, 9:] = self.Rwc[c].reshape(9), self.Ow[c]
            views[s] = MA.make_view(self.Rwc[c], self.Ow[c], self.camera, self.bf, self.bounds, 3.0)
        return twc, views

    def tri_rows(self):
        """F12 and epipole rows for a keyframe and its d-th previous keyframe on the circle, d = 1..TRI_NEIGHBOURS (the
        same for every keyframe: the circle's relative poses repeat; every baseline (>= 0.8 m) passes
        LocalMapping.cc:252-256).  (TRI_NEIGHBOURS, 12) float32 tensor on the CPU."""
        import torch
        from multiagent_orb_slam2_amd import multiagent as MA
        n = TRI_NEIGHBOURS + 1
        Rcw = torch.tensor(np.transpose(self.Rwc[:n], (0, 2, 1)))
        t = -(Rcw @ torch.tensor(self.Ow[:n])[:, :, None])[:, :, 0]
        pairs = torch.tensor([[n - 1, n - 1 - d] for d in range(1, n)])
        return MA.triangulation_geometry(torch.tensor(self.K()), Rcw, t, pairs)


def cpu_threads():
    """Every core this process may use, as SURVEY §8(d) asks (T = nproc): the CPUs of sched_getaffinity, bounded by the
    cgroup CPU quota when there is one (the GPU box shows 256 CPUs but grants 16: 256 threads there measured 238
    frames/s against 285 on 16).  ORBX_CPU_THREADS overrides (diagnostics)."""
    n = os.environ.get("ORBX_CPU_THREADS")
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    q = cpu_quota()
    if q:
        avail = min(avail, max(1, int(np.ceil(q))))
    return max(1, int(n)) if n and n.isdigit() else avail


def cpu_quota():
    """The cgroup CPU quota in CPUs (cgroup v2 cpu.max), None when unlimited or unknown."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


class CpuAgent:
    """The per-frame work on host cores with the oracle (oracle/*.cpp -O3, same FP pins): extract L and R,
    ComputeStereoMatches (band search + SAD refinement), the tracking matches (the last frame's stereo MapPoints
    projected and searched, SearchByProjection(F, LastF, 7), then SearchLocalPoints: isInFrustum +
    SearchByProjection(F, vpMapPoints, 1)), and every KF_EVERY-th frame a keyframe: BoW transform, CreateNewMapPoints'
    SearchForTriangulation vs TRI_NEIGHBOURS neighbours + the new MapPoints' descriptors, SearchInNeighbors' Fuse both
    ways with each neighbour, DetectLoopCandidates over a keyframe ring of the GPU store's size, SearchByBoW against the
    first KF_CANDIDATES candidates, then the keyframe joins the database (MapFusion's query-then-add) -- the GPU step's
    work.  One per thread, as one extractor per agent (Tracking.cc:119-125)."""

    def __init__(self, O, cfg, tables, voc, n_kf_step, geo, tri=True, track=True, fuse=True):
        from multiagent_orb_slam2_amd.orbx import PROJ_FUSE, PROJ_LASTFRAME, PROJ_MAPPOINTS, ProjParams, frame_grid
        self.O, self.cfg, self.tables, self.geo = O, cfg, tables, geo
        self.tri = geo.tri_rows().numpy() if tri else None
        self.track, self.fuse = track, fuse
        self.vocab = O.Vocabulary(voc)
        self.ring = STORE_STEPS * max(1, n_kf_step)
        self.db = O.Kfdb(int(np.sum(voc["is_leaf"])), self.ring)
        self.kfs = [None] * self.ring
        self.kps = [None] * self.ring
        self.kfx = [None] * self.ring                  # (kps, desc, uright, MapPoints) per slot, for Fuse
        self.n_kf = 0
        self.n = 0
        self.grid = frame_grid(0, 0, cfg["cols"], cfg["rows"])
        self.twc_last, self.v_lf, self.v_mp = geo.tracking_views()
        self.twc_slot, self.v_slot = geo.slot_tables(self.ring, 1, max(1, n_kf_step))
        self.log_sf = float(np.float32(np.log(SCALE)))
        isg = tables["inv_sigma2"]
        self.p_lf = ProjParams.make(PROJ_LASTFRAME, 100, 0.9, True, isg)
        self.p_mp = ProjParams.make(PROJ_MAPPOINTS, 100, 0.8, False, isg)
        self.p_fu = ProjParams.make(PROJ_FUSE, 50, 0.6, False, isg)
        self.modes = (PROJ_LASTFRAME, PROJ_MAPPOINTS, PROJ_FUSE)

    def frame(self, left, right):
        O, c = self.O, self.cfg
        a = O.extract(left, nfeatures=c["nfeatures"], want_pyramid=True)
        b = O.extract(right, nfeatures=c["nfeatures"], want_pyramid=True)
        ur, depth = O.compute_stereo_matches(a, b, self.tables["scale"], self.tables["inv_scale"], c["rows"], c["bf"],
                                             c["bf"] / c["fx"])
        if self.track:
            self.tracking(a, ur, depth)
        if self.n % KF_EVERY == 0:
            bow = self.vocab.transform(a["desc"], 4)
            kf = (a["desc"], a["kps"]["angle"], (depth > 0).astype(np.uint8),
                  (bow["fv_nodes"], bow["fv_offsets"], bow["fv_indices"]))
            slot = self.n_kf % self.ring
            if self.tri is not None:
                self.new_mappoints(a, kf)
            if self.fuse:
                self.local_fuse(slot, a, ur, depth)
            self.db.erase([slot])
            self.db.set_bow(slot, bow["bow_words"], bow["bow_values"])
            for cand in self.db.detect(0, slot, self.n_kf + 1, 0.0)[:KF_CANDIDATES]:
                O.search_by_bow_kfkf(*kf, *self.kfs[cand], 0.75, True)
            self.db.add([slot])
            self.kfs[slot] = kf
            self.kps[slot] = a["kps"]
            self.n_kf += 1
        self.n += 1

    def tracking(self, a, ur, depth):
        """TrackWithMotionModel's search and SearchLocalPoints, as multiagent.FrameTracker."""
        from multiagent_orb_slam2_amd import multiagent as MA
        from multiagent_orb_slam2_amd.orbx import PROJ_QUERY_DTYPE, QF_BLOCKS, QF_SKIP
        O, sc = self.O, self.tables["scale"]
        lf, mp, _ = self.modes
        pts = O.stereo_mappoints(a["kps"], depth, self.twc_last, self.geo.camera, sc, QF_BLOCKS)
        last = pts.copy()
        last["flags"][1::2] |= QF_SKIP                      # the last frame holds the even keypoints' MapPoints
        q1 = O.project(lf, last, self.v_lf, sc, self.log_sf).view(PROJ_QUERY_DTYPE).reshape(-1)
        _, qi1, _, own1 = O.proj_search(self.p_lf, self.grid, q1, a["desc"], a["kps"], a["desc"], uright=ur)
        pts["flags"][MA.found_in_frame(qi1, own1)] |= QF_SKIP      # in mCurrentFrame.mvpMapPoints (Tracking.cc:1158-1174)
        q2 = O.project(mp, pts, self.v_mp, sc, self.log_sf).view(PROJ_QUERY_DTYPE).reshape(-1)
        O.proj_search(self.p_mp, self.grid, q2, a["desc"], a["kps"], a["desc"], uright=ur,
                      blocked=(own1 >= 0).astype(np.uint8))

    def local_fuse(self, slot, a, ur, depth):
        """SearchInNeighbors' Fuse both ways with each of the previous TRI_NEIGHBOURS keyframes, as multiagent.LocalFuse."""
        from multiagent_orb_slam2_amd.orbx import PROJ_QUERY_DTYPE, QF_BLOCKS
        O, sc, fu = self.O, self.tables["scale"], self.modes[2]
        pts = O.stereo_mappoints(a["kps"], depth, self.twc_slot[slot], self.geo.camera, sc, QF_BLOCKS)
        self.kfx[slot] = (a["kps"], a["desc"], ur, pts)
        for d in range(1, TRI_NEIGHBOURS + 1):
            if self.n_kf - d < 0:
                break
            s2 = (self.n_kf - d) % self.ring
            k2, d2, ur2, p2 = self.kfx[s2]
            q = O.project(fu, pts, self.v_slot[s2], sc, self.log_sf).view(PROJ_QUERY_DTYPE).reshape(-1)
            O.proj_search(self.p_fu, self.grid, q, a["desc"], k2, d2, uright=ur2)
            q = O.project(fu, p2, self.v_slot[slot], sc, self.log_sf).view(PROJ_QUERY_DTYPE).reshape(-1)
            O.proj_search(self.p_fu, self.grid, q, d2, a["kps"], a["desc"], uright=ur)

    def new_mappoints(self, a, kf):
        """SearchForTriangulation against the previous TRI_NEIGHBOURS keyframes with ORBmatcher(0.6, false), then the
        distinctive descriptor of every new MapPoint (a keypoint with its first matching neighbour: two observations,
        LocalMapping.cc:440-448), as the GPU stage."""
        O, n = self.O, len(a["desc"])
        d1, mp1, fv1 = kf[0], kf[2], kf[3]
        ur = np.full(n, -1, np.float32)
        rows, m12s = [], []
        for d in range(1, TRI_NEIGHBOURS + 1):
            if self.n_kf - d < 0:
                break
            s2 = (self.n_kf - d) % self.ring
            d2, _, mp2, fv2 = self.kfs[s2]
            g = self.tri[d - 1]
            _, m12 = O.search_for_triangulation(d1, a["kps"], mp1, ur, fv1, d2, self.kps[s2], mp2,
                                                np.full(len(d2), -1, np.float32), fv2, g[:9].reshape(3, 3),
                                                self.tables["sigma2"], self.tables["scale"], float(g[9]), float(g[10]),
                                                False, False)
            rows.append(d2)
            m12s.append(m12)
        if not m12s:
            return
        hit = np.stack([m >= 0 for m in m12s], 1)                              # (n, k)
        has = hit.any(1)
        first = np.argmax(hit, 1)
        nb = np.stack([r[np.maximum(m, 0)] for r, m in zip(rows, m12s)], 1)      # (n, k, 32)
        parts = np.stack([nb[np.arange(n), first], d1], 1)[has]                 # (MapPoints, 2, 32)
        off = np.arange(0, 2 * len(parts) + 1, 2, dtype=np.int32)
        O.distinctive_descriptors_flat(parts.reshape(-1, 32), off)


def cpu_baseline(lefts, rights, cfg, voc, n_kf_step, seconds, geo, tri=True, track=True, fuse=True):
    """1-thread latency per stereo frame (median / p95) and T-thread throughput with one agent per thread on
    independent frames -- the reference drivers' timing pattern (generic_split_seq.cc:277-314, :369-379: per-frame
    steady_clock around TrackStereo, median and mean reported)."""
    from oracle import oracle as O
    tables = O.tables(cfg["nfeatures"])
    nd = len(lefts)
    mk = lambda: CpuAgent(O, cfg, tables, voc, n_kf_step, geo, tri=tri, track=track, fuse=fuse)  # noqa: E731
    # (i) latency, one thread
    ag = mk()
    lat = []
    t_end = time.perf_counter() + 0.4 * seconds
    while True:
        t0 = time.perf_counter()
        ag.frame(lefts[ag.n % nd], rights[ag.n % nd])
        lat.append(time.perf_counter() - t0)
        if time.perf_counter() >= t_end and ag.n >= 2 * KF_EVERY:
            break
    lat_ms = np.array(lat[1:] if len(lat) > 1 else lat) * 1e3
    # (ii) throughput, T threads (ctypes releases the GIL inside the oracle's C++)
    T = cpu_threads()
    agents = [mk() for _ in range(T)]
    stop = threading.Event()

    def run(i):
        a = agents[i]
        while not stop.is_set():
            k = (a.n * T + i) % nd
            a.frame(lefts[k], rights[k])

    th = [threading.Thread(target=run, args=(i,)) for i in range(T)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    time.sleep(0.6 * seconds)
    stop.set()
    for t in th:
        t.join()
    el = time.perf_counter() - t0
    done = sum(a.n for a in agents)
    work = "2 extractions + ComputeStereoMatches" + (" + the tracking matches (motion model + local map)" if track else "")
    kfw = "BoW" + (f" + CreateNewMapPoints matching vs {TRI_NEIGHBOURS} neighbours" if tri else "") + \
          (" + Fuse both ways with each neighbour" if fuse else "") + \
          f" + DetectLoopCandidates + SearchByBoW vs the first {KF_CANDIDATES} candidates"
    return {"value": round(done / el, 3), "unit": "frames/s", "cores": T, "kind": "port",
            "cpu_model": cpu_model(), "affinity_cpus": len(os.sched_getaffinity(0)), "cgroup_cpu_quota": cpu_quota(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "latency_ms_1thread": {"median": round(float(np.median(lat_ms)), 2),
                                   "p95": round(float(np.percentile(lat_ms, 95)), 2), "frames": len(lat_ms)},
            "throughput_1thread_fps": round(1e3 / float(np.mean(lat_ms)), 3),
            "sample": f"{done} stereo frames on {T} threads in {el:.1f} s (+ {len(lat)} on 1 thread for latency) of the "
                      f"same synthetic inputs and the same per-frame work ({work}; every {KF_EVERY}th frame {kfw}), "
                      f"oracle/*.cpp -O3 -ffp-contract=off, one agent per thread"}


def host_api_rate(pkg, cfg, lefts, rights, n_frames, device):
    """The per-call drop-in path: orbx_extract on host images (left, right) + orbx_compute_stereo_matches, host
    keypoints / descriptors / depths out -- what an unchanged Frame constructor pays per stereo frame (PCIe
    included, one frame at a time, as the reference calls it).  The caller passes 8 distinct stereo pairs, as the native
    driver (scripts/micro/host_api_bench.cpp) cycles through: with the bench's 255 pairs (119 MB of images) every
    image is cold in the CPU caches and its copy into the pinned staging costs ~0.1 ms more per frame (r5x)."""
    ex_l = pkg.ORBextractor(cfg["nfeatures"], SCALE, NLEV, INI, MINTH, device=device)
    ex_r = pkg.ORBextractor(cfg["nfeatures"], SCALE, NLEV, INI, MINTH, device=device)
    m = pkg.ORBmatcher(0.75, True, device=device)
    b = cfg["bf"] / cfg["fx"]
    from concurrent.futures import ThreadPoolExecutor
    pool = ThreadPoolExecutor(1)                     # the right extraction on its own thread, as Frame.cc:78-81
    # 10 untimed frames: among the first ~10 calls one takes 7-20 ms (one-time runtime set-up on the extractor's
    # thread, r4hac); their maximum is reported as warmup_ms_max
    n_warm = 10

    def two_threads(i):
        fr = pool.submit(ex_r, rights[i % len(rights)])
        kl, dl = ex_l(lefts[i % len(lefts)])       # ctypes releases the GIL: both extractions run natively at once
        kr, dr = fr.result()
        m.ComputeStereoMatches(ex_l, ex_r, kl, dl, kr, dr, cfg["bf"], b)

    def pair(i):
        (kl, dl), (kr, dr) = pkg.extract_pair(ex_l, ex_r, lefts[i % len(lefts)], rights[i % len(rights)])
        m.ComputeStereoMatches(ex_l, ex_r, kl, dl, kr, dr, cfg["bf"], b)

    def run(fn):
        lat, warm = [], []
        for i in range(n_frames + n_warm):
            t0 = time.perf_counter()
            fn(i)
            (lat if i >= n_warm else warm).append(time.perf_counter() - t0)
        lat_ms = np.array(lat) * 1e3
        return {"frames_per_s": round(1e3 / float(np.mean(lat_ms)), 1),
                "latency_ms_median": round(float(np.median(lat_ms)), 3),
                "latency_ms_p95": round(float(np.percentile(lat_ms, 95)), 3),
                "latency_ms_max": round(float(np.max(lat_ms)), 3), "frames": len(lat), "warmup_frames": n_warm,
                "warmup_ms_max": round(1e3 * max(warm), 3)}
    out = run(pair)
    out["path"] = ("Python ctypes: orbx_extract_pair (the left and right extractions of a stereo Frame, Frame.cc:78-81, "
                   "enqueued together from one thread) + orbx_compute_stereo_matches, host buffers, one frame per call")
    out["two_threads"] = dict(run(two_threads), path="Python ctypes: orbx_extract(L) and orbx_extract(R) on two threads "
                                                     "(as Frame.cc:78-81) + orbx_compute_stereo_matches")

    def frame(i):
        m.StereoFrame(ex_l, ex_r, lefts[i % len(lefts)], rights[i % len(rights)], cfg["bf"], b)
    out["stereo_frame"] = dict(run(frame), path="Python ctypes: orbx_stereo_frame (both extractions + ComputeStereoMatches "
                                                "in one call, the stereo search on the extractions' device outputs)")
    pool.shutdown()
    # the same per-call path from a C++ caller (the reference's own language): scripts/micro/host_api_bench.cpp, built
    # by build() into build/host_api_bench, run as a child process on the same GPU
    exe = os.path.join(ROOT, "build", "host_api_bench")
    lib = os.path.join(ROOT, "multiagent_orb_slam2_amd", "liborbx.so")
    if os.path.exists(exe):
        import subprocess
        try:
            r = subprocess.run([exe, lib, str(max(n_frames, 200)), str(cfg["rows"]), str(cfg["cols"]), str(cfg["nfeatures"])],
                               capture_output=True, text=True, timeout=120)
            if r.returncode == 0:
                out["native"] = json.loads(r.stdout.strip().splitlines()[-1])
                out["native"]["path"] = "C++ std::threads + dlopen'ed liborbx (scripts/micro/host_api_bench.cpp)"
            else:
                out["native_error"] = (r.stdout + r.stderr)[-500:]
        except (OSError, subprocess.TimeoutExpired, ValueError) as e:
            out["native_error"] = str(e)[:300]
    return out


def host_fed_block(step, last_handoff, host, stream, B, steps, dev):
    """The same step with its 2B input images arriving from host memory every step, as Frame's constructor receives
    host images (Frame.cc:61-117): a pinned host batch (a camera ring would fill it) is copied H2D on a copy stream into
    a ring of 3 device batches; step k's extraction waits for its copy, and the copy of step k+1 overlaps step k.  A
    slot is rewritten only after the stereo step that last read it (level 0 of the pyramid is the input image itself)."""
    import torch
    pinned = torch.from_numpy(host).pin_memory()
    nbytes = pinned.numel()
    ring = [torch.empty_like(pinned, device=dev) for _ in range(3)]
    consumed = [None] * 3
    cs = torch.cuda.Stream(dev)
    # PCIe H2D alone, for the ceiling
    for _ in range(2):
        with torch.cuda.stream(cs):
            ring[0].copy_(pinned, non_blocking=True)
    cs.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(cs)
    for i in range(5):
        with torch.cuda.stream(cs):
            ring[i % 3].copy_(pinned, non_blocking=True)
    e1.record(cs)
    e1.synchronize()
    h2d_gbs = 5 * nbytes / (e0.elapsed_time(e1) * 1e-3) / 1e9

    def fed_step(i):
        k = i % 3
        if consumed[k] is not None:
            cs.wait_event(consumed[k])
        with torch.cuda.stream(cs):
            ring[k].copy_(pinned, non_blocking=True)
        ready = torch.cuda.Event()
        ready.record(cs)
        stream.wait_event(ready)
        step(src=ring[k])
        consumed[k] = last_handoff[0]

    for i in range(3):
        fed_step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        fed_step(i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    fps = B * steps / el
    return {"frames_per_s": round(fps, 1), "ms_per_step": round(1e3 * el / steps, 3), "steps": steps,
            "input_bytes_per_step": nbytes, "h2d_GBps_needed": round(nbytes * steps / el / 1e9, 2),
            "h2d_GBps_alone": round(h2d_gbs, 2),
            "pcie_bound_frames_per_s": round(B * h2d_gbs * 1e9 / nbytes, 1),
            "path": "pinned host batch -> H2D on a copy stream into a 3-slot device ring, overlapped with the previous "
                    "step; the same step as `value` otherwise (stereo + keyframe path)"}


def cd_block(pkg, MA, kps, desc, cnt, vocab, B, reps=3):
    """A CovisibilityDiscovery-shaped batch (MapFusion.cc:774-885): the last step's B left keyframes are the matched
    map (in its KeyFrameDatabase), its B right keyframes the absorbed map; every absorbed keyframe computes minScore
    over its 10 covisible keyframes (the 5 before and after it), queries DetectCovisibilityCandidates ignoring the
    absorbed map, and runs SearchByBoW against every candidate (15-match gate).  Wall time per pass with the
    candidate-count readback it needs (the Fuse step after it is out of scope).  The reference's published CD stage
    (which also fuses MapPoints and stops / releases LocalMapping) is printed beside it as context only."""
    import torch
    dev = kps.device
    cap = kps.shape[1]
    fv = vocab.transform_batch_device(desc, cnt, 4)
    valid = (torch.arange(cap, device=dev)[None, :] < cnt[:, None]).to(torch.uint8)
    valid[:, 2::3] = 0                                         # ~2/3 of keypoints carry a MapPoint
    store = pkg.KfStore.from_fields(cap, desc=(desc, cap * 32), kps=(kps, cap * 28), valid=(valid, cap),
                                    fv_nodes=(fv["fv_nodes"], cap * 4), fv_offsets=(fv["fv_offsets"], (cap + 1) * 4),
                                    fv_indices=(fv["fv_indices"], cap * 4), n_fv=(fv["n_fv"], 4))
    db = pkg.KeyFrameDatabase(vocab.info()["n_words"], 2 * B, max_words=min(cap, 4096), device=dev.index)
    db.set_bow_device(torch.arange(2 * B, dtype=torch.int32, device=dev), fv["bow_words"], fv["bow_values"], fv["n_words"])
    db.add(list(range(B)))
    queries = list(range(B, 2 * B))
    covis = [[c for c in range(q - 5, q + 6) if c != q and B <= c < 2 * B] for q in queries]
    cd = MA.CovisibilityDiscovery(pkg.ORBmatcher(0.75, True, device=dev.index), db, store,
                                  max_fv_nodes=min(cap, 10 ** 2 + 1))
    times, last = [], None
    for r in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = cd.run(queries, [10_000_000 + r * B + i for i in range(B)], covis, queries)
        torch.cuda.synchronize()
        if r:
            times.append(time.perf_counter() - t0)
        last = res
    pr, m12, nm, passed, n_cand = last
    ms = 1e3 * float(np.median(times))
    real = int((pr[:, 1] >= 0).sum().item())
    return {"absorbed_keyframes": B, "matched_map_keyframes": B, "ms_per_pass": round(ms, 3),
            "ms_per_keyframe": round(ms / B, 4), "passes": [round(1e3 * t, 3) for t in times],
            "candidates_per_keyframe": round(float(np.mean(n_cand)), 2), "searchbybow_pairs": real,
            "pairs_passing_15": int(passed.sum().item()),
            "reference_cd_stage_ms (context: includes Fuse + LocalMapping stop/release, hardware unstated)":
                {"KITTI 00 (mkf 136.2)": 1850.51, "KITTI 02": 15297.20, "EuRoC MH01": 7362.53},
            "path": "multiagent.CovisibilityDiscovery: orbx_kfdb_score_device (minScore), orbx_kfdb_detect_device COVIS, "
                    "one candidate-count readback, orbx_kfdb_candidate_pairs_device, orbx_search_by_bow_kfkf_pairs_device"}


def alone_block(pkg, cfg, imgs, dev, reps=5):
    """The extraction of one step's batch with every stage on one stream (ORBX_PIPELINE=0) and nothing else on the GPU:
    per-stage spans of HIP events around each kernel, so each span is that kernel's own duration (plus launch gaps).
    `roofline_alone` divides the dominant kernel's algorithmic bytes by its span here; the contract's
    `roofline` uses the spans of the overlapped step, where every kernel shares the CUs with four other queues."""
    import torch
    saved = os.environ.get("ORBX_PIPELINE")
    os.environ["ORBX_PIPELINE"] = "0"                  # read at extractor creation
    try:
        ex = pkg.ORBextractor(cfg["nfeatures"], SCALE, NLEV, INI, MINTH, device=dev.index)
    finally:
        if saved is None:
            os.environ.pop("ORBX_PIPELINE")
        else:
            os.environ["ORBX_PIPELINE"] = saved
    s = torch.cuda.current_stream(dev)
    outs = ex.extract_batch_device(imgs, stream=s)
    for _ in range(2):
        ex.extract_batch_device(imgs, *outs, stream=s)
    torch.cuda.synchronize()
    ex.enable_timing(True)
    for _ in range(reps):
        ex.extract_batch_device(imgs, *outs, stream=s)
    torch.cuda.synchronize()
    st, calls = ex.stage_times()
    ex.close()
    per = {k: round(v / max(calls, 1), 4) for k, v in st.items()}
    return per, calls


def c3_bench(pkg, dev, n_problems=64, reps=30):
    """BASELINE config C3: brute-force 256-bit Hamming match of 2000 x 2000 descriptors (pair-index exact in the
    tests).  The reference has no unconstrained all-pairs matcher; its best/second loop is ORBmatcher.cc:568-598 and
    the stereo search of Frame.cc:528-548 without the band.  Timed with HIP events on the launch stream: one match per
    launch (latency) and n_problems matches per launch (throughput, e.g. every stereo pair of a bench step)."""
    import torch
    from multiagent_orb_slam2_amd import synthetic as S
    m = pkg.ORBmatcher(0.6, True, device=dev.index)
    qs, ts = zip(*[S.planted_pairs(7 + z, 2000, 2000) for z in range(8)])
    q1, t1 = torch.from_numpy(qs[0]).to(dev), torch.from_numpy(ts[0]).to(dev)
    qb = torch.from_numpy(np.stack([qs[z % 8] for z in range(n_problems)])).to(dev)
    tb = torch.from_numpy(np.stack([ts[z % 8] for z in range(n_problems)])).to(dev)
    s = torch.cuda.current_stream(dev)
    out = {}
    # both forms, the env switch read per call: the matrix-core form (k_bf_mfma, the default) and the VALU tile kernel
    # (ORBX_BF_MFMA=0, "tile_*"), each checked against the other on the batched outputs
    prev = os.environ.pop("ORBX_BF_MFMA", None)
    for name, fn, nprob in (("single", lambda: m.bf_match_device(q1, t1, stream=s), 1),
                            ("batched", lambda: m.bf_match_batch_device(qb, tb, stream=s), n_problems),
                            ("tile_single", lambda: m.bf_match_device(q1, t1, stream=s), 1),
                            ("tile_batched", lambda: m.bf_match_batch_device(qb, tb, stream=s), n_problems)):
        if name.startswith("tile"):
            os.environ["ORBX_BF_MFMA"] = "0"
        for _ in range(3):
            fn()
        rounds = []                                # median of 5 windows of `reps` launches (one window once read
        for _ in range(5):                         # 6x slow right after the bench step: a clock / power transient)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(reps):
                fn()
            e1.record(s)
            e1.synchronize()
            rounds.append(e0.elapsed_time(e1) * 1e3 / reps)
        us = float(np.median(rounds))
        pairs = 2000 * 2000 * nprob
        alg = 144000 * nprob                       # 2 x 2000 x 32 B in + 2000 x 8 B out per match
        out[name] = {"problems": nprob, "us_per_launch": round(us, 2), "us_per_launch_windows": [round(r, 2) for r in rounds], "matches_per_s": round(nprob / (us * 1e-6), 1),
                     "pair_distances_per_s": round(pairs / (us * 1e-6), 1),
                     "algorithmic_GBps": round(alg / (us * 1e-6) / 1e9, 2)}
    os.environ["ORBX_BF_MFMA"] = "0"
    ref = [x.cpu() for x in m.bf_match_batch_device(qb, tb, stream=s)]
    os.environ.pop("ORBX_BF_MFMA", None)
    got = [x.cpu() for x in m.bf_match_batch_device(qb, tb, stream=s)]
    if prev is not None:
        os.environ["ORBX_BF_MFMA"] = prev
    out["mfma_equals_tile"] = all(bool(torch.equal(a, b)) for a, b in zip(ref, got))
    out["kernels"] = ("k_bf_mfma (popcount(q & t) by v_mfma_i32_16x16x64_i8 on bits unpacked to 0/1 bytes, 64 queries "
                      "per workgroup, train rows unpacked into LDS; one chunk per problem writes the outputs directly, "
                      "else k_bf_merge(_g)); tile_*: k_bf_tile (256 queries per workgroup, one per lane, v_bcnt) + "
                      "k_bf_merge_g")
    c3p = load_profile("r2w_c3_summary.json")
    if c3p:   # VALU fraction of the tile kernel per launch shape (SQ_INSTS_VALU x 64 / profiled duration / peak)
        out["tile_valu_frac_profiled"] = {("batched" if e["grid"] >= 524288 else "single"): e["valu_frac"]
                                     for e in c3p["launches"].values() if e["kernel"] == "k_bf_tile"}
        out["profile"] = "profiles/r2w_c3_summary.json"
    return out


def load_profile(name):
    p = os.path.join(ROOT, "profiles", name)
    if os.path.exists(p):
        try:
            return json.load(open(p))
        except (OSError, ValueError):
            return None
    return None


# Live stage timers (orbx_extractor_stage_times: HIP events on the stream each launch is issued on) of a kernel family's
# launches over the whole batch: (launch spans, busy stage).  k_fast_wave and k_quadtree are two launches per call
# (level 0 on the extractor's side stream, levels 1..7 on the launch stream) that overlap each other; the busy stage is
# the union of the two spans (the wall time during which the kernel runs), which the roofline divides by.
# k_describe_m is one launch on the output stream, k_blur7 two launches in order on the side stream.
LIVE_STAGES = {"k_fast_wave": (("fast_cells", "fast_cells_l0"), "fast_busy"),
               "k_quadtree": (("quadtree", "quadtree_l0"), "quadtree_busy"),
               "k_describe_m": (("describe",), "describe"), "k_blur7": (("blur7",), "blur7")}


def kernel_family(name):
    return name.split("<")[0]


def source_sha16():
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from kernel_share import source_sha16 as f
    return f(ROOT)


def active_kernel_names():
    """Names (as rocprofv3 prints them) of the extractor kernels this process runs (csrc/orbx_extract.hip run_batch):
    k_fast_wave's padded pair rows are 19 dwords for every cell of the KITTI / EuRoC configs (cells up to 38 columns;
    the 40-dword form only for wider ones), 4 waves per workgroup."""
    return {"fast": "k_fast_wave<19, 4, 4>", "describe": "k_describe_m<2>", "blur": "k_blur7",
            "families": {"k_fast_wave", "k_describe_m", "k_quadtree", "k_blur7", "k_resize4"}}


def roofline_lines(per_call, cfg, units, config):
    """Roofline of the dominant kernel -- the one with the largest share of GPU time in the committed kernel trace of
    the bench command (profiles/kernel_share.json, scripts/kernel_share.py) -- and of the describe as a secondary
    line.  achieved = SURVEY §8(d) algorithmic bytes of the extractions the kernel's launches cover per step (one
    extraction = image in + nfeatures x 60 B out; every launch family covers all 2B images once) / the kernel's live
    busy time per step (the union of its launches' event spans: the two FAST launches run at once on two streams, so
    the sum of their spans counts the overlap twice).  The committed profile's figures sit beside it:
    rocprof_busy_ms_per_step (the union of the traced launch intervals per step) and rocprof_launch_avg_us (the
    average duration of each of the two launch grids); frac_rocprof = bytes / the traced busy time."""
    share = load_profile("kernel_share.json")
    cb = compulsory_bytes(cfg)["extraction"]
    names = active_kernel_names()
    fast_fam = kernel_family(names["fast"])
    dom = fast_fam
    prof, stale, tag = None, None, None
    if share and share.get("config", "kitti") == config and share.get("batch_images") == units \
            and kernel_family(share["dominant"]) in names["families"]:       # a profile of the kernels that run
        dom = kernel_family(share["dominant"])
        tag = share.get("tag")
        stale = share.get("source_sha16") != source_sha16()
        prof = [k for k in share["kernels"] if kernel_family(k["kernel"]) == dom]

    def line(fam, kernel_name):
        if fam not in LIVE_STAGES:
            return None
        stages, busy = LIVE_STAGES[fam]
        if busy not in per_call or any(st not in per_call for st in stages):
            return None
        t_ms = per_call[busy]
        bytes_step = cb * units
        achieved = bytes_step / (t_ms * 1e-3) / 1e9
        traffic = None
        pmc = load_profile("pmc_traffic.json")
        if pmc and kernel_family(pmc.get("kernel", "")) == fam and pmc.get("batch_images") == units \
                and pmc.get("config", "kitti") == config:
            traffic = pmc.get("hbm_bytes_per_step", pmc.get("hbm_bytes_per_launch"))
        return {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic, "kernel": kernel_name,
                "launches_per_step": len(stages), "live_stages": list(stages), "live_busy_stage": busy,
                "kernel_ms_per_step": round(t_ms, 4),
                "launch_span_ms": {st: round(per_call[st], 4) for st in stages},
                "algorithmic_bytes_per_step": bytes_step,
                "algorithmic_bytes_per_unit": cb, "units_per_step": units,
                "traffic_ratio": round(traffic / bytes_step, 2) if traffic else None,
                "unit_of_work": "one extraction (SURVEY §8d: image in + nfeatures x 60 B out); the kernel's launches of a "
                                "step together cover every image of the batch once"}
    desc_name = names["describe"]
    full = {kernel_family(n): n for n in (names["fast"], desc_name, "k_quadtree", names["blur"])}
    main_line = line(dom, full.get(dom, dom)) or line(fast_fam, names["fast"])
    if main_line is not None:
        main_line["selected_by"] = (f"largest share of GPU time in profiles/kernel_share.json ({tag})" if tag else
                                    "default (no kernel_share.json for this config)")
        # the live figure: the union of the launches' HIP-event spans in the overlapped step, which includes each
        # launch's wait for CU slots behind the other queues
        main_line["achieved_live"] = main_line["achieved"]
        main_line["frac_live"] = main_line["frac"]
        main_line["frac_source"] = "live"
        if prof:
            k0 = prof[0]
            grids = k0.get("grids", [])
            main_line["rocprof_busy_ms_per_step"] = k0.get("busy_ms_per_step")
            main_line["rocprof_launches_per_step"] = k0.get("launches_per_step")
            main_line["rocprof_launch_avg_us"] = [g["avg_us"] for g in grids]
            # headline: the kernel's own duration = the profiled average duration of each of its launches per step
            # (one launch per grid per step), summed; bytes per step / that time
            dur_ms = sum(g["avg_us"] for g in grids) * 1e-3 if grids else k0.get("busy_ms_per_step")
            if dur_ms and not stale:
                ach = main_line["algorithmic_bytes_per_step"] / (dur_ms * 1e-3) / 1e9
                main_line.update(achieved=round(ach, 3), frac=round(ach / HBM_PEAK_GBS, 6),
                                 kernel_ms_per_step=round(dur_ms, 4), frac_source="rocprof launch durations")
            if k0.get("busy_ms_per_step"):
                main_line["frac_rocprof"] = round(main_line["algorithmic_bytes_per_step"] /
                                                  (k0["busy_ms_per_step"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 6)
            main_line["profile"] = f"profiles/kernel_share.json ({tag})"
            main_line["profile_stale"] = stale
        pmc = load_profile("pmc_traffic.json")
        if pmc and pmc.get("step_hbm_bytes") and pmc.get("batch_images") == units and pmc.get("config", "kitti") == config:
            # every kernel of the step, not the dominant one only: what the whole step moves through HBM
            main_line["traffic_step"] = pmc["step_hbm_bytes"]
            main_line["traffic_step_kernels_ms"] = pmc.get("step_kernel_ms")
            main_line["traffic_step_source"] = pmc.get("source")
    sec = line(kernel_family(desc_name), desc_name) if kernel_family(desc_name) != dom else None
    return main_line, sec


def valu_line(roof, config, units):
    """VALU roofline of the same kernel: SQ_INSTS_VALU x 64 lane-ops per step from the committed SQ pass
    (profiles/sq_summary.json), over the same kernel time as the HBM line (profiled launch durations when the profile
    matches the sources, else the live spans); dropped when the SQ profile was taken on other sources."""
    sq = load_profile("sq_summary.json")
    if not (roof and sq and sq.get("config", "kitti") == config and sq.get("batch_images") == units):
        return None
    if sq.get("source_sha16") != source_sha16():
        return None
    fam = kernel_family(roof["kernel"])
    ks = [(k, v) for k, v in sq["kernels"].items() if kernel_family(k) == fam]
    if not ks:
        return None
    ops = sum(v["valu_lane_ops"] * v.get("launches_per_step", 1) for _, v in ks)
    t_ms = roof["kernel_ms_per_step"]
    tops = ops / (t_ms * 1e-3) / 1e12
    return {"bound": "valu", "achieved": round(tops, 3), "peak": round(VALU_PEAK_TOPS, 2), "unit": "Tlane-op/s",
            "frac": round(tops / VALU_PEAK_TOPS, 4), "kernel": roof["kernel"], "valu_lane_ops_per_step": ops,
            "profiled_valu_frac": {k: v.get("valu_frac") for k, v in ks},
            "source": f"SQ_INSTS_VALU x 64 per launch from profiles/sq_summary.json ({sq.get('tag')}, sources "
                      f"{sq.get('source_sha16')}), over the roofline's kernel_ms_per_step ({roof.get('frac_source', 'live')})"}


def world_from_env(gpus: int):
    """(launch here?, world size) from --gpus and a launcher's WORLD_SIZE: without WORLD_SIZE, --gpus N > 1 means this
    process starts the N ranks itself; with it, the two must agree (a torchrun of N ranks asked for M GPUs is an error,
    not a silent 1-rank line)."""
    env = os.environ.get("WORLD_SIZE")
    if env is None:
        return gpus > 1, 1
    if int(env) != gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={env} from the launcher but --gpus {gpus}")
    return False, int(env)


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    spawn, world = world_from_env(args.gpus)
    if spawn:
        # before anything touches the GPU: the children initialise it, one device each
        sys.exit(launch_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]))
    cfg = dict(CONFIGS[args.config])
    os.environ["ORBX_CU_EXCLUDE"] = str(max(args.cu_exclude, 0))   # the extractors' side streams (read at creation)
    ROWS, COLS, NFEAT, BF = cfg["rows"], cfg["cols"], cfg["nfeatures"], cfg["bf"]
    BASELINE_B = BF / cfg["fx"]
    import torch
    import torch.distributed as dist

    import multiagent_orb_slam2_amd as pkg
    from multiagent_orb_slam2_amd import multiagent as MA
    from multiagent_orb_slam2_amd import synthetic as S

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n_dev = torch.cuda.device_count()
    if world > 1:
        if n_dev < world and args.dist_backend == "nccl":
            raise SystemExit(f"bench.py: {world} ranks over RCCL need {world} GPUs, {n_dev} visible "
                             "(--dist-backend gloo rehearses the N>1 step with ranks sharing a GPU)")
        if args.exchange == "native" and args.dist_backend != "nccl":
            raise SystemExit("bench.py: --exchange native needs --dist-backend nccl (one GPU per rank)")
        local = local % max(1, n_dev)                        # (gloo rehearsal: more ranks than GPUs share them)
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
        if dist.get_world_size() != world:
            raise SystemExit(f"bench.py: process group has {dist.get_world_size()} ranks, expected {world}")
        world = dist.get_world_size()
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    devices_used = min(world, max(1, n_dev))

    B = args.batch
    # distinct scenes: a multiple of KF_EVERY by default (255 at B = 256: one scene shown twice in a step), so that every
    # agent's keyframes -- the frames f = 0 mod KF_EVERY of its chunk -- show the same nd / KF_EVERY scenes whatever its
    # chunk offset, as agents mapping one area revisit what the others saw, and MapFusion finds cross-agent candidates
    nd = max(1, min(args.distinct, B)) if args.distinct > 0 else (B - B % KF_EVERY if B >= KF_EVERY else B)
    # this agent's contiguous chunk of one synthetic sequence (generic_split_seq.cc:543-589); frame f of the
    # sequence is the synthetic stereo pair of seed f
    emu = max(args.emulate_agents, 1) if world == 1 else 1
    kfw = world if world > 1 else emu                 # agents whose keyframes fill the ring (emulated at N = 1)
    chunk = MA.split_sequence(cfg["seq_frames"], world)[rank]
    # frame f of the sequence shows synthetic scene f mod nd: every agent's chunk revisits the same nd scenes (in its
    # own order), as agents exploring one area do -- MapFusion's cross-agent candidates exist at every N, so the
    # keyframe path does the same matching work per rank at N > 1 as at N = 1 (where the agent revisits its own)
    seeds = [(chunk.start + i) % nd for i in range(nd)]
    lefts = [S.kitti_like_image(s, rows=ROWS, cols=COLS) for s in seeds]
    rights = [S.shifted_right_view(l, s) for s, l in zip(seeds, lefts)]
    host = np.stack([lefts[i % nd] for i in range(B)] + [rights[i % nd] for i in range(B)])
    imgs = torch.from_numpy(host).to(dev)               # resident in HBM before timing
    img_sets = [imgs] + [torch.roll(imgs, shifts=(3 * k, 11 * k), dims=(1, 2)).contiguous()
                         for k in range(1, max(1, args.input_sets))]

    n_ctx = max(1, args.inflight)
    exs = [pkg.ORBextractor(NFEAT, SCALE, NLEV, INI, MINTH, device=dev.index) for _ in range(n_ctx)]
    for e_ in exs:
        e_.reserve(ROWS, COLS, 2 * B)
    ex = exs[0]
    m = pkg.ORBmatcher(0.6, True, device=dev.index)
    scale = ex.GetScaleFactors()
    cap = ex.max_keypoints(ROWS, COLS)
    # NS sets of extractor outputs: step k's keyframe path (on its own queue) reads set k % NS while later steps'
    # front-end writes the other set; the front-end waits for the keyframe path of step k-1 before reusing a set
    NS = max(2, args.sets)
    outs = [(torch.empty((2 * B, cap, 28), dtype=torch.uint8, device=dev),
             torch.empty((2 * B, cap, 32), dtype=torch.uint8, device=dev),
             torch.empty((2 * B,), dtype=torch.int32, device=dev)) for _ in range(NS)]
    mk = (lambda prio=0: pkg.orbx.create_stream(dev.index, prio, args.cu_exclude)) if args.cu_exclude > 0 else \
        (lambda prio=0: torch.cuda.Stream(dev, priority=prio))
    streams = [mk(int(os.environ.get("ORBX_MAIN_PRIORITY", "0"))) for _ in range(n_ctx)]   # front-end queues
    torch.cuda.set_stream(streams[0])
    # stereo queue: step k's ComputeStereoMatches (band match + SAD refinement on step k's pyramids) runs beside
    # step k+1's extraction; the extractor cycles two pyramid sets so that step k+1 does not overwrite step k's
    stereo_stream = mk(int(os.environ.get("ORBX_STEREO_PRIORITY", "0")))
    # descriptor stage: on the stereo queue by default (stereo k needs describe k anyway), so that step k+1's resize
    # chain and level-0 FAST run beside step k's describe (2.115 -> 2.019 ms/step with 3 sets and an unthrottled
    # host; on the launch stream the describe ran alone).  A fifth busy queue (--desc-stream 2) is starved by the
    # hardware scheduler (measured: the keyframe path's small kernels then wait 0.1-0.3 ms each; 2.57 ms/step)
    desc_streams = ([stereo_stream] * n_ctx if args.desc_stream == 1 else
                    [mk() for _ in range(n_ctx)] if args.desc_stream == 2 else [None] * n_ctx)
    NP = args.pyr_sets if args.pyr_sets > 0 else NS
    for e_ in exs:
        e_.set_pyramid_ring(NP)
    stereo_done = [None] * NP                          # per pyramid set: the stereo step that last read it
    # keyframe queue: BoW, packets, exchange, KeyFrameDatabase, SearchByBoW -- the native orbx_fusion object.  As in
    # the reference, where LoopClosing and MapFusion run in their own threads beside Tracking, step k's keyframe work
    # overlaps step k+1's extraction.
    # Priority: -1 (high) until r5bt, where with the DistributeOctTree of levels >= 1 on the stereo queue (r5bk) the
    # keyframe stream at normal priority measured +0.8 % (76.5k -> 77.1k frames/s, three rounds; +0.9 % at 8 emulated
    # agents).  (A stream of another priority gets a hardware queue of its own; two same-priority streams can share one,
    # which in round 3 serialised front-end and keyframe kernels, +0.5 ms per step.)  ORBX_KF_PRIORITY overrides.
    kf_prio = int(os.environ.get("ORBX_KF_PRIORITY", "0"))
    kf_stream = (pkg.orbx.create_stream(dev.index, kf_prio, -args.kf_cus) if args.kf_cus > 0 else
                 torch.cuda.Stream(dev, priority=kf_prio))
    track_stream = mk() if args.track_stream == "own" else None
    kf_done = [None] * NS
    n_kf = max(1, B // KF_EVERY)
    voc = S.synthetic_vocabulary(2024, k=10, L=6)      # ORBvoc.txt's shape ("10 6 0 0"); the file is absent
    vocab = pkg.ORBVocabulary.from_arrays(voc, device=dev.index)
    exchange = None
    if world > 1:
        exchange = (MA.NativeKeyframeExchange(timed=not args.no_timing, device=dev.index) if args.exchange == "native"
                    else MA.KeyframeExchange(timed=not args.no_timing))
    engine = pkg.KeyframeFusionEngine(vocab, pkg.ORBmatcher(0.75, True, device=dev.index), cap,
                                      slots=STORE_STEPS * kfw * n_kf, max_keyframes=n_kf, candidates=KF_CANDIDATES,
                                      agent=rank, world=kfw, device=dev.index)
    # every 5th frame of the sequence becomes a keyframe: batch rows kf_off + 5j, the frames of the chunk = 0 mod 5
    # (kf_off <= 4, so the 51 rows of a 256-frame batch end at row <= 254)
    kf_off = (-chunk.start) % KF_EVERY
    if kf_off + KF_EVERY * (n_kf - 1) >= B:
        kf_off = 0
    kf_rows = range(kf_off, kf_off + KF_EVERY * n_kf, KF_EVERY)
    # CreateNewMapPoints' matching per new keyframe: SearchForTriangulation vs its TRI_NEIGHBOURS previous keyframes of
    # this agent (all pairs in one launch; MapPoint flags = the store's valid field, i.e. stereo depth > 0), then
    # the distinctive descriptors of its keypoints' observation lists.  FeatureVector nodes at levelsup 4 of a k=10,
    # L=6 tree: at most 10^2 per keyframe
    geo = Geometry(cfg, STORE_STEPS * n_kf)
    tri, tri_pat = None, {}

    def tri_pattern(q):
        """(new slots, neighbour slots) of this agent's keyframes q (a slot range) as device tensors and host arrays: the
        d-th previous keyframe of keyframe j sits (j - d) keyframes back in this agent's ring order."""
        if q.start not in tri_pat:
            nq, per = len(q), kfw * n_kf
            nb = [[(q.start + ((j - d) // nq) * per + (j - d) % nq) % engine.slots for d in range(1, TRI_NEIGHBOURS + 1)]
                  for j in range(nq)]
            tri_pat[q.start] = (torch.tensor(list(q), dtype=torch.int32, device=dev),
                                torch.tensor(nb, dtype=torch.int32, device=dev),
                                np.array(list(q), np.int64), np.array(nb, np.int64))
        return tri_pat[q.start]
    if args.tri:
        tri = MA.NewMapPoints(engine.store, 100, ex.GetScaleSigmaSquares(), ex.GetScaleFactors(),
                              matcher=pkg.ORBmatcher(0.6, False, device=dev.index))
        tri_geom = geo.tri_rows().float().to(dev).view(1, TRI_NEIGHBOURS, 12).expand(n_kf, -1, -1).contiguous()
    grid = pkg.frame_grid(0, 0, COLS, ROWS)
    log_sf = float(np.float32(np.log(SCALE)))
    inv_sigma2 = ex.GetInverseScaleSigmaSquares()
    tracker = None
    if args.tracking:
        twc_last, v_lf, v_mp = geo.tracking_views()
        tracker = MA.FrameTracker(pkg.ORBmatcher(0.9, True, device=dev.index), B, cap, grid, geo.camera, BF, scale, log_sf,
                                  dev, NS, twc_last, v_lf, v_mp, inv_sigma2)
    fuse = None
    kf_rows_t = torch.tensor(list(kf_rows), dtype=torch.int64, device=dev)
    if args.fuse:
        twc_s, views_s = geo.slot_tables(engine.slots, kfw, n_kf)
        fuse = MA.LocalFuse(pkg.ORBmatcher(0.6, True, device=dev.index), engine.store, engine.slots, cap, grid, geo.camera,
                            BF, scale, log_sf, inv_sigma2, twc_s, views_s, dev)
    if kfw > 1:
        send = torch.empty((n_kf, engine.packet_bytes), dtype=torch.uint8, device=dev)
        # --exchange-copy (A/B only): gather into a separate buffer and let commit copy it into the ring (round 5)
        gathered = torch.empty((kfw * n_kf, engine.packet_bytes), dtype=torch.uint8, device=dev) if args.exchange_copy else None
    frame_no = [chunk.start]
    n_step = [0]

    skip = set(filter(None, args.diag_skip.split(",")))
    stereo_ms = []
    track_ms = []
    kf_ms = []
    tri_ms = []
    fuse_ms = []
    host_split = [0.0, 0.0]                            # host enqueue seconds: front-end, keyframe path

    last_handoff = [None]
    timeline = []                                      # per timed step: {point: event}, read after the timed region

    def step(time_stereo=False, src=None):
        h0 = time.perf_counter()
        buf = n_step[0] % NS
        ex = exs[n_step[0] % n_ctx]
        stream = streams[n_step[0] % n_ctx]
        dstream = desc_streams[n_step[0] % n_ctx]       # the descriptor stage (writes the outputs)
        ostream = dstream if dstream is not None else stream
        kps, desc, cnt = outs[buf]
        if kf_done[buf] is not None:
            # the keyframe path of two steps ago has read this output set (written by the descriptor stage), and the
            # stereo step before it the pyramid set this call's resize chain overwrites
            stream.wait_event(kf_done[buf])
            if dstream is not None:
                dstream.wait_event(kf_done[buf])
        pslot = n_step[0] % NP
        if stereo_done[pslot] is not None:
            stream.wait_event(stereo_done[pslot])     # the resize chain overwrites the set that stereo step read
        if src is None:
            src = img_sets[n_step[0] % len(img_sets)]
        tl = {}                                        # timeline events of this step (timed steps only)
        if time_stereo:
            tl["front_end_start"] = torch.cuda.Event(enable_timing=True)
            tl["front_end_start"].record(stream)
        ex.extract_batch_device(src, kps, desc, cnt, stream=stream, out_stream=dstream)
        extracted = torch.cuda.Event(enable_timing=time_stereo)
        extracted.record(ostream)
        if time_stereo:
            tl["describe_end"] = extracted
            timeline.append(tl)
        pyr = ex.pyramid_device()                      # this call's pyramid set (a slot of the ring of 2)
        if "stereo" in skip:
            n_step[0] += 1
            return None, None
        stereo_stream.wait_event(extracted)
        with torch.cuda.stream(stereo_stream):         # outputs allocated on (and owned by) the stereo queue
            if time_stereo:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stereo_stream)
            bi, bd = m.stereo_match_batch_device(kps[:B], desc[:B], cnt[:B], kps[B:], desc[B:], cnt[B:], cap, scale,
                                                 ROWS, BF, BASELINE_B, stream=stereo_stream)
            ur, depth = m.stereo_refine_batch_device(kps[:B], cnt[:B], kps[B:], bi, pyr, 0, pyr, B, BF, BASELINE_B,
                                                     stream=stereo_stream,
                                                     out=tracker.stereo_out(buf) if tracker is not None else None)
            if time_stereo:
                e1.record(stereo_stream)
                stereo_ms.append((e0, e1))
                tl["stereo_start"], tl["stereo_end"] = e0, e1
            if tracker is not None and args.track_stream == "stereo":
                # Tracking's matches of every frame: TrackWithMotionModel's SearchByProjection(F, LastF) and
                # SearchLocalPoints (Tracking.cc:882-904, :1160-1205) on the frame's stereo MapPoints
                tracker.run(buf, kps[:B], desc[:B], cnt[:B], stream=stereo_stream)
                if time_stereo:
                    e1t = torch.cuda.Event(enable_timing=True)
                    e1t.record(stereo_stream)
                    track_ms.append((e1, e1t))
                    tl["tracking_end"] = e1t
        handoff = torch.cuda.Event()
        handoff.record(stereo_stream)
        stereo_done[pslot] = handoff
        last_handoff[0] = handoff
        if tracker is not None and args.track_stream in ("kf", "own"):
            # the tracking matches on the keyframe queue (or a queue of their own), after the stereo step that gives
            # their MapPoints (depth), so that the stereo queue (describe, stereo) is free for the next step
            tq = kf_stream if args.track_stream == "kf" else track_stream
            tq.wait_event(handoff)
            with torch.cuda.stream(tq):
                if time_stereo:
                    e0t = torch.cuda.Event(enable_timing=True)
                    e0t.record(tq)
                tracker.run(buf, kps[:B], desc[:B], cnt[:B], stream=tq)
                if time_stereo:
                    e1t = torch.cuda.Event(enable_timing=True)
                    e1t.record(tq)
                    track_ms.append((e0t, e1t))
                    tl["tracking_end"] = e1t
            if args.track_stream == "own":
                tdone = torch.cuda.Event()
                tdone.record(track_stream)
                kf_stream.wait_event(tdone)            # kf_done[buf] then also covers the tracking's reads of set buf
        h1 = time.perf_counter()
        if "keyframes" in skip:
            n_step[0] += 1
            return bi, bd
        # keyframe path: rows of this step's batch -> BoW -> packets -> all-gather (N>1) into the ring -> sequential
        # DetectLoopCandidates -> batched SearchByBoW; MapPoint-valid = stereo depth > 0
        kf_stream.wait_event(handoff)
        depth.record_stream(kf_stream)
        if time_stereo:
            e2 = torch.cuda.Event(enable_timing=True)
            e2.record(kf_stream)
        if kfw == 1:
            engine.step(kps, desc, cnt, kf_rows, frame_no[0] + kf_off, KF_EVERY, depth=depth, stream=kf_stream)
        else:
            engine.pack(kps, desc, cnt, kf_rows, frame_no[0] + kf_off, KF_EVERY, depth=depth, send=send, stream=kf_stream)
            # the all-gather lands in the ring slots pack() reserved (engine.exchange_view()), and commit takes them in
            # place; with --exchange-copy through a separate buffer that commit copies into the ring
            dst = gathered if gathered is not None else engine.exchange_view()
            with torch.cuda.stream(kf_stream):
                if world > 1:
                    exchange.exchange(send, out=dst)
                else:                                  # --emulate-agents: every agent's block is this rank's packets
                    dst.view(kfw, n_kf, -1).copy_(send.unsqueeze(0).expand(kfw, -1, -1))
            engine.commit(gathered, stream=kf_stream)
        if time_stereo:
            e3 = torch.cuda.Event(enable_timing=True)
            e3.record(kf_stream)
            kf_ms.append((e2, e3))
            tl["keyframe_start"], tl["keyframe_bow_fusion_end"] = e2, e3
        qs = engine.last_step()[1]
        ns, nb, ns_h, nb_h = tri_pattern(qs)
        e5 = e3 if time_stereo else None
        if tri is not None:
            with torch.cuda.stream(kf_stream):
                tri.run(ns, nb, tri_geom)
            if time_stereo:
                e5 = torch.cuda.Event(enable_timing=True)
                e5.record(kf_stream)
                tri_ms.append((e3, e5))
        if fuse is not None:
            # SearchInNeighbors' Fuse (LocalMapping.cc:486-520): the new keyframes' MapPoints into each neighbour and
            # the neighbours' MapPoints into them
            fuse.add_keyframes(qs, kps, desc, cnt, ur, depth, kf_rows_t, stream=kf_stream)
            fuse.run(ns_h, nb_h, stream=kf_stream)
            if time_stereo:
                e6 = torch.cuda.Event(enable_timing=True)
                e6.record(kf_stream)
                fuse_ms.append((e5, e6))
                tl["keyframe_end"] = e6
        done = torch.cuda.Event()
        done.record(kf_stream)
        kf_done[buf] = done
        frame_no[0] += B
        n_step[0] += 1
        h2 = time.perf_counter()
        host_split[0] += h1 - h0
        host_split[1] += h2 - h1
        return bi, bd

    for _ in range(STORE_STEPS):                       # fill the keyframe store ring (setup, untimed)
        step()

    # pure host cost of a step: the last warmup steps start on an idle GPU (no back-pressure wait inside)
    pure_s, pure_n = 0.0, 0
    for i in range(args.warmup):
        if i >= args.warmup - 3:
            torch.cuda.synchronize()
            host_split[0] = host_split[1] = 0.0
            th = time.perf_counter()
            step()
            pure_s += time.perf_counter() - th
            pure_n += 1
            pure_split = list(host_split)
        else:
            step()
    torch.cuda.synchronize()
    if not args.no_timing:
        for e_ in exs:
            e_.enable_timing(True)
    if exchange is not None:
        exchange.reset_stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    tl_base = torch.cuda.Event(enable_timing=True)
    tl_base.record(streams[0])
    t0 = time.perf_counter()
    host_s = 0.0
    split0 = list(host_split)
    for _ in range(args.steps):
        th = time.perf_counter()
        step(time_stereo=not args.no_timing)
        host_s += time.perf_counter() - th               # host time to enqueue one step (no sync inside)
        if args.sync_each:
            torch.cuda.synchronize()
    split1 = list(host_split)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    frames = B * args.steps * world
    value = frames / el
    collective = ("gloo all-gather staged through host memory (rehearsal, not xGMI)" if args.dist_backend == "gloo" else
                  "RCCL all-gather (liborbx orbx_exchange: native communicator, xGMI)" if args.exchange == "native" else
                  "RCCL all-gather (torch.distributed nccl, xGMI)")
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1000 * el / args.steps, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        # host CPU time to enqueue one step, measured on steps that start with the GPU idle; the host wall time per
        # timed step also holds the waits that keep it a few steps ahead of the GPU (back-pressure)
        "host_enqueue_ms_per_step": round(1000 * pure_s / max(pure_n, 1), 3),
        "host_enqueue_split_ms": {"front_end": round(1000 * pure_split[0], 3) if pure_n else None,
                                  "keyframe_path": round(1000 * pure_split[1], 3) if pure_n else None},
        "host_wall_ms_per_timed_step": round(1000 * host_s / args.steps, 3),
        "host_wall_split_ms_per_timed_step": {"front_end": round(1000 * (split1[0] - split0[0]) / args.steps, 3),
                                              "keyframe_path": round(1000 * (split1[1] - split0[1]) / args.steps, 3)},
        "config": {"workload": f"{args.config}: stereo frame = ORBextractor x2 ({COLS}x{ROWS}, 8 levels, {NFEAT} kpts) + "
                               "stereo L<->R 256-bit Hamming band match + SAD sub-pixel refinement" +
                               ("; tracking matches: the last frame's stereo MapPoints projected + SearchByProjection "
                                "(motion model, th 7) + isInFrustum + SearchByProjection (local map, th 1)"
                                if args.tracking else "") +
                               "; every 5th frame a keyframe: DBoW2 transform (k=10, L=6) + " +
                               (f"{collective} of KF packets + " if world > 1 else "") +
                               "KeyFrameDatabase DetectLoopCandidates (query, then add) over the KF store + "
                               f"SearchByBoW vs the first {KF_CANDIDATES} candidates" +
                               (" of other agents' maps (MapFusion.cc:136-144)" if world > 1 else
                                " of the agent's own map with minScore 0 (LoopClosing-like: N=1 has no other map, so these "
                                "pairs are work MapFusion itself would not do)") +
                               (f"; CreateNewMapPoints matching: SearchForTriangulation vs {TRI_NEIGHBOURS} neighbour "
                                "keyframes + the new MapPoints' distinctive descriptors" if args.tri else "") +
                               (f"; SearchInNeighbors' Fuse: the new keyframe's MapPoints into each of its "
                                f"{TRI_NEIGHBOURS} neighbours and theirs into it (projection + window search, th 3)"
                                if args.fuse else ""),
                   "settings": cfg["source"],
                   "keyframes_per_gpu_per_step": n_kf, "bow_pairs_per_gpu_per_step": n_kf * KF_CANDIDATES,
                   "global_batch": B * world, "frames_per_gpu_per_step": B, "image": [ROWS, COLS],
                   "nfeatures": NFEAT, "nlevels": NLEV, "distinct_stereo_pairs_per_gpu": nd,
                   "keyframe_rows": [kf_rows.start, kf_rows.stop, kf_rows.step],
                   "input_sets": len(img_sets), "input_bytes_resident": int(sum(t.numel() for t in img_sets)),
                   "sequence_chunk": [chunk.start, chunk.stop],
                   "parallelism": f"agent-per-gpu x{world}"},
        "ranks": {"world_size": world, "devices_used": devices_used, "backend": args.dist_backend if world > 1 else None,
                  "launched_by": os.environ.get("ORBX_LAUNCHER", "torchrun" if "TORCHELASTIC_RUN_ID" in os.environ
                                                else "bench.py" if world > 1 else "single process")},
    }
    if world > devices_used:
        out["rehearsal"] = f"{world} ranks sharing {devices_used} GPU(s): not a scaling measurement"
    if emu > 1:
        out["emulated_agents"] = {"agents": emu, "ring_slots": engine.slots,
                                  "note": "diagnostics: rank 0's keyframe path under an N-agent ring load on one GPU; the "
                                          "packets are this rank's own copied N times, no collective"}

    if not args.no_timing:
        st, calls = {}, 0
        for e_ in exs:
            s_, c_ = e_.stage_times()
            calls += c_
            for k, v in s_.items():
                st[k] = st.get(k, 0.0) + v
        per_call = {k: v / max(calls, 1) for k, v in st.items()}
        sms = [a.elapsed_time(b) for a, b in stereo_ms]
        per_call["stereo_match"] = float(np.mean(sms)) if sms else 0.0
        kms = [a.elapsed_time(b) for a, b in kf_ms]
        per_call["keyframe_bow_fusion"] = float(np.mean(kms)) if kms else 0.0
        tms = [a.elapsed_time(b) for a, b in tri_ms]
        if tms:
            per_call["keyframe_new_mappoints"] = float(np.mean(tms))   # after keyframe_bow_fusion, same stream
        fms = [a.elapsed_time(b) for a, b in fuse_ms]
        if fms:
            per_call["keyframe_fuse"] = float(np.mean(fms))            # after keyframe_new_mappoints, same stream
        trk = [a.elapsed_time(b) for a, b in track_ms]
        if trk:
            per_call["tracking_match"] = float(np.mean(trk))           # after stereo_match, the stereo stream
        out["stage_ms_per_step"] = {k: round(v, 4) for k, v in per_call.items()}
        if len(timeline) >= 4:
            # when each stage of step i happens, relative to step i's front-end start (the launch stream reaching the
            # extraction, after its waits); medians over the timed steps from the 2nd on.  Read with the period
            # (median front-end start to the next step's) to see how consecutive steps overlap.
            offs = [{k: tl_base.elapsed_time(e) for k, e in t.items()} for t in timeline]
            period = [offs[i + 1]["front_end_start"] - offs[i]["front_end_start"] for i in range(1, len(offs) - 1)]
            rel = {k: round(float(np.median([o[k] - o["front_end_start"] for o in offs[1:] if k in o])), 3)
                   for k in offs[1]}
            out["timeline_ms"] = dict(rel, step_period=round(float(np.median(period)), 3))
        out["roofline"], sec = roofline_lines(per_call, cfg, 2 * B, args.config)
        if sec:
            out["roofline_secondary"] = sec
        v = valu_line(out["roofline"], args.config, 2 * B)
        if v:
            out["roofline_valu"] = v
    if exchange is not None:
        xs = exchange.stats()
        if xs:
            out["exchange"] = dict(xs, collective=collective,
                                   packet_bytes=engine.packet_bytes, keyframes_per_rank=n_kf)
        sizes = [float(s) for s in args.xgmi_mb.split(",") if s.strip()]
        if sizes:
            # after the timed region: the same collective alone, at the step's packet payload and larger ones
            torch.cuda.synchronize()
            with torch.cuda.stream(kf_stream):
                sweep = MA.allgather_sweep(exchange, dev, sizes)
            out["xgmi_allgather"] = {"collective": collective, "world_size": world, "sweep": sweep,
                                     "link_peak_GBps_per_direction": 153.6 if args.dist_backend == "nccl" else None,
                                     "note": "busbw = bytes each rank receives / time; xGMI is point-to-point (7 links "
                                             "per MI355X), so a ring all-gather's busbw is bounded by one link"}

    if rank == 0 and world == 1 and args.c3:
        out["c3_bruteforce"] = c3_bench(pkg, dev)
    if rank == 0 and world == 1 and not args.no_timing and args.alone_reps > 0:
        per, calls = alone_block(pkg, cfg, img_sets[0], dev, args.alone_reps)
        fam = kernel_family(active_kernel_names()["fast"])
        t_ms = sum(per.get(st_, 0.0) for st_ in LIVE_STAGES[fam][0])            # serial: the spans do not overlap
        cb = compulsory_bytes(cfg)["extraction"] * 2 * B
        ach = cb / (t_ms * 1e-3) / 1e9 if t_ms > 0 else 0.0
        out["roofline_alone"] = {"bound": "hbm", "achieved": round(ach, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": round(ach / HBM_PEAK_GBS, 6), "kernel": active_kernel_names()["fast"],
                                 "kernel_ms_per_step": round(t_ms, 4), "algorithmic_bytes_per_step": cb,
                                 "stage_ms_alone": per, "calls": calls,
                                 "schedule": "the step's extraction only, every stage on one stream (ORBX_PIPELINE=0), "
                                             "HIP events around each kernel: each kernel's own duration"}
    gate, _ = engine.stats()
    out["fusion_gate_passed_per_step"] = round(gate / (args.steps + args.warmup + STORE_STEPS), 2)
    if rank == 0 and world == 1 and args.host_fed_steps > 0:
        out["host_fed"] = host_fed_block(step, last_handoff, host, streams[0], B, args.host_fed_steps, dev)
    if rank == 0 and world == 1 and args.cd:
        torch.cuda.synchronize()
        kps_l, desc_l, cnt_l = outs[(n_step[0] - 1) % NS]
        out["covisibility_discovery"] = cd_block(pkg, MA, kps_l, desc_l, cnt_l, vocab, B)
    if rank == 0 and world == 1 and args.host_api_frames > 0:
        out["host_api"] = host_api_rate(pkg, cfg, lefts[:8], rights[:8], args.host_api_frames, dev.index)
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        out["cpu_baseline"] = cpu_baseline(lefts[:16], rights[:16], cfg, S.synthetic_vocabulary(2024, k=10, L=6), n_kf,
                                           args.cpu_seconds, geo, tri=args.tri, track=args.tracking, fuse=args.fuse)
    if skip:
        out["diag_skip"] = sorted(skip)
    engine.check()
    if rank == 0:
        print(json.dumps(out), flush=True)
    # ordered teardown while the runtime is up: every queue drained, then the library objects destroyed newest first
    torch.cuda.synchronize()
    pkg.orbx.close_all()
    pkg.orbx.device_check(dev.index)                   # raises (exit status 1) on a pending device error
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
