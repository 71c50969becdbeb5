"""Seeded test cases for the projection / radius matchers and a pure-Python
restatement of the reference's sequential loops (src/ORBmatcher.cc, src/Frame.cc) used to check the
C++ oracle on small cases.  No reference code or data is copied: cases are synthetic keypoint sets whose
queries are perturbed copies of target keypoints (true matches), distractors, and dense conflicts."""
from __future__ import annotations

import math

import numpy as np

from multiagent_orb_slam2_amd.orbx import (KP_DTYPE, PROJ_BEST, PROJ_FUSE, PROJ_INIT, PROJ_KEYFRAME, PROJ_LASTFRAME,
                                           PROJ_MAPPOINTS, PROJ_QUERY_DTYPE, PROJ_SIM3, QF_BLOCKS, QF_SKIP, ProjParams,
                                           frame_grid)

SCALE = np.array([1.2 ** i for i in range(8)], np.float32)
INV_SIGMA2 = (np.float32(1) / (SCALE * SCALE)).astype(np.float32)
MODES = {"mappoints": PROJ_MAPPOINTS, "lastframe": PROJ_LASTFRAME, "keyframe": PROJ_KEYFRAME, "sim3": PROJ_SIM3,
         "fuse": PROJ_FUSE, "best": PROJ_BEST, "init": PROJ_INIT}


def make_case(seed: int, mode: int, n_target: int = 400, n_query: int = 300, W: int = 640, H: int = 480,
              dense: bool = False, check_ori: bool = True):
    """Target view (keypoints, descriptors, uright, blocked) + queries + params for one mode."""
    rng = np.random.default_rng(seed)
    if dense:
        n_target = max(8, n_target // 6)
    k = np.zeros(n_target, KP_DTYPE)
    k["x"] = rng.uniform(-4, W + 4, n_target).astype(np.float32)        # a few fall outside the grid
    k["y"] = rng.uniform(-4, H + 4, n_target).astype(np.float32)
    k["octave"] = np.minimum(rng.geometric(0.45, n_target) - 1, 7)
    k["angle"] = rng.uniform(0, 360, n_target).astype(np.float32)
    k["size"] = 31 * SCALE[k["octave"]]
    k["response"] = rng.integers(7, 120, n_target)
    k["class_id"] = -1
    if dense:   # many keypoints in a few places -> many queries per window
        c = rng.integers(0, 6, n_target)
        k["x"] = (W * (0.15 + 0.14 * c) + rng.normal(0, 6, n_target)).astype(np.float32)
        k["y"] = (H * 0.5 + rng.normal(0, 6, n_target)).astype(np.float32)
    desc = rng.integers(0, 256, (n_target, 32), dtype=np.uint8)
    uright = np.where(rng.random(n_target) < 0.5, k["x"] - rng.uniform(0, 40, n_target), -1).astype(np.float32)
    uright[rng.random(n_target) < 0.05] = 0.0                            # uright == 0: neither > 0 nor < 0
    blocked = (rng.random(n_target) < 0.15).astype(np.uint8)

    q = np.zeros(n_query, PROJ_QUERY_DTYPE)
    qd = rng.integers(0, 256, (n_query, 32), dtype=np.uint8)
    tgt = rng.integers(0, n_target, n_query)
    true = rng.random(n_query) < (0.9 if dense else 0.7)
    lvl = np.where(true, k["octave"][tgt], rng.integers(0, 8, n_query)).astype(np.int32)
    lvl = np.clip(lvl + rng.integers(-1, 2, n_query) * (rng.random(n_query) < 0.2), 0, 7).astype(np.int32)
    q["x"] = np.where(true, k["x"][tgt] + rng.normal(0, 2, n_query), rng.uniform(0, W, n_query)).astype(np.float32)
    q["y"] = np.where(true, k["y"][tgt] + rng.normal(0, 2, n_query), rng.uniform(0, H, n_query)).astype(np.float32)
    flips = (rng.random((n_query, 32)) < 0.03) * rng.integers(1, 256, (n_query, 32))
    qd = np.where(true[:, None], desc[tgt] ^ flips.astype(np.uint8), qd).astype(np.uint8)
    dup = rng.random(n_query) < 0.1                                      # exact duplicates -> ties
    qd[dup] = desc[tgt[dup]]
    q["angle"] = np.where(rng.random(n_query) < 0.8, k["angle"][tgt] + rng.normal(0, 4, n_query),
                          rng.uniform(0, 360, n_query)).astype(np.float32) % np.float32(360)
    q["ur"] = np.where(uright[tgt] > 0, uright[tgt] + rng.normal(0, 1.5, n_query), q["x"] - 10).astype(np.float32)
    q["ur_tol"] = -1
    q["level"] = lvl
    flags = np.where(rng.random(n_query) < 0.08, QF_SKIP, 0) | np.where(rng.random(n_query) < 0.8, QF_BLOCKS, 0)
    th = {PROJ_MAPPOINTS: 4.0, PROJ_LASTFRAME: 7.0, PROJ_KEYFRAME: 10.0, PROJ_SIM3: 10.0, PROJ_FUSE: 3.0,
          PROJ_BEST: 7.5, PROJ_INIT: 30.0}[mode]
    q["r"] = (np.float32(th) * SCALE[lvl]).astype(np.float32)
    q["min_level"], q["max_level"] = lvl - 1, lvl
    if mode == PROJ_MAPPOINTS:
        q["ur_tol"] = q["r"]
    elif mode == PROJ_LASTFRAME:
        kind = rng.integers(0, 3, n_query)           # :1387-1392 forward / backward / both
        q["min_level"] = np.where(kind == 0, lvl, np.where(kind == 1, 0, lvl - 1))
        q["max_level"] = np.where(kind == 0, -1, np.where(kind == 1, lvl, lvl + 1))
        q["ur_tol"] = q["r"]
    elif mode == PROJ_KEYFRAME:
        q["min_level"], q["max_level"] = lvl - 1, lvl + 1
        flags |= QF_BLOCKS
    elif mode == PROJ_SIM3:
        flags |= QF_BLOCKS
    elif mode == PROJ_INIT:
        q["min_level"], q["max_level"] = 0, 0
        q["r"] = np.float32(th)
        flags = np.where(lvl > 0, QF_SKIP, 0)
    q["flags"] = flags
    accept = {PROJ_MAPPOINTS: 100, PROJ_LASTFRAME: 100, PROJ_KEYFRAME: 64, PROJ_SIM3: 50, PROJ_FUSE: 50,
              PROJ_BEST: 100, PROJ_INIT: 50}[mode]
    nnratio = {PROJ_MAPPOINTS: 0.8, PROJ_INIT: 0.9}.get(mode, 0.6)
    params = ProjParams.make(mode, accept, nnratio, check_ori and mode in (PROJ_LASTFRAME, PROJ_KEYFRAME, PROJ_INIT),
                             INV_SIGMA2)
    grid = frame_grid(0.0, 0.0, float(W), float(H))
    return dict(params=params, grid=grid, queries=q, qdesc=qd, kps=k, desc=desc, uright=uright,
                blocked=blocked if mode <= PROJ_SIM3 else None)


# --------------------------------------------------------------------------------------------------
# pure-Python restatement (float32 arithmetic via numpy scalars), small cases only
# --------------------------------------------------------------------------------------------------
f32 = np.float32


def _round_away(v) -> int:                   # std::round: half away from zero
    v = float(v)
    return int(math.floor(v + 0.5)) if v >= 0 else -int(math.floor(-v + 0.5))


def py_grid(kps, g):
    cells = [[] for _ in range(g.cols * g.rows)]
    for i, kp in enumerate(kps):
        px = _round_away(f32(f32(kp["x"]) - f32(g.min_x)) * f32(g.inv_w))
        py = _round_away(f32(f32(kp["y"]) - f32(g.min_y)) * f32(g.inv_h))
        if 0 <= px < g.cols and 0 <= py < g.rows:
            cells[px * g.rows + py].append(i)
    return cells


def py_features_in_area(kps, cells, g, x, y, r, min_level, max_level):
    x, y, r = f32(x), f32(y), f32(r)
    nminx = max(0, int(math.floor(f32(f32(f32(x - f32(g.min_x)) - r) * f32(g.inv_w)))))
    if nminx >= g.cols:
        return []
    nmaxx = min(g.cols - 1, int(math.ceil(f32(f32(f32(x - f32(g.min_x)) + r) * f32(g.inv_w)))))
    if nmaxx < 0:
        return []
    nminy = max(0, int(math.floor(f32(f32(f32(y - f32(g.min_y)) - r) * f32(g.inv_h)))))
    if nminy >= g.rows:
        return []
    nmaxy = min(g.rows - 1, int(math.ceil(f32(f32(f32(y - f32(g.min_y)) + r) * f32(g.inv_h)))))
    if nmaxy < 0:
        return []
    check = min_level > 0 or max_level >= 0
    out = []
    for ix in range(nminx, nmaxx + 1):
        for iy in range(nminy, nmaxy + 1):
            for i in cells[ix * g.rows + iy]:
                kp = kps[i]
                if check:
                    if kp["octave"] < min_level:
                        continue
                    if max_level >= 0 and kp["octave"] > max_level:
                        continue
                if abs(f32(f32(kp["x"]) - x)) < r and abs(f32(f32(kp["y"]) - y)) < r:
                    out.append(i)
    return out


def _ham(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def _rot_bin(a1, a2):
    rot = f32(f32(a1) - f32(a2))
    if rot < 0:
        rot = f32(rot + f32(360))
    b = _round_away(f32(rot * f32(f32(1) / f32(30))))
    return 0 if b == 30 else b


def _three_maxima(h):
    m1 = m2 = m3 = 0
    i1 = i2 = i3 = -1
    for i, s in enumerate(h):
        if s > m1:
            m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, i
        elif s > m2:
            m3, m2, i3, i2 = m2, s, i2, i
        elif s > m3:
            m3, i3 = s, i
    if m2 < f32(0.1) * f32(m1):
        i2 = i3 = -1
    elif m3 < f32(0.1) * f32(m1):
        i3 = -1
    return i1, i2, i3


def py_proj_search(c):
    """The reference's loops (ORBmatcher.cc :45-131, :292-405, :407-522, :894-951, :1053-1081, :1330-1472,
    :1474-1601) on a case from make_case."""
    P, g, Q, qd, k, d = c["params"], c["grid"], c["queries"], c["qdesc"], c["kps"], c["desc"]
    ur, bl = c["uright"], c["blocked"]
    mode = P.mode
    n, nq = len(k), len(Q)
    cells = py_grid(k, g)
    own, own_blocks = [-1] * n, [0] * n
    mdist, m21 = [2 ** 31 - 1] * n, [-1] * n
    q_idx, q_dist = [-1] * nq, [-1] * nq
    rot_mode = P.check_ori and mode in (PROJ_LASTFRAME, PROJ_KEYFRAME, PROJ_INIT)
    rot = []
    nm = 0
    big = 2 ** 31 - 1
    for qi in range(nq):
        q = Q[qi]
        if q["flags"] & QF_SKIP:
            continue
        cand = py_features_in_area(k, cells, g, q["x"], q["y"], q["r"], int(q["min_level"]), int(q["max_level"]))
        if not cand:
            continue
        init = big if mode in (PROJ_INIT, PROJ_BEST) else 256
        bd, bi, bl1, bd2, bl2 = init, -1, -1, init, -1
        for idx in cand:
            kp = k[idx]
            if mode <= PROJ_SIM3:
                if bl is not None and bl[idx]:
                    continue
                if own[idx] >= 0 and own_blocks[idx]:
                    continue
            if mode in (PROJ_MAPPOINTS, PROJ_LASTFRAME) and ur is not None and q["ur_tol"] >= 0 and ur[idx] > 0:
                if abs(f32(f32(q["ur"]) - f32(ur[idx]))) > f32(q["ur_tol"]):
                    continue
            if mode == PROJ_FUSE:
                ex, ey = f32(f32(q["x"]) - f32(kp["x"])), f32(f32(q["y"]) - f32(kp["y"]))
                if ur is not None and ur[idx] >= 0:
                    er = f32(f32(q["ur"]) - f32(ur[idx]))
                    e2 = f32(f32(f32(ex * ex) + f32(ey * ey)) + f32(er * er))
                    if float(f32(e2 * f32(P.inv_sigma2[int(kp["octave"])]))) > 7.8:
                        continue
                else:
                    e2 = f32(f32(ex * ex) + f32(ey * ey))
                    if float(f32(e2 * f32(P.inv_sigma2[int(kp["octave"])]))) > 5.99:
                        continue
            dist = _ham(qd[qi], d[idx])
            if mode == PROJ_INIT and mdist[idx] <= dist:
                continue
            if dist < bd:
                bd2, bl2, bd, bl1, bi = bd, bl1, dist, int(kp["octave"]), idx
            elif dist < bd2:
                bl2, bd2 = int(kp["octave"]), dist
        if bi < 0 or bd > P.accept_max:
            continue
        if mode == PROJ_MAPPOINTS and bl1 == bl2 and f32(bd) > f32(f32(P.nnratio) * f32(bd2)):
            continue
        if mode == PROJ_INIT and not (f32(bd) < f32(f32(bd2) * f32(P.nnratio))):
            continue
        q_idx[qi], q_dist[qi] = bi, bd
        nm += 1
        if mode <= PROJ_SIM3:
            own[bi], own_blocks[bi] = qi, 1 if q["flags"] & QF_BLOCKS else 0
        if mode == PROJ_INIT:
            if m21[bi] >= 0:
                q_idx[m21[bi]] = -1
                nm -= 1
            m21[bi], mdist[bi] = qi, bd
        if rot_mode:
            rot.append((_rot_bin(q["angle"], k[bi]["angle"]), qi if mode == PROJ_INIT else bi))
    if rot_mode:
        hist = [0] * 30
        for b, _ in rot:
            hist[b] += 1
        keep = _three_maxima(hist)
        for b in range(30):
            if b in keep:
                continue
            for bb, e in rot:
                if bb != b:
                    continue
                if mode == PROJ_INIT:
                    if q_idx[e] >= 0:
                        q_idx[e] = -1
                        nm -= 1
                else:
                    own[e] = -2
                    nm -= 1
    if mode > PROJ_SIM3:
        own = [-1] * n
    q_dist = [dd if ii >= 0 else -1 for ii, dd in zip(q_idx, q_dist)]
    return nm, np.array(q_idx, np.int32), np.array(q_dist, np.int32), np.array(own, np.int32)


# ---- the projection step (orbx_proj_project; src/ORBmatcher.cc:1363-1392, Frame.cc:269-325, ORBmatcher.cc:854-893) ----
def make_projection_case(seed: int, n: int = 600, W: int = 1242, H: int = 375):
    """MapPoints around a camera with a small random pose: most project inside the image with distances inside their
    scale-invariance range; some lie behind the camera, outside the image, outside the distance range, or are seen at
    more than 60 degrees from their normal; a few are flagged SKIP / BLOCKS.  Returns (points, view, scale, log_sf) with
    the dtypes of oracle.MAP_POINT_DTYPE / VIEW_DTYPE."""
    from oracle.oracle import MAP_POINT_DTYPE, VIEW_DTYPE
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy, bf = 718.856, 718.856, 607.1928, 185.2157, 386.1448
    yaw, pitch = rng.normal(0, 0.05), rng.normal(0, 0.02)
    cyw, syw, cp, sp = math.cos(yaw), math.sin(yaw), math.cos(pitch), math.sin(pitch)
    Ry = np.array([[cyw, 0, syw], [0, 1, 0], [-syw, 0, cyw]])
    Rx = np.array([[1, 0, 0], [0, cp, -sp], [0, sp, cp]])
    R = (Rx @ Ry).astype(np.float32)
    Ow = rng.normal(0, 0.5, 3).astype(np.float32)
    t = (-(R.astype(np.float64) @ Ow.astype(np.float64))).astype(np.float32)
    # points: pixel + depth in the camera, then to the world
    u = rng.uniform(-60, W + 60, n)
    v = rng.uniform(-30, H + 30, n)
    z = rng.uniform(1.5, 70.0, n)
    z[rng.random(n) < 0.04] *= -1                                       # behind the camera
    Xc = np.stack([(u - cx) * z / fx, (v - cy) * z / fy, z], 1)
    Xw = (R.astype(np.float64).T @ (Xc.T - t.astype(np.float64)[:, None])).T
    p = np.zeros(n, MAP_POINT_DTYPE)
    p["x"], p["y"], p["z"] = Xw[:, 0], Xw[:, 1], Xw[:, 2]
    d = Xw - Ow.astype(np.float64)
    dist = np.linalg.norm(d, axis=1)
    nrm = d / dist[:, None]
    tilt = rng.random(n) < 0.1                                          # seen from > 60 degrees
    nrm[tilt] = np.cross(nrm[tilt], rng.normal(0, 1, (int(tilt.sum()), 3)))
    nrm /= np.linalg.norm(nrm, axis=1)[:, None]
    p["nx"], p["ny"], p["nz"] = nrm[:, 0], nrm[:, 1], nrm[:, 2]
    octave = np.minimum(rng.geometric(0.45, n) - 1, 7)
    # mfMaxDistance = creation distance x scale^octave, mfMinDistance = max / scale^7 (MapPoint::UpdateNormalAndDepth)
    created = dist * rng.uniform(0.7, 1.4, n)
    created[rng.random(n) < 0.08] *= 3.0                                # now outside the invariance range
    p["max_dist"] = (created * SCALE[octave]).astype(np.float32)
    p["min_dist"] = (p["max_dist"] / SCALE[7]).astype(np.float32)
    p["angle"] = rng.uniform(0, 360, n).astype(np.float32)
    p["octave"] = octave
    p["flags"] = np.where(rng.random(n) < 0.05, QF_SKIP, 0) | np.where(rng.random(n) < 0.7, QF_BLOCKS, 0)
    view = np.zeros(1, VIEW_DTYPE)[0]
    view["R"], view["t"], view["Ow"] = R.reshape(9), t, Ow
    view["fx"], view["fy"], view["cx"], view["cy"], view["bf"] = fx, fy, cx, cy, bf
    view["min_x"], view["max_x"], view["min_y"], view["max_y"] = 0.0, W, 0.0, H
    view["th"] = [7.0, 1.0, 3.0, 5.0][seed % 4]
    view["view_cos_limit"] = 0.5
    view["level_mode"] = [1, -1, 0][seed % 3]
    return p, view, SCALE, np.float32(math.log(1.2))


def project_py(mode, points, view, scale, log_sf):
    """Pure-Python restatement of the projection step (numpy float32 scalars: IEEE single, no contraction; float64 for
    the double parts), independent of oracle/proj_oracle.cpp.  Returns PROJ_QUERY_DTYPE queries."""
    f = np.float32
    out = np.zeros(len(points), PROJ_QUERY_DTYPE)
    R, t, Ow = view["R"].astype(np.float32), view["t"].astype(np.float32), view["Ow"].astype(np.float32)
    fx, fy, cx, cy, bf = (f(view[k]) for k in ("fx", "fy", "cx", "cy", "bf"))
    nlev = len(scale)
    for i, p in enumerate(points):
        q = out[i]
        q["min_level"] = q["max_level"] = q["level"] = -1
        q["ur_tol"] = -1
        q["flags"] = QF_SKIP
        if p["flags"] & QF_SKIP:
            continue
        X = (f(p["x"]), f(p["y"]), f(p["z"]))
        c = [R[3 * r] * X[0] + R[3 * r + 1] * X[1] + R[3 * r + 2] * X[2] + t[r] for r in range(3)]
        xc, yc, zc = c
        if mode == PROJ_LASTFRAME:
            invz = f(1.0 / float(zc)) if zc != 0 else f(np.inf)
            if invz < 0:
                continue
            u, v = fx * xc * invz + cx, fy * yc * invz + cy
            if u < view["min_x"] or u > view["max_x"] or v < view["min_y"] or v > view["max_y"]:
                continue
            o = int(p["octave"])
            rad = f(view["th"]) * scale[o]
            q["x"], q["y"], q["r"] = u, v, rad
            lm = int(view["level_mode"])
            q["min_level"], q["max_level"] = (o, -1) if lm > 0 else (0, o) if lm < 0 else (o - 1, o + 1)
            q["ur"], q["ur_tol"], q["angle"], q["level"] = u - bf * invz, rad, p["angle"], o
        else:
            if zc < 0:
                continue
            invz = f(1) / zc
            if mode == PROJ_MAPPOINTS:
                u, v = fx * xc * invz + cx, fy * yc * invz + cy
                if u < view["min_x"] or u > view["max_x"] or v < view["min_y"] or v > view["max_y"]:
                    continue
            else:
                u, v = fx * (xc * invz) + cx, fy * (yc * invz) + cy
                if not (view["min_x"] <= u < view["max_x"] and view["min_y"] <= v < view["max_y"]):
                    continue
            maxD, minD = f(1.2) * f(p["max_dist"]), f(0.8) * f(p["min_dist"])
            PO = [X[k] - Ow[k] for k in range(3)]
            dist = f(math.sqrt(norm2_d(PO)))                       # cv::norm: double squares summed in double
            if dist < minD or dist > maxD:
                continue
            N = (f(p["nx"]), f(p["ny"]), f(p["nz"]))
            dot = 0.0
            for k in range(3):
                dot += float(PO[k]) * float(N[k])                     # Mat::dot: double products
            ratio = f(p["max_dist"]) / dist
            pred = min(max(int(math.ceil(math.log(float(ratio)) / float(log_sf))), 0), nlev - 1)
            if mode == PROJ_MAPPOINTS:
                vc = f(dot / float(dist))
                if vc < f(view["view_cos_limit"]):
                    continue
                r = f(2.5) if float(vc) > 0.998 else f(4.0)
                if f(view["th"]) != f(1):
                    r = r * f(view["th"])
                q["x"], q["y"], q["r"] = u, v, r * scale[pred]
                q["ur"], q["ur_tol"] = u - bf * invz, r * scale[pred]
            else:
                if dot < 0.5 * float(dist):
                    continue
                q["x"], q["y"], q["r"] = u, v, f(view["th"]) * scale[pred]
                q["ur"] = u - bf * invz
            q["min_level"], q["max_level"], q["level"] = pred - 1, pred, pred
        q["flags"] = int(p["flags"]) & ~QF_SKIP
    return out


def norm2_d(v):
    """cv::norm's sum of squares for a 3x1 CV_32F Mat (OpenCV 3.2 normL2Sqr<float, double>): elements widened to double,
    squared and summed left to right in double."""
    s = 0.0
    for x in v:
        s += float(x) * float(x)
    return s


def stereo_frame_case(seed: int, n: int = 700, W: int = 1242, H: int = 375):
    """Keypoints of a stereo frame with depths (a share without depth), its pose Twc (Rwc 9 + Ow 3) and camera."""
    rng = np.random.default_rng(seed)
    k = np.zeros(n, KP_DTYPE)
    k["x"] = rng.uniform(0, W, n).astype(np.float32)
    k["y"] = rng.uniform(0, H, n).astype(np.float32)
    k["octave"] = np.minimum(rng.geometric(0.45, n) - 1, 7)
    k["angle"] = rng.uniform(0, 360, n).astype(np.float32)
    k["size"] = 31 * SCALE[k["octave"]]
    depth = rng.uniform(1.0, 60.0, n).astype(np.float32)
    depth[rng.random(n) < 0.3] = -1.0
    depth[rng.random(n) < 0.02] = 0.0
    a = rng.normal(0, 0.1)
    Rwc = np.array([[math.cos(a), 0, math.sin(a)], [0, 1, 0], [-math.sin(a), 0, math.cos(a)]], np.float32)
    Ow = rng.normal(0, 2.0, 3).astype(np.float32)
    twc = np.concatenate([Rwc.reshape(9), Ow]).astype(np.float32)
    cam = np.array([718.856, 718.856, 607.1928, 185.2157], np.float32)
    return k, depth, twc, cam


def stereo_mappoints_py(k, depth, twc, cam, scale, flags):
    """numpy-float32 restatement of Frame::UnprojectStereo + MapPoint::MapPoint(Pos, pMap, pFrame, idxF)."""
    from oracle.oracle import MAP_POINT_DTYPE
    f = np.float32
    out = np.zeros(len(k), MAP_POINT_DTYPE)
    T = twc.astype(np.float32)
    invfx, invfy = f(1) / f(cam[0]), f(1) / f(cam[1])
    for i in range(len(k)):
        p = out[i]
        p["octave"], p["angle"], p["flags"] = k["octave"][i], k["angle"][i], QF_SKIP
        z = f(depth[i])
        if not z > 0:
            continue
        x = (f(k["x"][i]) - f(cam[2])) * z * invfx
        y = (f(k["y"][i]) - f(cam[3])) * z * invfy
        X = [T[3 * r] * x + T[3 * r + 1] * y + T[3 * r + 2] * z + T[9 + r] for r in range(3)]
        d = [X[r] - T[9 + r] for r in range(3)]
        nrm = math.sqrt(norm2_d(d))
        inv = f(1.0 / nrm)
        p["x"], p["y"], p["z"] = X
        p["nx"], p["ny"], p["nz"] = d[0] * inv, d[1] * inv, d[2] * inv
        p["max_dist"] = f(nrm) * scale[int(k["octave"][i])]
        p["min_dist"] = f(p["max_dist"]) / scale[len(scale) - 1]
        p["flags"] = flags & ~QF_SKIP
    return out
