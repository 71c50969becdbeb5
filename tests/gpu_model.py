"""numpy model of the data-parallel formulations used by the HIP kernels (test-only).

The HIP extractor does not run the reference's sequential loops; it uses two reformulations that are
checked here, on the CPU, against the oracle's line-by-line restatement:

* FAST (k_fast_cells): threshold-independent closed-form score s = max(m_dark, m_bright) - 1 plus a
  per-cell masked strict 3x3 NMS, instead of OpenCV's FAST_t loop + cornerScore<16> per threshold.
* DistributeOctTree (k_quadtree): list positions computed with prefix sums per pass instead of a
  std::list with push_front/erase.
"""
from __future__ import annotations

import math

import numpy as np

CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
          (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def score_map(img: np.ndarray) -> np.ndarray:
    """s = max(m_dark, m_bright) - 1 for every pixel at least 3 px from the border (else -1000)."""
    h, w = img.shape
    I = img.astype(np.int32)
    v = I[3:h - 3, 3:w - 3]
    d = np.stack([v - I[3 + dy:h - 3 + dy, 3 + dx:w - 3 + dx] for dx, dy in CIRCLE])   # (16, h-6, w-6)
    dd = np.concatenate([d, d[:9]], axis=0)
    mins = np.stack([dd[k:k + 9].min(axis=0) for k in range(16)])
    maxs = np.stack([dd[k:k + 9].max(axis=0) for k in range(16)])
    s = np.maximum(mins.max(axis=0), -maxs.min(axis=0)) - 1
    out = np.full((h, w), -1000, np.int32)
    out[3:h - 3, 3:w - 3] = s
    return out


def pretest_map(img: np.ndarray, t: int) -> np.ndarray:
    """k_fast_cells' compass pre-test: True where max over compass pairs (0,4),(4,8),(8,12),(12,0) of
    min(d_k, d_k+4) > t, or min of max < -t (a necessary condition for 'corner at t')."""
    h, w = img.shape
    I = img.astype(np.int32)
    v = I[3:h - 3, 3:w - 3]
    d = [v - I[3 + dy:h - 3 + dy, 3 + dx:w - 3 + dx] for dx, dy in (CIRCLE[0], CIRCLE[4], CIRCLE[8], CIRCLE[12])]
    dk = np.max([np.minimum(d[k], d[(k + 1) % 4]) for k in range(4)], axis=0)
    br = np.min([np.maximum(d[k], d[(k + 1) % 4]) for k in range(4)], axis=0)
    out = np.zeros((h, w), bool)
    out[3:h - 3, 3:w - 3] = np.maximum(dk, -br) > t
    return out


def cells_of_level(h: int, w: int):
    """ComputeKeyPointsOctTree cell grid (src/ORBextractor.cc:773-807): list of (x0, y0, x1, y1, i, j)."""
    minB, maxBX, maxBY = 16, w - 16, h - 16
    width, height = np.float32(maxBX - minB), np.float32(maxBY - minB)
    nCols, nRows = int(width / np.float32(30)), int(height / np.float32(30))
    if nCols <= 0 or nRows <= 0:
        return [], 0, 0
    wCell, hCell = int(math.ceil(width / nCols)), int(math.ceil(height / nRows))
    cells = []
    for i in range(nRows):
        iniY = minB + i * hCell
        maxY = iniY + hCell + 6
        if iniY >= maxBY - 3:
            continue
        maxY = min(maxY, maxBY)
        for j in range(nCols):
            iniX = minB + j * wCell
            maxX = iniX + wCell + 6
            if iniX >= maxBX - 6:
                continue
            maxX = min(maxX, maxBX)
            cells.append((iniX, iniY, maxX, maxY, i, j))
    return cells, wCell, hCell


def fast_candidates(level: np.ndarray, ini_th=20, min_th=7):
    """Candidates of one level in reference order, window-relative (x, y, response)."""
    h, w = level.shape
    cells, wCell, hCell = cells_of_level(h, w)
    out = []
    for (x0, y0, x1, y1, i, j) in cells:
        roi = level[y0:y1, x0:x1]
        H, W = roi.shape
        det = np.zeros((H, W), bool)
        det[3:H - 3, 3:W - 3] = True
        T1, T2 = max(min(max(ini_th, 0), 255), 1), max(min(max(min_th, 0), 255), 1)
        # kernel form: exact scores only where the compass pre-test at min(T1, T2) passes, 0 elsewhere;
        # NMS against the raw 8 neighbours (-1 outside the detection window)
        s = np.where(pretest_map(roi, min(T1, T2)), score_map(roi), 0)
        s = np.where(det, s, -1)
        for t in (T1, T2):
            pad = np.pad(s, 1, constant_values=-1)
            keep = det & (s >= t)
            for dy in (-1, 0, 1):
                for dx in (-1, 0, 1):
                    if dy == 0 and dx == 0:
                        continue
                    keep &= s > pad[1 + dy:1 + dy + H, 1 + dx:1 + dx + W]
            if keep.any():
                break
        ys, xs = np.nonzero(keep)   # row-major
        for y, x in zip(ys, xs):
            out.append((x0 + x - 16, y0 + y - 16, float(s[y, x])))
    return np.array(out, np.float32).reshape(-1, 3)


def _half(a: int) -> int:
    return int(math.ceil(np.float32(a) / np.float32(2)))


def distribute_parallel(xyr: np.ndarray, win_w: int, win_h: int, N: int):
    """Prefix-sum formulation of DistributeOctTree (what k_quadtree computes)."""
    K = len(xyr)
    kx = xyr[:, 0].astype(np.int64)
    ky = xyr[:, 1].astype(np.int64)
    nIni = int(round(float(np.float32(win_w) / np.float32(win_h))))
    hX = np.float32(win_w) / np.float32(nIni)
    # nodes: list of dicts in list order
    rect = [(int(np.float32(hX) * np.float32(i)), int(np.float32(hX) * np.float32(i + 1)), 0, win_h)
            for i in range(nIni)]
    node = np.array([min(int(np.float32(x) / hX), nIni - 1) for x in kx], np.int64) if K else np.zeros(0, np.int64)
    cnt = np.bincount(node, minlength=nIni) if K else np.zeros(nIni, np.int64)
    keep = [i for i in range(nIni) if cnt[i] > 0]
    remap = {o: n for n, o in enumerate(keep)}
    node = np.array([remap[o] for o in node], np.int64)
    nodes = [dict(r=rect[o], cnt=int(cnt[o]), seq=o) for o in keep]

    def quad(k, r):
        x0, x1, y0, y1 = r
        mx, my = x0 + _half(x1 - x0), y0 + _half(y1 - y0)
        return (0 if kx[k] < mx else 1) + (0 if ky[k] < my else 2)

    def child_rect(r, q):
        x0, x1, y0, y1 = r
        mx, my = x0 + _half(x1 - x0), y0 + _half(y1 - y0)
        return ((mx if q & 1 else x0), (x1 if q & 1 else mx), (my if q & 2 else y0), (y1 if q & 2 else my))

    phase2 = False
    while True:
        n, prev = len(nodes), len(nodes)
        cc = np.zeros((n, 4), np.int64)
        for k in range(K):
            i = node[k]
            if nodes[i]["cnt"] > 1:
                cc[i, quad(k, nodes[i]["r"])] += 1
        if not phase2:
            split = [nd["cnt"] > 1 for nd in nodes]
            nch = np.array([(cc[i] > 0).sum() if split[i] else 0 for i in range(n)], np.int64)
            chpre = np.concatenate([[0], np.cumsum(nch)])[:-1]
            C = int(nch.sum())
            surv = np.array([0 if s else 1 for s in split], np.int64)
            upre = np.concatenate([[0], np.cumsum(surv)])[:-1]
            nexp = sum(int((cc[i] > 1).sum()) for i in range(n) if split[i])
            new = [None] * (C + int(surv.sum()))
            base = np.zeros(n, np.int64)
            for i in range(n):
                if split[i]:
                    gb = C - chpre[i] - nch[i]
                    base[i] = gb
                    for q in range(4):
                        if cc[i, q] == 0:
                            continue
                        p = gb + sum(1 for qq in range(q + 1, 4) if cc[i, qq] > 0)
                        new[p] = dict(r=child_rect(nodes[i]["r"], q), cnt=int(cc[i, q]),
                                      seq=int(chpre[i]) + sum(1 for qq in range(q) if cc[i, qq] > 0))
                else:
                    base[i] = C + upre[i]
                    new[base[i]] = nodes[i]
            for k in range(K):
                i = node[k]
                if split[i]:
                    q = quad(k, nodes[i]["r"])
                    node[k] = base[i] + sum(1 for qq in range(q + 1, 4) if cc[i, qq] > 0)
                else:
                    node[k] = base[i]
            nodes = new
            if len(nodes) >= N or len(nodes) == prev:
                break
            if len(nodes) + 3 * nexp > N:
                phase2 = True
        else:
            V = sorted([i for i in range(n) if nodes[i]["cnt"] > 1],
                       key=lambda i: (nodes[i]["cnt"], nodes[i]["seq"], i))
            order = V[::-1]
            nchs = [int((cc[i] > 0).sum()) for i in order]
            size, nproc = n, len(order)
            for p, c in enumerate(nchs):
                size += c - 1
                if size >= N:
                    nproc = p + 1
                    break
            CH = np.concatenate([[0], np.cumsum(nchs[:nproc])]).astype(np.int64)
            Cn = int(CH[-1])
            base = {}
            cre = {}
            for p in range(nproc):
                i = order[p]
                base[i] = Cn - CH[p] - nchs[p]
                cre[i] = CH[p]
            rest = [i for i in range(n) if i not in base]
            new = [None] * (Cn + len(rest))
            for i, gb in base.items():
                for q in range(4):
                    if cc[i, q] == 0:
                        continue
                    p = gb + sum(1 for qq in range(q + 1, 4) if cc[i, qq] > 0)
                    new[p] = dict(r=child_rect(nodes[i]["r"], q), cnt=int(cc[i, q]),
                                  seq=int(cre[i]) + sum(1 for qq in range(q) if cc[i, qq] > 0))
            rpos = {}
            for r, i in enumerate(rest):
                rpos[i] = Cn + r
                new[Cn + r] = nodes[i]
            for k in range(K):
                i = node[k]
                if i in base:
                    q = quad(k, nodes[i]["r"])
                    node[k] = base[i] + sum(1 for qq in range(q + 1, 4) if cc[i, qq] > 0)
                else:
                    node[k] = rpos[i]
            nodes = new
            if len(nodes) >= N or len(nodes) == prev:
                break
    best = {}
    for k in range(K):
        i = node[k]
        key = (xyr[k, 2], -k)
        if i not in best or key > best[i]:
            best[i] = key
    out = [xyr[-best[i][1]] for i in range(len(nodes))]
    return np.array(out, np.float32).reshape(-1, 3)
