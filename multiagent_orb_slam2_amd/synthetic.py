"""Seeded synthetic inputs for the ORB front-end and the Hamming matchers.

The reference's datasets (KITTI / EuRoC) and its DBoW2 vocabulary are absent in this image
(SURVEY.md §4, §8d), so every test and the bench use these generators.  Images follow SURVEY §8d:
a smooth gradient background, a few hundred random axis-aligned rectangles and disks, Gaussian
noise (sigma 4), clipped to uint8 — FAST-rich but structured texture.
"""
from __future__ import annotations

import numpy as np


def kitti_like_image(seed: int, rows: int = 375, cols: int = 1242, n_shapes: int | None = None,
                     noise: float = 4.0) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    yy, xx = np.mgrid[0:rows, 0:cols].astype(np.float32)
    g0, gx, gy = rng.uniform(40, 200), rng.uniform(-0.08, 0.08), rng.uniform(-0.2, 0.2)
    img = g0 + gx * xx + gy * yy
    if n_shapes is None:
        n_shapes = int(rng.integers(200, 401))
    for _ in range(n_shapes):
        val = rng.uniform(0, 255)
        if rng.random() < 0.5:
            w, h = rng.integers(4, 80), rng.integers(4, 60)
            x0, y0 = rng.integers(-20, cols), rng.integers(-20, rows)
            img[max(y0, 0):max(y0 + h, 0), max(x0, 0):max(x0 + w, 0)] = val
        else:
            r = rng.uniform(3, 40)
            cx, cy = rng.uniform(0, cols), rng.uniform(0, rows)
            x0, x1 = int(max(cx - r, 0)), int(min(cx + r + 1, cols))
            y0, y1 = int(max(cy - r, 0)), int(min(cy + r + 1, rows))
            if x1 <= x0 or y1 <= y0:
                continue
            sub_y, sub_x = yy[y0:y1, x0:x1], xx[y0:y1, x0:x1]
            m = (sub_x - cx) ** 2 + (sub_y - cy) ** 2 <= r * r
            img[y0:y1, x0:x1][m] = val
    img = img + rng.normal(0.0, noise, size=img.shape).astype(np.float32)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def shifted_right_view(left: np.ndarray, seed: int, max_disp: int = 64) -> np.ndarray:
    """Right image of a synthetic rectified stereo pair: each row block of the left image shifted
    left by a smooth seeded disparity (0..max_disp px), plus fresh noise — gives the stereo matcher
    real row/octave structure."""
    rng = np.random.Generator(np.random.PCG64(seed + 7919))
    rows, cols = left.shape
    base = rng.uniform(0, max_disp)
    slope = rng.uniform(-0.05, 0.05)
    out = np.empty_like(left)
    for y in range(rows):
        d = int(np.clip(round(base + slope * y), 0, max_disp))
        out[y, : cols - d] = left[y, d:]
        out[y, cols - d:] = left[y, -1]
    noise = rng.normal(0.0, 2.0, size=left.shape)
    return np.clip(np.rint(out.astype(np.float32) + noise), 0, 255).astype(np.uint8)


def uniform_noise_image(seed: int, rows: int = 375, cols: int = 1242) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.integers(0, 256, size=(rows, cols), dtype=np.uint8)


def random_descriptors(seed: int, n: int) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.integers(0, 256, size=(n, 32), dtype=np.uint8)


def planted_pairs(seed: int, n_query: int = 2000, n_train: int = 2000, frac: float = 0.3,
                  flip_p: float = 0.05):
    """C3 pure-random variant: iid Bernoulli(1/2) descriptors, a fraction of train rows planted as
    query rows with Binomial(256, flip_p) bit flips."""
    rng = np.random.Generator(np.random.PCG64(seed))
    q = rng.integers(0, 256, size=(n_query, 32), dtype=np.uint8)
    t = rng.integers(0, 256, size=(n_train, 32), dtype=np.uint8)
    k = min(int(frac * n_train), n_query)
    src = rng.choice(n_query, size=k, replace=False)
    dst = rng.choice(n_train, size=k, replace=False)
    bits = np.unpackbits(q[src], axis=1)
    flips = rng.random(bits.shape) < flip_p
    t[dst] = np.packbits(bits ^ flips, axis=1)
    return q, t


def random_featvec(seed: int, n: int, n_nodes: int = 60, node_space: int = 100):
    """Synthetic DBoW2 FeatureVector (level-2 node -> ascending feature indices) as CSR.

    The vocabulary is absent, so node ids are drawn from a small id space so that two
    keyframes share most nodes, like two views of the same place."""
    rng = np.random.Generator(np.random.PCG64(seed))
    ids = np.sort(rng.choice(node_space, size=min(n_nodes, node_space), replace=False)).astype(np.uint32)
    assign = rng.integers(0, len(ids), size=n)
    order = np.argsort(assign, kind="stable")
    counts = np.bincount(assign, minlength=len(ids))
    keep = counts > 0
    offs = np.concatenate([[0], np.cumsum(counts[keep])]).astype(np.int32)
    return ids[keep], offs, order.astype(np.int32)


def synthetic_vocabulary(seed: int, k: int = 10, L: int = 4, flip_p: float = 0.12, stop_frac: float = 0.02,
                         scoring: int = 0, weighting: int = 0):
    """A DBoW2-style k-ary vocabulary tree of depth L (ORBvoc.txt itself is absent).

    Children descriptors are their parent's with Bernoulli(flip_p) bit flips, so descending the tree
    is meaningful for ORB descriptors; leaves get idf-like weights log(N/n_i) with a few stopped (0)
    words.  Returns the node lines in loadFromTextFile order (node id = line + 1, root = 0):
    dict(k, L, scoring, weighting, parent, is_leaf, desc, weight)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    flip_t = int(round(flip_p * 256))                      # bit flips with probability flip_t/256
    f_ids = np.zeros(1, np.int64)
    f_bits = np.unpackbits(rng.integers(0, 256, (1, 32), dtype=np.uint8), axis=1)
    parent, leaf, desc, weight = [], [], [], []
    next_id = 1
    for depth in range(L):                                 # breadth first: the order saveToTextFile writes
        n = len(f_ids) * k
        par = np.repeat(f_ids, k)
        bits = np.repeat(f_bits, k, axis=0)
        for c0 in range(0, n, 1 << 16):                     # chunked: L=6 has 10^6 leaves
            c1 = min(n, c0 + (1 << 16))
            bits[c0:c1] ^= (rng.integers(0, 256, (c1 - c0, 256), dtype=np.uint8) < flip_t).astype(np.uint8)
        is_leaf = depth + 1 == L
        parent.append(par.astype(np.int32))
        leaf.append(np.full(n, 1 if is_leaf else 0, np.uint8))
        desc.append(np.packbits(bits, axis=1))
        if is_leaf:
            stop = rng.random(n) < stop_frac
            w = np.log(1e6 / rng.integers(1, 5000, n).astype(np.float64))
            weight.append(np.where(stop, 0.0, w))
        else:
            weight.append(np.zeros(n))
        f_ids = next_id + np.arange(n, dtype=np.int64)
        f_bits = bits
        next_id += n
    return dict(k=k, L=L, scoring=scoring, weighting=weighting, parent=np.concatenate(parent),
                is_leaf=np.concatenate(leaf), desc=np.concatenate(desc).astype(np.uint8),
                weight=np.concatenate(weight).astype(np.float64))


def write_vocabulary_text(voc, path: str):
    """DBoW2 text format (TemplatedVocabulary::saveToTextFile): header 'k L scoring weighting', then
    'parent isLeaf d0 .. d31 weight' per node (no trailing newline)."""
    lines = [f"{voc['k']} {voc['L']} {voc['scoring']} {voc['weighting']}"]
    for p, lf, d, w in zip(voc["parent"], voc["is_leaf"], voc["desc"], voc["weight"]):
        lines.append(f"{int(p)} {int(lf)} " + " ".join(str(int(x)) for x in d) + " " + repr(float(w)))
    with open(path, "w") as f:
        f.write("\n".join(lines))
