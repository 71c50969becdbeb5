"""ctypes wrapper of the CPU oracle (oracle/orb_oracle.cpp).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, never by the product package.  Parity status: "parity unpinned" (see orb_oracle.cpp header and
DESIGN.md §Oracle).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liborb_oracle.so")

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _lib.orc_fast_atan2.restype = C.c_float
        _lib.orc_fast_atan2.argtypes = [C.c_float, C.c_float]
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class FV(C.Structure):
    _fields_ = [("node", C.c_void_p), ("off", C.c_void_p), ("n_nodes", C.c_int), ("idx", C.c_void_p)]


def make_fv(fv):
    node, off, idx = (np.ascontiguousarray(fv[0], np.uint32), np.ascontiguousarray(fv[1], np.int32),
                      np.ascontiguousarray(fv[2], np.int32))
    s = FV(_p(node), _p(off), len(node), _p(idx))
    s._keep = (node, off, idx)
    return s


def tables(nfeatures=2000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7):
    f = lambda: np.zeros(nlevels, np.float32)
    scale, inv, s2, is2 = f(), f(), f(), f()
    npl = np.zeros(nlevels, np.int32)
    umax = np.zeros(16, np.int32)
    lib().orc_tables(nfeatures, C.c_float(scale_factor), nlevels, ini_th, min_th, _p(scale), _p(inv), _p(s2),
                     _p(is2), _p(npl), _p(umax))
    return dict(scale=scale, inv_scale=inv, sigma2=s2, inv_sigma2=is2, n_per_level=npl, umax=umax)


def level_sizes(rows, cols, nlevels=8, scale_factor=1.2):
    inv = tables(nlevels=nlevels, scale_factor=scale_factor)["inv_scale"]
    out = []
    for l in range(nlevels):
        w = int(np.rint(np.float32(cols) * inv[l]))
        h = int(np.rint(np.float32(rows) * inv[l]))
        out.append((h, w))
    return out


def extract(img, nfeatures=2000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7, want_pyramid=False):
    img = np.ascontiguousarray(img, np.uint8)
    rows, cols = img.shape
    cap = 4 * nfeatures + 64 * nlevels
    kps = np.zeros(cap, KP_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    sizes = level_sizes(rows, cols, nlevels, scale_factor)
    pyr = np.zeros(sum(h * w for h, w in sizes), np.uint8) if want_pyramid else None
    ncand = np.zeros(nlevels, np.int32)
    n = lib().orc_extract(nfeatures, C.c_float(scale_factor), nlevels, ini_th, min_th, _p(img), rows, cols, cols,
                          _p(kps), _p(desc), cap, _p(pyr) if pyr is not None else None, _p(ncand))
    if n < 0:
        raise RuntimeError("oracle capacity too small: %d" % -n)
    out = dict(kps=kps[:n].copy(), desc=desc[:n].copy(), ncand=ncand)
    if want_pyramid:
        levels, o = [], 0
        for h, w in sizes:
            levels.append(pyr[o:o + h * w].reshape(h, w).copy())
            o += h * w
        out["pyramid"] = levels
    return out


def resize(src, dh, dw):
    src = np.ascontiguousarray(src, np.uint8)
    dst = np.zeros((dh, dw), np.uint8)
    lib().orc_resize(_p(src), src.shape[1], src.shape[0], _p(dst), dw, dh)
    return dst


def blur7(src):
    src = np.ascontiguousarray(src, np.uint8)
    dst = np.zeros_like(src)
    lib().orc_blur7(_p(src), src.shape[1], src.shape[0], _p(dst))
    return dst


def fast_atan2(y, x):
    return lib().orc_fast_atan2(float(y), float(x))


def descriptor_distance(a, b):
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    return lib().orc_descriptor_distance(_p(a), _p(b))


def bf_match(q, t):
    q = np.ascontiguousarray(q, np.uint8)
    t = np.ascontiguousarray(t, np.uint8)
    nq = q.shape[0]
    bi, b1, b2 = (np.zeros(nq, np.int32) for _ in range(3))
    lib().orc_bf_match(_p(q), nq, _p(t), t.shape[0], _p(bi), _p(b1), _p(b2))
    return bi, b1, b2


def distinctive_descriptors_flat(flat, off):
    """distinctive_descriptors over a flat (total, 32) descriptor array and (M+1,) list offsets."""
    flat = np.ascontiguousarray(flat, np.uint8).reshape(-1, 32)
    off = np.ascontiguousarray(off, np.int32)
    if not len(flat):
        flat = np.zeros((1, 32), np.uint8)
    best = np.zeros(max(len(off) - 1, 1), np.int32)
    lib().orc_distinctive(_p(flat), _p(off), len(off) - 1, _p(best))
    return best[:len(off) - 1]


def distinctive_descriptors(lists):
    """MapPoint::ComputeDistinctiveDescriptors restated (oracle/orb_oracle.cpp orc_distinctive): best index per
    descriptor list (-1 for an empty list)."""
    lists = [np.ascontiguousarray(d, np.uint8).reshape(-1, 32) for d in lists]
    off = np.zeros(len(lists) + 1, np.int32)
    off[1:] = np.cumsum([len(d) for d in lists])
    flat = np.ascontiguousarray(np.concatenate(lists) if off[-1] else np.zeros((1, 32), np.uint8))
    best = np.zeros(max(len(lists), 1), np.int32)
    lib().orc_distinctive(_p(flat), _p(off), len(lists), _p(best))
    return best[:len(lists)]


def stereo_match(kl, dl, kr, dr, scale, rows, bf, b):
    kl, kr = np.ascontiguousarray(kl, KP_DTYPE), np.ascontiguousarray(kr, KP_DTYPE)
    dl, dr = np.ascontiguousarray(dl, np.uint8), np.ascontiguousarray(dr, np.uint8)
    scale = np.ascontiguousarray(scale, np.float32)
    idx = np.zeros(len(kl), np.int32)
    dist = np.zeros(len(kl), np.int32)
    n = lib().orc_stereo_match(_p(kl), _p(dl), len(kl), _p(kr), _p(dr), len(kr), _p(scale), rows,
                               C.c_float(bf), C.c_float(b), _p(idx), _p(dist))
    return n, idx, dist


def stereo_refine(kl, kr, best_idx, scale, inv_scale, pyr_l, pyr_r, bf, b):
    """Frame.cc:554-639 (SAD window, parabola, median rejection) -> (n, uright, depth, sad)."""
    kl, kr = np.ascontiguousarray(kl, KP_DTYPE), np.ascontiguousarray(kr, KP_DTYPE)
    bi = np.ascontiguousarray(best_idx, np.int32)
    scale, inv_scale = np.ascontiguousarray(scale, np.float32), np.ascontiguousarray(inv_scale, np.float32)
    n = len(kl)
    ur, dp, sad = np.zeros(n, np.float32), np.zeros(n, np.float32), np.zeros(n, np.int32)

    def lv(pyr):
        pyr = [np.ascontiguousarray(x, np.uint8) for x in pyr]
        ptrs = (C.c_void_p * len(pyr))(*[x.ctypes.data for x in pyr])
        step = np.array([x.strides[0] for x in pyr], np.int32)
        rows = np.array([x.shape[0] for x in pyr], np.int32)
        cols = np.array([x.shape[1] for x in pyr], np.int32)
        return pyr, ptrs, step, rows, cols

    L, R = lv(pyr_l), lv(pyr_r)
    k = lib().orc_stereo_refine(_p(kl), n, _p(kr), _p(bi), _p(scale), _p(inv_scale), L[1], _p(L[2]), _p(L[3]), _p(L[4]),
                                R[1], _p(R[2]), _p(R[3]), _p(R[4]), C.c_float(bf), C.c_float(b), _p(ur), _p(dp), _p(sad))
    return k, ur, dp, sad


def compute_stereo_matches(left, right, scale, inv_scale, rows, bf, b):
    """Frame::ComputeStereoMatches (src/Frame.cc:466-639) on two oracle extractions made with
    want_pyramid=True -> (uright, depth)."""
    _, bi, _ = stereo_match(left["kps"], left["desc"], right["kps"], right["desc"], scale, rows, bf, b)
    _, ur, dp, _ = stereo_refine(left["kps"], right["kps"], bi, scale, inv_scale, left["pyramid"], right["pyramid"], bf, b)
    return ur, dp


def search_by_bow_kfkf(d1, ang1, valid1, fv1, d2, ang2, valid2, fv2, nnratio=0.75, check_ori=True):
    d1, d2 = np.ascontiguousarray(d1, np.uint8), np.ascontiguousarray(d2, np.uint8)
    ang1, ang2 = np.ascontiguousarray(ang1, np.float32), np.ascontiguousarray(ang2, np.float32)
    v1, v2 = np.ascontiguousarray(valid1, np.uint8), np.ascontiguousarray(valid2, np.uint8)
    m = np.zeros(len(d1), np.int32)
    f1, f2 = make_fv(fv1), make_fv(fv2)
    n = lib().orc_search_by_bow_kfkf(_p(d1), _p(ang1), _p(v1), len(d1), f1, _p(d2), _p(ang2), _p(v2), len(d2), f2,
                                     C.c_float(nnratio), int(check_ori), _p(m))
    return n, m


def search_by_bow_kff(dk, angk, validk, fvk, df, angf, fvf, nnratio=0.7, check_ori=True):
    dk, df = np.ascontiguousarray(dk, np.uint8), np.ascontiguousarray(df, np.uint8)
    angk, angf = np.ascontiguousarray(angk, np.float32), np.ascontiguousarray(angf, np.float32)
    vk = np.ascontiguousarray(validk, np.uint8)
    m = np.zeros(len(df), np.int32)
    fk, ff = make_fv(fvk), make_fv(fvf)
    n = lib().orc_search_by_bow_kff(_p(dk), _p(angk), _p(vk), len(dk), fk, _p(df), _p(angf), len(df), ff,
                                    C.c_float(nnratio), int(check_ori), _p(m))
    return n, m


def search_for_triangulation(d1, k1, mp1, ur1, fv1, d2, k2, mp2, ur2, fv2, F12, sigma2, scale2, ex, ey,
                             only_stereo=False, check_ori=True):
    a = [np.ascontiguousarray(x, t) for x, t in
         ((d1, np.uint8), (k1, KP_DTYPE), (mp1, np.uint8), (ur1, np.float32), (d2, np.uint8), (k2, KP_DTYPE),
          (mp2, np.uint8), (ur2, np.float32), (F12, np.float32), (sigma2, np.float32), (scale2, np.float32))]
    d1, k1, mp1, ur1, d2, k2, mp2, ur2, F12, sigma2, scale2 = a
    m = np.zeros(len(d1), np.int32)
    f1, f2 = make_fv(fv1), make_fv(fv2)
    n = lib().orc_search_for_triangulation(_p(d1), _p(k1), _p(mp1), _p(ur1), len(d1), f1, _p(d2), _p(k2), _p(mp2),
                                           _p(ur2), len(d2), f2, _p(F12), _p(sigma2), _p(scale2), C.c_float(ex),
                                           C.c_float(ey), int(only_stereo), int(check_ori), _p(m))
    return n, m


def level_candidates(img, nfeatures=2000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7):
    """FAST candidates per level in reference order, window-relative (x, y, response)."""
    img = np.ascontiguousarray(img, np.uint8)
    cap = img.size
    xyr = np.zeros((cap, 3), np.float32)
    per = np.zeros(nlevels, np.int32)
    n = lib().orc_level_candidates(nfeatures, C.c_float(scale_factor), nlevels, ini_th, min_th, _p(img),
                                   img.shape[0], img.shape[1], _p(xyr), cap, _p(per))
    if n < 0:
        raise RuntimeError("capacity")
    out, o = [], 0
    for c in per:
        out.append(xyr[o:o + c].copy())
        o += c
    return out


def distribute(xyr, minX, maxX, minY, maxY, N):
    xyr = np.ascontiguousarray(xyr, np.float32).reshape(-1, 3)
    cap = max(4 * len(xyr) + 64, 64)
    out = np.zeros((cap, 3), np.float32)
    m = lib().orc_distribute(_p(xyr), len(xyr), minX, maxX, minY, maxY, N, _p(out), cap)
    if m < 0:
        raise RuntimeError("capacity")
    return out[:m].copy()


class Vocabulary:
    """Oracle vocabulary built once (for timing many transforms: bench.py's cpu_baseline)."""

    def __init__(self, voc):
        self._arrs = [np.ascontiguousarray(voc["parent"], np.int32), np.ascontiguousarray(voc["is_leaf"], np.uint8),
                      np.ascontiguousarray(voc["desc"], np.uint8), np.ascontiguousarray(voc["weight"], np.float64)]
        P, lf, D, W = self._arrs
        lib().orc_vocab_new.restype = C.c_void_p
        self._h = C.c_void_p(lib().orc_vocab_new(voc["L"], voc["scoring"], voc["weighting"], len(P), _p(P), _p(lf),
                                                 _p(D), _p(W)))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_vocab_free(self._h)
            self._h = None

    def transform(self, feats, levelsup):
        feats = np.ascontiguousarray(feats, np.uint8)
        n = len(feats)
        bw, bv = np.zeros(max(n, 1), np.uint32), np.zeros(max(n, 1), np.float64)
        fn, fo, fi = np.zeros(max(n, 1), np.uint32), np.zeros(n + 1, np.int32), np.zeros(max(n, 1), np.int32)
        nw, nf = C.c_int(), C.c_int()
        lib().orc_vocab_apply(self._h, _p(feats), n, levelsup, _p(bw), _p(bv), C.byref(nw), _p(fn), _p(fo), _p(fi),
                              C.byref(nf))
        return dict(bow_words=bw[:nw.value].copy(), bow_values=bv[:nw.value].copy(), fv_nodes=fn[:nf.value].copy(),
                    fv_offsets=fo[:nf.value + 1].copy(), fv_indices=fi[:fo[nf.value]].copy())


def vocab_transform(voc, feats, levelsup):
    """Oracle TemplatedVocabulary::transform; voc = dict(k, L, scoring, weighting, parent, is_leaf, desc, weight)."""
    feats = np.ascontiguousarray(feats, np.uint8)
    n = len(feats)
    P = np.ascontiguousarray(voc["parent"], np.int32)
    leaf = np.ascontiguousarray(voc["is_leaf"], np.uint8)
    D = np.ascontiguousarray(voc["desc"], np.uint8)
    W = np.ascontiguousarray(voc["weight"], np.float64)
    bw, bv = np.zeros(max(n, 1), np.uint32), np.zeros(max(n, 1), np.float64)
    fn, fo, fi = np.zeros(max(n, 1), np.uint32), np.zeros(n + 1, np.int32), np.zeros(max(n, 1), np.int32)
    nw, nf = C.c_int(), C.c_int()
    lib().orc_vocab_transform(voc["k"], voc["L"], voc["scoring"], voc["weighting"], len(P), _p(P), _p(leaf), _p(D),
                              _p(W), _p(feats), n, levelsup, _p(bw), _p(bv), C.byref(nw), _p(fn), _p(fo), _p(fi),
                              C.byref(nf))
    return dict(bow_words=bw[:nw.value].copy(), bow_values=bv[:nw.value].copy(), fv_nodes=fn[:nf.value].copy(),
                fv_offsets=fo[:nf.value + 1].copy(), fv_indices=fi[:fo[nf.value]].copy())


# ---- keypoint grid + projection / radius matchers (oracle/proj_oracle.cpp) ----------------------------
class OGrid(C.Structure):
    _fields_ = [("min_x", C.c_float), ("min_y", C.c_float), ("max_x", C.c_float), ("max_y", C.c_float),
                ("inv_w", C.c_float), ("inv_h", C.c_float), ("cols", C.c_int32), ("rows", C.c_int32)]


class OParams(C.Structure):
    _fields_ = [("mode", C.c_int32), ("accept_max", C.c_int32), ("nnratio", C.c_float), ("check_ori", C.c_int32),
                ("nlevels", C.c_int32), ("inv_sigma2", C.c_float * 32)]


def _ogrid(g):
    return OGrid(g.min_x, g.min_y, g.max_x, g.max_y, g.inv_w, g.inv_h, g.cols, g.rows)


def grid_assign(kps, grid):
    """Frame::AssignFeaturesToGrid -> (cell_start (cols*rows+1,), cell_idx (n,))."""
    k = np.ascontiguousarray(kps, KP_DTYPE)
    cs = np.zeros(grid.cols * grid.rows + 1, np.int32)
    ci = np.zeros(max(len(k), 1), np.int32)
    L = lib()
    L.orc_grid_assign.argtypes = [C.c_void_p, C.c_int, OGrid, C.c_void_p, C.c_void_p]
    n = L.orc_grid_assign(_p(k), len(k), _ogrid(grid), _p(cs), _p(ci))
    return cs, ci[:n]


def features_in_area(kps, cs, ci, grid, x, y, r, min_level=-1, max_level=-1):
    k = np.ascontiguousarray(kps, KP_DTYPE)
    cs = np.ascontiguousarray(cs, np.int32)
    ci = np.ascontiguousarray(ci if len(ci) else np.zeros(1, np.int32), np.int32)
    out = np.zeros(max(len(k), 1), np.int32)
    L = lib()
    L.orc_features_in_area.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, OGrid, C.c_float, C.c_float, C.c_float,
                                       C.c_int, C.c_int, C.c_void_p, C.c_int]
    m = L.orc_features_in_area(_p(k), _p(cs), _p(ci), _ogrid(grid), x, y, r, min_level, max_level, _p(out), len(out))
    return out[:m]


def proj_search(params, grid, queries, qdesc, kps, desc, uright=None, blocked=None):
    """The sequential restatement of the projection matchers: (nmatches, q_idx, q_dist, owner)."""
    q = np.ascontiguousarray(queries)
    assert q.dtype.itemsize == 40
    qd = np.ascontiguousarray(qdesc, np.uint8).reshape(-1, 32)
    k = np.ascontiguousarray(kps, KP_DTYPE)
    d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    cs, ci = grid_assign(k, grid)
    ci = np.ascontiguousarray(ci if len(ci) else np.zeros(1, np.int32), np.int32)
    P = OParams()
    P.mode, P.accept_max, P.nnratio, P.check_ori, P.nlevels = (params.mode, params.accept_max, params.nnratio,
                                                                 params.check_ori, params.nlevels)
    for i in range(32):
        P.inv_sigma2[i] = params.inv_sigma2[i]
    nq, n = len(q), len(k)
    qi, qdist = np.zeros(max(nq, 1), np.int32), np.zeros(max(nq, 1), np.int32)
    own = np.zeros(max(n, 1), np.int32)
    ur = None if uright is None else np.ascontiguousarray(uright, np.float32)
    bl = None if blocked is None else np.ascontiguousarray(blocked, np.uint8)
    L = lib()
    L.orc_proj_search.argtypes = [OParams, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                  C.c_void_p, C.c_int, OGrid, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    nm = L.orc_proj_search(P, _p(q), _p(qd), nq, _p(k), _p(d), None if ur is None else _p(ur),
                           None if bl is None else _p(bl), n, _ogrid(grid), _p(cs), _p(ci), _p(qi), _p(qdist), _p(own))
    if params.mode > 3:
        own[:] = -1
    return nm, qi[:nq], qdist[:nq], own[:n]


# orbx_map_point (48 B) / orbx_view (112 B) of include/orbx.h
MAP_POINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("nx", "<f4"), ("ny", "<f4"), ("nz", "<f4"),
                            ("min_dist", "<f4"), ("max_dist", "<f4"), ("angle", "<f4"), ("octave", "<i4"),
                            ("flags", "<i4"), ("pad", "<i4")])
VIEW_DTYPE = np.dtype([("R", "<f4", (9,)), ("t", "<f4", (3,)), ("Ow", "<f4", (3,)), ("fx", "<f4"), ("fy", "<f4"),
                       ("cx", "<f4"), ("cy", "<f4"), ("bf", "<f4"), ("min_x", "<f4"), ("max_x", "<f4"), ("min_y", "<f4"),
                       ("max_y", "<f4"), ("th", "<f4"), ("view_cos_limit", "<f4"), ("level_mode", "<i4"), ("pad", "<i4")])


def project(mode, points, view, scale_factors, log_scale_factor):
    """The projection step before the searches (oracle/proj_oracle.cpp orc_project): one query per MapPoint."""
    p = np.ascontiguousarray(points, MAP_POINT_DTYPE)
    v = np.ascontiguousarray(np.asarray(view, VIEW_DTYPE).reshape(1))
    sc = np.ascontiguousarray(scale_factors, np.float32)
    out = np.zeros(max(len(p), 1), np.dtype([("b", "V40")]))
    L = lib()
    L.orc_project.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_float, C.c_void_p]
    L.orc_project(int(mode), _p(p), len(p), _p(v), _p(sc), len(sc), float(log_scale_factor), _p(out))
    return out[:len(p)].view(np.uint8).reshape(-1, 40).copy()


def found_in_frame(q_idx, owner):
    """Tracking::SearchLocalPoints' skip set (src/Tracking.cc:1158-1183: the MapPoints in mCurrentFrame.mvpMapPoints
    get mnLastFrameSeen = this frame and are skipped): after SearchByProjection(F, LastF) (src/ORBmatcher.cc:1330-1470)
    MapPoint q is there iff it took keypoint q_idx[q] >= 0 and that keypoint's slot still holds it (the rotation
    filter, :1448-1468, resets the slots it drops to NULL -- owner -2 here; a later query may hold the slot).
    Sequential restatement, one query at a time.  Returns a bool array over q."""
    q_idx = np.asarray(q_idx)
    owner = np.asarray(owner)
    out = np.zeros(len(q_idx), bool)
    for q in range(len(q_idx)):
        k = int(q_idx[q])
        out[q] = k >= 0 and k < len(owner) and int(owner[k]) == q
    return out


def stereo_mappoints(kps, depth, twc, camera, scale_factors, flags):
    """MapPoints of one stereo frame (orc_stereo_mappoints): MAP_POINT_DTYPE records, SKIP where depth <= 0."""
    k = np.ascontiguousarray(kps, KP_DTYPE)
    d = np.ascontiguousarray(depth, np.float32)
    T = np.ascontiguousarray(twc, np.float32).reshape(12)
    cam = np.ascontiguousarray(camera, np.float32).reshape(4)
    sc = np.ascontiguousarray(scale_factors, np.float32)
    out = np.zeros(max(len(k), 1), MAP_POINT_DTYPE)
    L = lib()
    L.orc_stereo_mappoints.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                       C.c_void_p]
    L.orc_stereo_mappoints(_p(k), _p(d), len(k), _p(T), _p(cam), _p(sc), len(sc), int(flags), _p(out))
    return out[:len(k)]


def undistort_points(xy, K, dist):
    """Frame::UndistortKeyPoints' cv::undistortPoints(K, D, R=I, P=K), OpenCV 3.2 semantics restated."""
    xy = np.ascontiguousarray(xy, np.float32).reshape(-1, 2)
    Km = np.ascontiguousarray(K, np.float32).reshape(9)
    d = np.ascontiguousarray(dist if len(dist) else [0.0], np.float32)
    out = np.zeros_like(xy)
    L = lib()
    L.orc_undistort_points.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    L.orc_undistort_points(_p(xy), len(xy), _p(Km), _p(d), len(dist), _p(out))
    return out


# ---- keyframe database queries (oracle/kfdb_oracle.cpp) ---------------------------------------------
class Kfdb:
    """Sequential restatement of KeyFrameDatabase (src/KeyFrameDatabase.cc) over keyframe slots."""

    def __init__(self, n_vocab_words, n_slots):
        L = lib()
        L.orc_kfdb_create.restype = C.c_void_p
        L.orc_kfdb_create.argtypes = [C.c_int, C.c_int]
        L.orc_kfdb_destroy.argtypes = [C.c_void_p]
        L.orc_kfdb_set_bow.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int]
        L.orc_kfdb_set_covis.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int]
        for n in ("orc_kfdb_add", "orc_kfdb_erase"):
            getattr(L, n).argtypes = [C.c_void_p, C.c_int]
        L.orc_kfdb_clear.argtypes = [C.c_void_p]
        L.orc_kfdb_set_state.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_kfdb_get_state.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_kfdb_score.restype = C.c_double
        L.orc_kfdb_score.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.orc_kfdb_detect.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_uint64, C.c_float, C.c_void_p, C.c_int,
                                      C.c_void_p, C.c_int]
        self._L = L
        self.n_slots = n_slots
        self._h = L.orc_kfdb_create(n_vocab_words, n_slots)

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.orc_kfdb_destroy(self._h)
            self._h = None

    def set_bow(self, slot, words, values):
        w = np.ascontiguousarray(words, np.uint32)
        v = np.ascontiguousarray(values, np.float64)
        self._L.orc_kfdb_set_bow(self._h, slot, _p(w), _p(v), len(w))

    def set_covisibility(self, slot_lists):
        for k, lst in slot_lists.items():
            a = np.ascontiguousarray(list(lst)[:10], np.int32)
            self._L.orc_kfdb_set_covis(self._h, int(k), _p(a), len(a))

    def add(self, slots):
        for k in np.atleast_1d(slots):
            self._L.orc_kfdb_add(self._h, int(k))

    def erase(self, slots):
        for k in np.atleast_1d(slots):
            self._L.orc_kfdb_erase(self._h, int(k))

    def clear(self):
        self._L.orc_kfdb_clear(self._h)

    def get_state(self, kind):
        q = np.zeros(self.n_slots, np.uint64)
        w = np.zeros(self.n_slots, np.int32)
        s = np.zeros(self.n_slots, np.float32)
        self._L.orc_kfdb_get_state(self._h, kind, _p(q), _p(w), _p(s))
        return q, w, s

    def set_state(self, kind, q, w, s):
        q, w, s = (np.ascontiguousarray(q, np.uint64), np.ascontiguousarray(w, np.int32),
                   np.ascontiguousarray(s, np.float32))
        self._L.orc_kfdb_set_state(self._h, kind, _p(q), _p(w), _p(s))

    def score(self, a, b):
        return self._L.orc_kfdb_score(self._h, int(a), int(b))

    def detect(self, kind, slot, query_id, min_score=0.0, exclusions=()):
        ex = np.ascontiguousarray(list(exclusions) or [0], np.int32)
        out = np.zeros(self.n_slots, np.int32)
        n = self._L.orc_kfdb_detect(self._h, kind, int(slot), int(query_id), float(min_score), _p(ex),
                                    len(list(exclusions)), _p(out), len(out))
        if n < 0:
            raise RuntimeError("oracle candidate capacity")
        return out[:n].copy()
