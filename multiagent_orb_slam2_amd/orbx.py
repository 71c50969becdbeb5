"""Host-side mirror of the reference's ORBextractor / ORBmatcher class API over liborbx.so (C-ABI in
include/orbx.h).

The reference classes are ORB_SLAM2::ORBextractor (include/ORBextractor.h:45-111) and
ORB_SLAM2::ORBmatcher (include/ORBmatcher.h:37-102); method names and argument meaning follow them.
Every compute call runs the HIP kernels in liborbx.so; there is no CPU fallback — if the library or a
GPU is missing the constructors raise.
"""
from __future__ import annotations

import atexit
import ctypes as C
import os
import re
import weakref
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ORBX_LIB") or os.path.join(HERE, "liborbx.so")   # ORBX_LIB: A/B of diagnostic builds
HEADER_PATH = os.path.join(os.path.dirname(HERE), "include", "orbx.h")

ORBX_OK, ORBX_ERR_ARG, ORBX_ERR_HIP, ORBX_ERR_CAPACITY, ORBX_ERR_UNSUPPORTED = 0, -1, -2, -3, -4

# cv::KeyPoint layout (28 B) — orbx_keypoint
KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])


class OrbxError(RuntimeError):
    def __init__(self, code: int, what: str):
        super().__init__(f"orbx error {code}: {what}")
        self.code = code


# Every live library object, keyed by creation number.  At interpreter exit they are destroyed newest first by
# close_all: each destroy drains the device and then frees its memory while the HIP runtime is fully up, instead of in
# whatever order module teardown and garbage collection reach them.  close_all is registered with atexit on the first
# registration, after importing torch (whose own exit handlers are then registered first and run after ours: atexit
# is last in, first out).  Dead objects drop out of the table through their weakref callback.
_LIVE: dict = {}
_NEXT = [0]
_ATEXIT = [False]


def _register(obj):
    if not _ATEXIT[0]:
        try:
            import torch  # noqa: F401  (its atexit handlers first, so close_all runs before them)
        except ImportError:
            pass
        atexit.register(close_all)
        _ATEXIT[0] = True
    k = _NEXT[0]
    _NEXT[0] += 1
    _LIVE[k] = weakref.ref(obj, lambda _r, k=k: _LIVE.pop(k, None))


def close_all():
    """Destroy every live library object (newest first).  Called at exit; callable earlier."""
    for k in sorted(_LIVE, reverse=True):
        r = _LIVE.pop(k, None)
        o = r() if r is not None else None
        if o is not None:
            try:
                o.close()
            except Exception:
                pass


def device_check(device: int = 0):
    """Drain the device and raise OrbxError if it holds a pending HIP error (a kernel fault, an illegal address):
    bench.py and smoke() call it last, so a fault during or after the timed work cannot end in exit status 0."""
    _check(load_library().orbx_device_check(int(device)))


class FeatVec(C.Structure):
    _fields_ = [("node_ids", C.c_void_p), ("offsets", C.c_void_p), ("n_nodes", C.c_int), ("indices", C.c_void_p)]


class KfStore(C.Structure):
    """orbx_kf_store: per-field device pointer + slot stride in bytes (include/orbx.h)."""
    _fields_ = [("desc", C.c_void_p), ("desc_stride", C.c_size_t), ("kps", C.c_void_p), ("kps_stride", C.c_size_t),
                ("valid", C.c_void_p), ("valid_stride", C.c_size_t), ("fv_nodes", C.c_void_p),
                ("fv_nodes_stride", C.c_size_t), ("fv_offsets", C.c_void_p), ("fv_offsets_stride", C.c_size_t),
                ("fv_indices", C.c_void_p), ("fv_indices_stride", C.c_size_t), ("n_fv", C.c_void_p),
                ("n_fv_stride", C.c_size_t), ("capacity", C.c_int)]

    FIELDS = ("desc", "kps", "valid", "fv_nodes", "fv_offsets", "fv_indices", "n_fv")

    @classmethod
    def from_fields(cls, capacity: int, **fields):
        """fields: name -> (device tensor whose data_ptr is slot 0 of that field, slot stride in bytes).  A field left
        out is NULL (for callers that read only some fields, e.g. the projection matchers: desc and kps).  The tensors
        are kept alive by the returned struct."""
        s = cls()
        s._keep = []
        for name in cls.FIELDS:
            if name not in fields:
                continue
            t, stride = fields[name]
            setattr(s, name, t.data_ptr())
            setattr(s, name + "_stride", int(stride))
            s._keep.append(t)
        s.capacity = int(capacity)
        return s


class Pyramid(C.Structure):
    """orbx_pyramid (include/orbx.h): device description of an extractor's last image pyramids."""
    _fields_ = [("nlevels", C.c_int), ("batch", C.c_int), ("level0", C.c_void_p), ("level0_step", C.c_size_t),
                ("level0_image_stride", C.c_size_t), ("levels", C.c_void_p), ("image_stride", C.c_size_t),
                ("offset", C.c_size_t * 32), ("rows", C.c_int * 32), ("cols", C.c_int * 32),
                ("scale", C.c_float * 32), ("inv_scale", C.c_float * 32)]


class Grid(C.Structure):
    """orbx_grid (include/orbx.h): Frame grid bounds and inverse cell size."""
    _fields_ = [("min_x", C.c_float), ("min_y", C.c_float), ("max_x", C.c_float), ("max_y", C.c_float),
                ("inv_w", C.c_float), ("inv_h", C.c_float), ("cols", C.c_int32), ("rows", C.c_int32)]


def frame_grid(min_x: float, min_y: float, max_x: float, max_y: float, cols: int = 64, rows: int = 48) -> Grid:
    """The grid a Frame builds (src/Frame.cc:99-104: FRAME_GRID_COLS / (mnMaxX - mnMinX) in float)."""
    f = np.float32
    return Grid(f(min_x), f(min_y), f(max_x), f(max_y), f(cols) / (f(max_x) - f(min_x)),
                f(rows) / (f(max_y) - f(min_y)), cols, rows)


# orbx_proj_query (40 B)
PROJ_QUERY_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("r", "<f4"), ("min_level", "<i4"), ("max_level", "<i4"),
                             ("ur", "<f4"), ("ur_tol", "<f4"), ("angle", "<f4"), ("level", "<i4"), ("flags", "<i4")])
PROJ_MAPPOINTS, PROJ_LASTFRAME, PROJ_KEYFRAME, PROJ_SIM3, PROJ_FUSE, PROJ_BEST, PROJ_INIT = range(7)
QF_SKIP, QF_BLOCKS = 1, 2


# orbx_map_point (48 B) and orbx_view (112 B): the projection step's inputs (orbx_proj_project)
MAP_POINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("nx", "<f4"), ("ny", "<f4"), ("nz", "<f4"),
                            ("min_dist", "<f4"), ("max_dist", "<f4"), ("angle", "<f4"), ("octave", "<i4"),
                            ("flags", "<i4"), ("pad", "<i4")])
VIEW_DTYPE = np.dtype([("R", "<f4", (9,)), ("t", "<f4", (3,)), ("Ow", "<f4", (3,)), ("fx", "<f4"), ("fy", "<f4"),
                       ("cx", "<f4"), ("cy", "<f4"), ("bf", "<f4"), ("min_x", "<f4"), ("max_x", "<f4"), ("min_y", "<f4"),
                       ("max_y", "<f4"), ("th", "<f4"), ("view_cos_limit", "<f4"), ("level_mode", "<i4"), ("pad", "<i4")])


class ProjParams(C.Structure):
    """orbx_proj_params (include/orbx.h)."""
    _fields_ = [("mode", C.c_int32), ("accept_max", C.c_int32), ("nnratio", C.c_float), ("check_ori", C.c_int32),
                ("nlevels", C.c_int32), ("inv_sigma2", C.c_float * 32)]

    @classmethod
    def make(cls, mode, accept_max, nnratio=0.6, check_ori=False, inv_sigma2=None):
        p = cls()
        p.mode, p.accept_max, p.nnratio, p.check_ori = int(mode), int(accept_max), float(nnratio), int(bool(check_ori))
        sig = np.ones(8, np.float32) if inv_sigma2 is None else np.asarray(inv_sigma2, np.float32)
        p.nlevels = len(sig)
        for i, v in enumerate(sig):
            p.inv_sigma2[i] = float(v)
        return p


class ProjProblem(C.Structure):
    """orbx_proj_problem (include/orbx.h): device pointers of one query set against one view."""
    _fields_ = [("queries", C.c_void_p), ("qdesc", C.c_void_p), ("nq", C.c_int32), ("kps", C.c_void_p),
                ("desc", C.c_void_p), ("uright", C.c_void_p), ("blocked", C.c_void_p), ("n", C.c_int32),
                ("cell_start", C.c_void_p), ("cell_idx", C.c_void_p), ("q_idx", C.c_void_p), ("q_dist", C.c_void_p),
                ("owner", C.c_void_p), ("nmatches", C.c_void_p)]


_lib = None


def load_library(path: str = LIB_PATH):
    """Load liborbx.so (raises if it was not built: there is no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(f"liborbx.so not found at {path}; run `make` (or __graft_entry__.build())")
    # One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64.so (SONAME libamdhip64.so.7).
    # Loading torch first lets liborbx's DT_NEEDED libamdhip64.so.7 bind to that same copy, so device
    # pointers, streams and events are shared with torch (and torch.distributed/RCCL).  Loading liborbx
    # first would pull /opt/rocm's copy and torch would then load a second, conflicting runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    vp, i32, f32 = C.c_void_p, C.c_int, C.c_float
    lib.orbx_last_error.restype = C.c_char_p
    lib.orbx_version.restype = C.c_char_p
    lib.orbx_extractor_stage_name.restype = C.c_char_p
    lib.orbx_extractor_get_scale_factor.restype = f32
    lib.orbx_extractor_get_scale_factor.argtypes = [vp]
    lib.orbx_extractor_create.argtypes = [i32, f32, i32, i32, i32, i32, C.POINTER(vp)]
    lib.orbx_stream_create.argtypes = [i32, i32, i32, C.POINTER(vp)]
    lib.orbx_stream_destroy.argtypes = [vp]
    lib.orbx_device_check.argtypes = [i32]
    lib.orbx_proj_project.argtypes = [vp, i32, vp, i32, vp, vp, i32, f32, vp]
    lib.orbx_proj_project_device.argtypes = [vp, i32, vp, vp, i32, i32, vp, vp, vp, i32, f32, vp, vp, vp]
    lib.orbx_stereo_mappoints_device.argtypes = [vp, vp, vp, vp, i32, i32, vp, vp, vp, i32, i32, vp, vp]
    lib.orbx_keyframe_prep_device.argtypes = [vp, vp, vp, vp, i32, i32, vp, vp, vp, i32, i32, vp, Grid, vp, vp, vp]
    lib.orbx_proj_found_device.argtypes = [vp, vp, vp, i32, i32, i32, vp, vp, vp]
    lib.orbx_matcher_create.argtypes = [f32, i32, i32, C.POINTER(vp)]
    for name in ("orbx_extractor_destroy", "orbx_matcher_destroy", "orbx_extractor_get_levels"):
        getattr(lib, name).argtypes = [vp]
    lib.orbx_extract.argtypes = [vp, vp, i32, i32, C.c_size_t, vp, vp, i32, C.POINTER(i32)]
    lib.orbx_extract_pair.argtypes = [vp, vp, vp, C.c_size_t, vp, C.c_size_t, i32, i32, vp, vp, i32, C.POINTER(i32), vp, vp,
                                      i32, C.POINTER(i32)]
    lib.orbx_extract_batch_device.argtypes = [vp, vp, i32, i32, i32, C.c_size_t, C.c_size_t, vp, vp, vp, i32, vp]
    lib.orbx_extract_batch_device_split.argtypes = [vp, vp, i32, i32, i32, C.c_size_t, C.c_size_t, vp, vp, vp, i32, vp, vp]
    lib.orbx_extractor_reserve.argtypes = [vp, i32, i32, i32]
    lib.orbx_extractor_set_pyramid_ring.argtypes = [vp, i32]
    lib.orbx_extractor_max_keypoints.argtypes = [vp, i32, i32]
    lib.orbx_extractor_level_sizes.argtypes = [vp, i32, i32, vp, vp]
    lib.orbx_extractor_copy_level.argtypes = [vp, i32, i32, vp, C.c_size_t]
    lib.orbx_extractor_copy_blurred_level.argtypes = [vp, i32, i32, vp, C.c_size_t]
    lib.orbx_extractor_level_device.argtypes = [vp, i32, i32, C.POINTER(vp), C.POINTER(i32), C.POINTER(i32),
                                                C.POINTER(C.c_size_t)]
    lib.orbx_extractor_enable_timing.argtypes = [vp, i32]
    lib.orbx_extractor_status.argtypes = [vp, C.POINTER(i32), i32]
    lib.orbx_debug_spin_device.argtypes = [vp, C.c_double]
    lib.orbx_extractor_stage_times.argtypes = [vp, vp, C.POINTER(i32)]
    for name in ("orbx_extractor_get_scale_factors", "orbx_extractor_get_inverse_scale_factors",
                 "orbx_extractor_get_scale_sigma_squares", "orbx_extractor_get_inverse_scale_sigma_squares",
                 "orbx_extractor_get_features_per_level"):
        getattr(lib, name).argtypes = [vp, vp]
    lib.orbx_descriptor_distance_device.argtypes = [vp, vp, vp, i32, vp, vp]
    lib.orbx_bf_match.argtypes = [vp, vp, i32, vp, i32, vp, vp, vp]
    lib.orbx_bf_match_device.argtypes = [vp, vp, i32, vp, i32, vp, vp, vp, vp]
    lib.orbx_bf_match_batch_device.argtypes = [vp, vp, i32, C.c_size_t, vp, i32, C.c_size_t, i32, vp, vp, vp, vp]
    lib.orbx_stereo_match.argtypes = [vp, vp, vp, i32, vp, vp, i32, vp, i32, i32, f32, f32, vp, vp, C.POINTER(i32)]
    lib.orbx_stereo_match_batch_device.argtypes = [vp, vp, vp, vp, vp, vp, vp, i32, i32, vp, i32, i32, f32, f32, vp,
                                                   vp, vp]
    lib.orbx_extractor_pyramid_device.argtypes = [vp, C.POINTER(Pyramid)]
    lib.orbx_stereo_refine_batch_device.argtypes = [vp, vp, vp, vp, vp, i32, i32, C.POINTER(Pyramid), i32,
                                                    C.POINTER(Pyramid), i32, f32, f32, vp, vp, vp]
    lib.orbx_compute_stereo_matches.argtypes = [vp, vp, vp, vp, vp, i32, vp, vp, i32, f32, f32, vp, vp, C.POINTER(i32)]
    lib.orbx_stereo_frame.argtypes = [vp, vp, vp, vp, C.c_size_t, vp, C.c_size_t, i32, i32, vp, vp, i32, C.POINTER(i32), vp, vp,
                                      i32, C.POINTER(i32), f32, f32, vp, vp, C.POINTER(i32)]
    lib.orbx_search_by_bow_kfkf.argtypes = [vp, vp, vp, vp, i32, FeatVec, vp, vp, vp, i32, FeatVec, vp,
                                            C.POINTER(i32)]
    lib.orbx_search_by_bow_kff.argtypes = [vp, vp, vp, vp, i32, FeatVec, vp, vp, i32, FeatVec, vp, C.POINTER(i32)]
    lib.orbx_search_for_triangulation.argtypes = [vp, vp, vp, vp, vp, i32, FeatVec, vp, vp, vp, vp, i32, FeatVec,
                                                  vp, vp, vp, i32, f32, f32, i32, vp, C.POINTER(i32)]
    lib.orbx_search_by_bow_kfkf_pairs_device.argtypes = [vp, C.POINTER(KfStore), vp, i32, i32, vp, vp, vp]
    lib.orbx_search_for_triangulation_pairs_device.argtypes = [vp, C.POINTER(KfStore), vp, C.c_size_t, vp, C.c_size_t, vp,
                                                               vp, i32, i32, vp,
                                                               vp, i32, i32, vp, vp, vp]
    lib.orbx_distinctive_descriptors.argtypes = [vp, vp, vp, i32, vp, vp]
    lib.orbx_distinctive_descriptors_device.argtypes = [vp, vp, vp, i32, vp, vp, vp]
    lib.orbx_distinctive_descriptors_store_device.argtypes = [vp, C.POINTER(KfStore), vp, vp, i32, vp, vp, vp]
    lib.orbx_distinctive_descriptors_neighbours_device.argtypes = [vp, C.POINTER(KfStore), vp, vp, i32, i32, vp, vp, vp, vp]
    lib.orbx_grid_build_device.argtypes = [vp, Grid, vp, vp, i32, i32, vp, vp, vp]
    lib.orbx_undistort_keypoints.argtypes = [vp, vp, i32, vp, vp, i32, vp]
    lib.orbx_undistort_keypoints_device.argtypes = [vp, vp, vp, i32, i32, vp, vp, i32, vp, vp]
    lib.orbx_compute_image_bounds.argtypes = [vp, vp, vp, i32, i32, i32, vp]
    lib.orbx_proj_search_batch_device.argtypes = [vp, C.POINTER(ProjParams), Grid, vp, i32, i32, i32, vp]
    lib.orbx_proj_search_grid_batch_device.argtypes = [vp, C.POINTER(ProjParams), Grid, vp, i32, i32, i32, vp, vp]
    lib.orbx_proj_search.argtypes = [vp, C.POINTER(ProjParams), Grid, vp, vp, i32, vp, vp, vp, vp, i32, vp, vp, vp,
                                     C.POINTER(i32)]
    lib.orbx_vocab_load_text.argtypes = [C.c_char_p, i32, C.POINTER(vp)]
    lib.orbx_vocab_create.argtypes = [i32, i32, i32, i32, i32, vp, vp, vp, vp, i32, C.POINTER(vp)]
    lib.orbx_vocab_destroy.argtypes = [vp]
    lib.orbx_vocab_info.argtypes = [vp, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32), C.POINTER(i32)]
    lib.orbx_vocab_transform.argtypes = [vp, vp, i32, i32, vp, vp, C.POINTER(i32), vp, vp, vp, C.POINTER(i32)]
    lib.orbx_vocab_words_device.argtypes = [vp, vp, i32, i32, vp, vp, vp, vp]
    lib.orbx_vocab_transform_batch_device.argtypes = [vp, vp, vp, i32, i32, i32] + [vp] * 11
    lib.orbx_kfdb_create.argtypes = [i32, i32, i32, i32, C.POINTER(vp)]
    lib.orbx_kfdb_destroy.argtypes = [vp]
    lib.orbx_kfdb_info.argtypes = [vp] + [C.POINTER(i32)] * 4
    lib.orbx_kfdb_set_strategy.argtypes = [vp, i32]
    lib.orbx_kfdb_set_bow.argtypes = [vp, i32, vp, vp, i32]
    ll = C.c_longlong
    lib.orbx_kfdb_set_bow_device.argtypes = [vp, vp, i32, vp, ll, vp, ll, vp, ll, vp]
    lib.orbx_kfdb_candidate_pairs_device.argtypes = [vp, i32, vp, vp, i32, vp, vp, i32, vp, vp]
    lib.orbx_kfdb_set_covisibility.argtypes = [vp, vp, i32, vp]
    for name in ("orbx_kfdb_add", "orbx_kfdb_erase"):
        getattr(lib, name).argtypes = [vp, vp, i32]
    lib.orbx_kfdb_clear.argtypes = [vp]
    lib.orbx_kfdb_get_state.argtypes = [vp, i32, vp, vp, vp]
    lib.orbx_kfdb_set_state.argtypes = [vp, i32, vp, vp, vp]
    lib.orbx_kfdb_score.argtypes = [vp, vp, i32, vp]
    lib.orbx_kfdb_score_device.argtypes = [vp, vp, i32, vp, vp]
    lib.orbx_kfdb_detect.argtypes = [vp, i32, vp, vp, vp, i32, vp, vp, vp, vp, i32]
    lib.orbx_kfdb_detect_device.argtypes = [vp, i32, vp, vp, vp, i32, vp, vp, vp, i32, vp, vp, vp]
    lib.orbx_kfdb_detect_sequential.argtypes = [vp, i32, vp, vp, vp, i32, vp, vp, vp, vp, i32]
    lib.orbx_kfdb_detect_sequential_device.argtypes = [vp, i32, vp, vp, vp, i32, vp, vp, vp, i32, vp, vp, vp]
    ll = C.c_longlong
    lib.orbx_packet_layout.argtypes = [i32, vp, C.POINTER(C.c_size_t)]
    lib.orbx_fusion_create.argtypes = [vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, C.POINTER(vp)]
    lib.orbx_fusion_destroy.argtypes = [vp]
    lib.orbx_fusion_info.argtypes = [vp, C.POINTER(C.c_size_t), C.POINTER(i32), C.POINTER(vp), C.POINTER(KfStore)]
    lib.orbx_fusion_pack_device.argtypes = [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, ll, i32, vp, C.POINTER(vp),
                                            C.POINTER(vp), vp]
    lib.orbx_fusion_commit_device.argtypes = [vp, vp, vp, vp, vp, vp]
    lib.orbx_fusion_step_device.argtypes = [vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, ll, i32, vp, vp, vp, vp]
    lib.orbx_fusion_last_step.argtypes = [vp] + [C.POINTER(i32)] * 4
    lib.orbx_fusion_stats.argtypes = [vp, C.POINTER(ll), C.POINTER(i32)]
    lib.orbx_fusion_read_ring.argtypes = [vp, vp]
    lib.orbx_exchange_unique_id.argtypes = [vp]
    lib.orbx_exchange_create.argtypes = [vp, i32, i32, i32, C.POINTER(vp)]
    lib.orbx_exchange_destroy.argtypes = [vp]
    lib.orbx_exchange_allgather_device.argtypes = [vp, vp, C.c_size_t, vp, vp]
    _lib = lib
    return lib


def declared_symbols(header: str = HEADER_PATH) -> list[str]:
    """Function names declared in include/orbx.h."""
    text = open(header).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w]+\**\s+\**(orbx_\w+)\s*\(", text, flags=re.M)))


def _check(code: int):
    if code != ORBX_OK:
        raise OrbxError(code, load_library().orbx_last_error().decode())


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def _as_8uc1(image) -> np.ndarray:
    """An 8UC1 image as the C-ABI takes it: rows of contiguous bytes at a row step (a cv::Mat ROI's layout).  A
    uint8 view whose pixels are contiguous within a row (a crop of a larger frame) is passed as it is, with its step;
    anything else is copied."""
    a = np.asarray(image)
    if a.dtype == np.uint8 and a.ndim == 2 and a.strides[1] == 1 and a.strides[0] >= a.shape[1]:
        return a
    return np.ascontiguousarray(a, np.uint8)


def _tp(t):
    """device pointer of a torch tensor"""
    return C.c_void_p(t.data_ptr())


def device_count() -> int:
    return load_library().orbx_device_count()


def debug_spin(stream, ms: float):
    """Diagnostics: occupy a torch stream (or raw hipStream_t int, 0 = null stream) for about ms milliseconds."""
    ptr = stream if isinstance(stream, int) else stream.cuda_stream
    _check(load_library().orbx_debug_spin_device(C.c_void_p(ptr), float(ms)))


def create_stream(device: int = 0, priority: int = 0, cu_exclude: int = 0):
    """A torch ExternalStream over orbx_stream_create: cu_exclude > 0 leaves that many CUs out of its CU mask (so
    unmasked streams -- the keyframe path -- keep free CUs).  The stream lives as long as the process."""
    import torch
    h = C.c_void_p()
    _check(load_library().orbx_stream_create(device, priority, cu_exclude, C.byref(h)))
    return torch.cuda.ExternalStream(h.value, device=torch.device("cuda", device))


def _featvec(fv):
    """(node_ids, offsets, indices) -> FeatVec struct (keeps arrays alive)."""
    node = np.ascontiguousarray(fv[0], np.uint32)
    off = np.ascontiguousarray(fv[1], np.int32)
    idx = np.ascontiguousarray(fv[2], np.int32)
    s = FeatVec(_p(node), _p(off), len(node), _p(idx))
    s._keep = (node, off, idx)
    return s


class ORBextractor:
    """ORB_SLAM2::ORBextractor (src/ORBextractor.cc:410-1132) on a MI355X."""

    def __init__(self, nfeatures: int, scaleFactor: float, nlevels: int, iniThFAST: int, minThFAST: int,
                 device: int = 0):
        self._lib = load_library()
        h = C.c_void_p()
        _check(self._lib.orbx_extractor_create(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, device,
                                               C.byref(h)))
        self._h = h
        self.nfeatures, self.nlevels, self.device = nfeatures, nlevels, device
        _register(self)
        self._last_shape = None
        self._out = None          # host output staging of __call__
        self._cap, self._cap_for = 0, None

    def close(self):
        if getattr(self, "_h", None):
            self._lib.orbx_extractor_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- getters (include/ORBextractor.h:63-83)
    def GetLevels(self) -> int:
        return self._lib.orbx_extractor_get_levels(self._h)

    def GetScaleFactor(self) -> float:
        return self._lib.orbx_extractor_get_scale_factor(self._h)

    def _vec(self, fn, dtype=np.float32):
        out = np.zeros(self.nlevels, dtype)
        _check(fn(self._h, _p(out)))
        return out

    def GetScaleFactors(self):
        return self._vec(self._lib.orbx_extractor_get_scale_factors)

    def GetInverseScaleFactors(self):
        return self._vec(self._lib.orbx_extractor_get_inverse_scale_factors)

    def GetScaleSigmaSquares(self):
        return self._vec(self._lib.orbx_extractor_get_scale_sigma_squares)

    def GetInverseScaleSigmaSquares(self):
        return self._vec(self._lib.orbx_extractor_get_inverse_scale_sigma_squares)

    def features_per_level(self):
        return self._vec(self._lib.orbx_extractor_get_features_per_level, np.int32)

    def max_keypoints(self, rows: int, cols: int) -> int:
        n = self._lib.orbx_extractor_max_keypoints(self._h, rows, cols)
        if n < 0:
            _check(n)
        return n

    def level_sizes(self, rows: int, cols: int):
        r = np.zeros(self.nlevels, np.int32)
        c = np.zeros(self.nlevels, np.int32)
        _check(self._lib.orbx_extractor_level_sizes(self._h, rows, cols, _p(r), _p(c)))
        return list(zip(r.tolist(), c.tolist()))

    def set_pyramid_ring(self, n: int):
        """Cycle through n pyramid sets: pyramid_device() of call k stays valid until call k+n."""
        _check(self._lib.orbx_extractor_set_pyramid_ring(self._h, n))

    def reserve(self, rows: int, cols: int, max_batch: int):
        _check(self._lib.orbx_extractor_reserve(self._h, rows, cols, max_batch))

    # --- operator() (src/ORBextractor.cc:1043-1105)
    def __call__(self, image: np.ndarray, mask=None):
        """Returns (keypoints: structured array KP_DTYPE, descriptors: (n, 32) uint8).  Mask is ignored, as in
        the reference (include/ORBextractor.h:58)."""
        img = _as_8uc1(image)
        if img.size == 0:
            return np.zeros(0, KP_DTYPE), np.zeros((0, 32), np.uint8)
        assert img.ndim == 2, "8UC1 image expected"
        rows, cols = img.shape
        kps, desc = self._staging(rows, cols)
        n = C.c_int()
        _check(self._lib.orbx_extract(self._h, _p(img), rows, cols, img.strides[0], _p(kps), _p(desc), len(kps),
                                      C.byref(n)))
        self._last_shape = (rows, cols)
        return kps[: n.value].copy(), desc[: n.value].copy()

    def _staging(self, rows: int, cols: int):
        """Output staging reused across calls (only the first n entries are written and copied out; fresh zeroed arrays
        of the full capacity, 480 KB at KITTI, cost page faults and a memset per call); the capacity is asked once per
        image size."""
        if self._cap_for != (rows, cols):
            self._cap = self.max_keypoints(rows, cols)
            self._cap_for = (rows, cols)
        if self._out is None or len(self._out[0]) < self._cap:
            self._out = (np.empty(self._cap, KP_DTYPE), np.empty((self._cap, 32), np.uint8))
        return self._out[0][: self._cap], self._out[1][: self._cap]

    def pyramid_device(self) -> "Pyramid":
        """orbx_pyramid of the last call (device pointers; valid until the next call on this extractor)."""
        p = Pyramid()
        _check(self._lib.orbx_extractor_pyramid_device(self._h, C.byref(p)))
        return p

    @property
    def mvImagePyramid(self):
        """Host copies of the pyramid levels of the last image (include/ORBextractor.h:85)."""
        if self._last_shape is None:
            return []
        out = []
        for l, (h, w) in enumerate(self.level_sizes(*self._last_shape)):
            a = np.zeros((h, w), np.uint8)
            _check(self._lib.orbx_extractor_copy_level(self._h, 0, l, _p(a), w))
            out.append(a)
        return out

    def blurred_levels(self, index: int = 0, shape=None):
        """Diagnostics: host copies of the GaussianBlur'd pyramid levels of image 'index' of the last call (the
        images computeDescriptors reads, src/ORBextractor.cc:1085-1086), borders included.  shape = (rows, cols) of
        the call's images (default: the last host-API image)."""
        shape = shape or self._last_shape
        if shape is None:
            return []
        out = []
        for l, (h, w) in enumerate(self.level_sizes(*shape)):
            a = np.zeros((h, w), np.uint8)
            _check(self._lib.orbx_extractor_copy_blurred_level(self._h, index, l, _p(a), w))
            out.append(a)
        return out

    # --- batched device path (torch tensors on cuda:device)
    def extract_batch_device(self, images, kps=None, desc=None, counts=None, stream=None, out_stream=None):
        """images: uint8 tensor (B, rows, cols) on the GPU.  Returns (kps (B, cap, 28) uint8 view-able as
        KP_DTYPE, desc (B, cap, 32) uint8, counts (B,) int32), all device tensors.  With out_stream the descriptor
        stage runs there and the outputs are complete in out_stream order (orbx_extract_batch_device_split): the
        next call on `stream` overlaps this call's descriptor stage."""
        import torch
        B, rows, cols = images.shape
        cap = self.max_keypoints(rows, cols)
        dev = images.device
        if kps is None:
            kps = torch.empty((B, cap, 28), dtype=torch.uint8, device=dev)
        if desc is None:
            desc = torch.empty((B, cap, 32), dtype=torch.uint8, device=dev)
        if counts is None:
            counts = torch.empty((B,), dtype=torch.int32, device=dev)
        s = C.c_void_p(stream.cuda_stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream)
        if out_stream is None:
            _check(self._lib.orbx_extract_batch_device(self._h, _tp(images), B, rows, cols, images.stride(1),
                                                       images.stride(0), _tp(kps), _tp(desc), _tp(counts), cap, s))
        else:
            _check(self._lib.orbx_extract_batch_device_split(self._h, _tp(images), B, rows, cols, images.stride(1),
                                                             images.stride(0), _tp(kps), _tp(desc), _tp(counts), cap, s,
                                                             C.c_void_p(out_stream.cuda_stream)))
        return kps, desc, counts

    def status(self, reset: bool = False) -> int:
        """Device error word after every call issued so far (orbx_extractor_status): 1 = quadtree node capacity,
        4 = ordering canary (a descriptor stage read another call's keypoints)."""
        f = C.c_int()
        _check(self._lib.orbx_extractor_status(self._h, C.byref(f), int(reset)))
        return f.value

    def enable_timing(self, on: bool = True):
        _check(self._lib.orbx_extractor_enable_timing(self._h, int(on)))

    def stage_times(self):
        n = self._lib.orbx_extractor_stage_count()
        ms = np.zeros(n, np.float64)
        calls = C.c_int()
        _check(self._lib.orbx_extractor_stage_times(self._h, _p(ms), C.byref(calls)))
        names = [self._lib.orbx_extractor_stage_name(i).decode() for i in range(n)]
        return dict(zip(names, ms.tolist())), calls.value


@dataclass
class StereoResult:
    best_idx: np.ndarray   # right index or -1 (accepted if best_dist < 75)
    best_dist: np.ndarray
    n_matched: int


def extract_pair(left: "ORBextractor", right: "ORBextractor", image_left: np.ndarray, image_right: np.ndarray):
    """The stereo Frame constructor's two extractions (src/Frame.cc:78-81) from one thread (orbx_extract_pair: both
    enqueued before either is waited for).  Returns ((keypoints, descriptors) left, (keypoints, descriptors) right), as
    two ORBextractor calls would."""
    il = _as_8uc1(image_left)
    ir = _as_8uc1(image_right)
    assert il.ndim == 2 and il.shape == ir.shape, "two 8UC1 images of one size expected"
    rows, cols = il.shape
    if il.size == 0:
        e = (np.zeros(0, KP_DTYPE), np.zeros((0, 32), np.uint8))
        return e, e
    kl, dl = left._staging(rows, cols)
    kr, dr = right._staging(rows, cols)
    nl, nr = C.c_int(), C.c_int()
    _check(left._lib.orbx_extract_pair(left._h, right._h, _p(il), il.strides[0], _p(ir), ir.strides[0], rows, cols, _p(kl),
                                       _p(dl), len(kl), C.byref(nl), _p(kr), _p(dr), len(kr), C.byref(nr)))
    left._last_shape = right._last_shape = (rows, cols)
    return (kl[: nl.value].copy(), dl[: nl.value].copy()), (kr[: nr.value].copy(), dr[: nr.value].copy())


class ORBmatcher:
    """ORB_SLAM2::ORBmatcher (src/ORBmatcher.cc) on a MI355X."""

    TH_HIGH = 100
    TH_LOW = 50
    HISTO_LENGTH = 30

    def __init__(self, nnratio: float = 0.6, checkOri: bool = True, device: int = 0):
        self._lib = load_library()
        h = C.c_void_p()
        _check(self._lib.orbx_matcher_create(nnratio, int(checkOri), device, C.byref(h)))
        self._h = h
        self.mfNNratio, self.mbCheckOrientation, self.device = nnratio, checkOri, device
        _register(self)
        assert self._lib.orbx_th_high() == self.TH_HIGH and self._lib.orbx_th_low() == self.TH_LOW

    def close(self):
        if getattr(self, "_h", None):
            self._lib.orbx_matcher_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def DescriptorDistance(self, a, b):
        """ORBmatcher::DescriptorDistance (src/ORBmatcher.cc:1649-1665) for row-aligned descriptor arrays
        (one pair or many), computed on the GPU."""
        import torch
        a = np.atleast_2d(np.ascontiguousarray(a, np.uint8))
        b = np.atleast_2d(np.ascontiguousarray(b, np.uint8))
        dev = torch.device("cuda", self.device)
        ta, tb = torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)
        out = torch.empty(a.shape[0], dtype=torch.int32, device=dev)
        s = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        _check(self._lib.orbx_descriptor_distance_device(self._h, _tp(ta), _tp(tb), a.shape[0], _tp(out), s))
        r = out.cpu().numpy()
        return int(r[0]) if r.shape[0] == 1 else r

    def bf_match(self, query, train):
        q = np.ascontiguousarray(query, np.uint8)
        t = np.ascontiguousarray(train, np.uint8)
        n = q.shape[0]
        bi, bd, sd = (np.zeros(n, np.int32) for _ in range(3))
        _check(self._lib.orbx_bf_match(self._h, _p(q), n, _p(t), t.shape[0], _p(bi), _p(bd), _p(sd)))
        return bi, bd, sd

    def bf_match_device(self, query, train, stream=None):
        import torch
        n = query.shape[0]
        bi, bd, sd = (torch.empty(n, dtype=torch.int32, device=query.device) for _ in range(3))
        s = C.c_void_p(stream.cuda_stream if stream is not None else torch.cuda.current_stream(query.device).cuda_stream)
        _check(self._lib.orbx_bf_match_device(self._h, _tp(query), n, _tp(train), train.shape[0], _tp(bi), _tp(bd),
                                              _tp(sd), s))
        return bi, bd, sd

    def bf_match_batch_device(self, query, train, stream=None, out=None):
        """query (P, nq, 32), train (P, nt, 32) uint8 device tensors (rows contiguous within a problem) -> best_idx,
        best_dist, second_dist (P, nq) int32: P independent all-pairs matches in one launch."""
        import torch
        P, nq, nt = query.shape[0], query.shape[1], train.shape[1]
        assert query.stride(1) == 32 and query.stride(2) == 1 and (nt == 0 or (train.stride(1) == 32 and train.stride(2) == 1))
        bi, bd, sd = out if out is not None else \
            (torch.empty((P, nq), dtype=torch.int32, device=query.device) for _ in range(3))
        s = C.c_void_p(stream.cuda_stream if stream is not None else torch.cuda.current_stream(query.device).cuda_stream)
        _check(self._lib.orbx_bf_match_batch_device(self._h, _tp(query), nq, query.stride(0),
                                                    _tp(train) if nt else None, nt, train.stride(0) if nt else 0, P,
                                                    _tp(bi), _tp(bd), _tp(sd), s))
        return bi, bd, sd

    def stereo_descriptor_search(self, kps_left, desc_left, kps_right, desc_right, scale_factors, rows, bf, b):
        """Descriptor search half of Frame::ComputeStereoMatches (src/Frame.cc:466-552)."""
        kl = np.ascontiguousarray(kps_left, KP_DTYPE)
        kr = np.ascontiguousarray(kps_right, KP_DTYPE)
        dl = np.ascontiguousarray(desc_left, np.uint8)
        dr = np.ascontiguousarray(desc_right, np.uint8)
        sc = np.ascontiguousarray(scale_factors, np.float32)
        bi = np.zeros(len(kl), np.int32)
        bd = np.zeros(len(kl), np.int32)
        n = C.c_int()
        _check(self._lib.orbx_stereo_match(self._h, _p(kl), _p(dl), len(kl), _p(kr), _p(dr), len(kr), _p(sc), len(sc),
                                           rows, bf, b, _p(bi), _p(bd), C.byref(n)))
        return StereoResult(bi, bd, n.value)

    def ComputeStereoMatches(self, left, right, kps_left, desc_left, kps_right, desc_right, bf, b):
        """Frame::ComputeStereoMatches (src/Frame.cc:466-639): left/right are the ORBextractors whose last
        host call produced the keypoints (their pyramids are read).  Returns (mvuRight, mvDepth)."""
        kl = np.ascontiguousarray(kps_left, KP_DTYPE)
        kr = np.ascontiguousarray(kps_right, KP_DTYPE)
        dl = np.ascontiguousarray(desc_left, np.uint8)
        dr = np.ascontiguousarray(desc_right, np.uint8)
        ur = np.zeros(len(kl), np.float32)
        dp = np.zeros(len(kl), np.float32)
        n = C.c_int()
        _check(self._lib.orbx_compute_stereo_matches(self._h, left._h, right._h, _p(kl), _p(dl), len(kl), _p(kr), _p(dr),
                                                     len(kr), bf, b, _p(ur), _p(dp), C.byref(n)))
        return ur, dp

    def StereoFrame(self, left, right, image_left, image_right, bf, b):
        """The stereo Frame constructor's ORB work in one call (orbx_stereo_frame: src/Frame.cc:78-81 ExtractORB x2,
        :101 ComputeStereoMatches): ((keypoints, descriptors) left, (keypoints, descriptors) right, mvuRight, mvDepth),
        the values of extract_pair + ComputeStereoMatches without the keypoints' host round trip between them."""
        il = _as_8uc1(image_left)
        ir = _as_8uc1(image_right)
        assert il.ndim == 2 and il.shape == ir.shape, "two 8UC1 images of one size expected"
        rows, cols = il.shape
        if il.size == 0:
            e = (np.zeros(0, KP_DTYPE), np.zeros((0, 32), np.uint8))
            return e, e, np.zeros(0, np.float32), np.zeros(0, np.float32)
        kl, dl = left._staging(rows, cols)
        kr, dr = right._staging(rows, cols)
        ur = np.empty(len(kl), np.float32)
        dp = np.empty(len(kl), np.float32)
        nl, nr, ns = C.c_int(), C.c_int(), C.c_int()
        _check(self._lib.orbx_stereo_frame(self._h, left._h, right._h, _p(il), il.strides[0], _p(ir), ir.strides[0], rows,
                                           cols, _p(kl), _p(dl), len(kl), C.byref(nl), _p(kr), _p(dr), len(kr), C.byref(nr),
                                           bf, b, _p(ur), _p(dp), C.byref(ns)))
        left._last_shape = right._last_shape = (rows, cols)
        n = nl.value
        return ((kl[:n].copy(), dl[:n].copy()), (kr[: nr.value].copy(), dr[: nr.value].copy()), ur[:n].copy(),
                dp[:n].copy())

    def stereo_refine_batch_device(self, kl, nl, kr, best_idx, left_pyramid, left_first, right_pyramid, right_first,
                                   bf, b, stream=None, out=None):
        """Sub-pixel half of Frame::ComputeStereoMatches (src/Frame.cc:554-639) on device batches; pyramids
        from ORBextractor.pyramid_device().  Returns (uright, depth) (B, capacity) float32 device tensors (written into
        out = (uright, depth) when given)."""
        import torch
        B, cap = best_idx.shape
        if out is None:
            ur = torch.empty((B, cap), dtype=torch.float32, device=kl.device)
            dp = torch.empty((B, cap), dtype=torch.float32, device=kl.device)
        else:
            ur, dp = out
        s = C.c_void_p(stream.cuda_stream if stream is not None else torch.cuda.current_stream(kl.device).cuda_stream)
        _check(self._lib.orbx_stereo_refine_batch_device(self._h, _tp(kl), _tp(nl), _tp(kr), _tp(best_idx), B, cap,
                                                         C.byref(left_pyramid), left_first, C.byref(right_pyramid),
                                                         right_first, bf, b, _tp(ur), _tp(dp), s))
        return ur, dp

    def stereo_match_batch_device(self, kl, dl, nl, kr, dr, nr, capacity, scale_factors, rows, bf, b, stream=None):
        import torch
        B = nl.shape[0]
        bi = torch.empty((B, capacity), dtype=torch.int32, device=kl.device)
        bd = torch.empty((B, capacity), dtype=torch.int32, device=kl.device)
        sc = np.ascontiguousarray(scale_factors, np.float32)
        s = C.c_void_p(stream.cuda_stream if stream is not None else torch.cuda.current_stream(kl.device).cuda_stream)
        _check(self._lib.orbx_stereo_match_batch_device(self._h, _tp(kl), _tp(dl), _tp(nl), _tp(kr), _tp(dr), _tp(nr), B,
                                                        capacity, _p(sc), len(sc), rows, bf, b, _tp(bi), _tp(bd), s))
        return bi, bd

    def SearchByBoW_KF_KF(self, desc1, angle1, valid1, fv1, desc2, angle2, valid2, fv2):
        """ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*, ...) (src/ORBmatcher.cc:524-657).  Returns
        (nmatches, match12) with match12[i1] = KF2 index or -1."""
        d1, d2 = np.ascontiguousarray(desc1, np.uint8), np.ascontiguousarray(desc2, np.uint8)
        a1, a2 = np.ascontiguousarray(angle1, np.float32), np.ascontiguousarray(angle2, np.float32)
        v1, v2 = np.ascontiguousarray(valid1, np.uint8), np.ascontiguousarray(valid2, np.uint8)
        m = np.zeros(len(d1), np.int32)
        n = C.c_int()
        _check(self._lib.orbx_search_by_bow_kfkf(self._h, _p(d1), _p(a1), _p(v1), len(d1), _featvec(fv1), _p(d2),
                                                 _p(a2), _p(v2), len(d2), _featvec(fv2), _p(m), C.byref(n)))
        return n.value, m

    def SearchByBoW_pairs_device(self, store: "KfStore", pairs, max_fv_nodes, stream=None):
        """SearchByBoW(KF, KF) for many (kf1, kf2) slot pairs of a device keyframe store in one launch
        (MapFusion.cc:275 / :849 call shape).  pairs: (P, 2) int32 device tensor.
        Returns (match12 (P, capacity) int32, nmatches (P,) int32) device tensors."""
        import torch
        P, cap = pairs.shape[0], store.capacity
        dev = pairs.device
        m12 = torch.empty((P, cap), dtype=torch.int32, device=dev)
        nm = torch.empty((P,), dtype=torch.int32, device=dev)
        s = C.c_void_p(stream.cuda_stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream)
        _check(self._lib.orbx_search_by_bow_kfkf_pairs_device(self._h, C.byref(store), _tp(pairs), P, int(max_fv_nodes),
                                                              _tp(m12), _tp(nm), s))
        return m12, nm

    def SearchForTriangulation_pairs_device(self, store: "KfStore", pairs, geom, sigma2_2, scale_2, max_fv_nodes,
                                            has_mp=None, uright=None, bOnlyStereo=False, stream=None):
        """SearchForTriangulation for many (kf1, kf2) slot pairs of a device keyframe store in one launch
        (LocalMapping::CreateNewMapPoints' neighbour loop, src/LocalMapping.cc:243-274).  pairs: (P, 2) int32; geom:
        (P, 12) float32 rows = F12 (row-major 3x3), epipole ex, ey, pad; has_mp / uright: (slots, capacity) uint8 /
        float32 device tensors, or (1, capacity) for one row shared by all slots (None = the store's valid field / no
        stereo).  Returns (match12 (P, capacity) int32, nmatches (P,) int32) device tensors."""
        import torch
        P, cap = pairs.shape[0], store.capacity
        dev = pairs.device
        assert geom.shape == (P, 12) and geom.dtype == torch.float32 and geom.is_contiguous()
        m12 = torch.empty((P, cap), dtype=torch.int32, device=dev)
        nm = torch.empty((P,), dtype=torch.int32, device=dev)
        s2 = np.ascontiguousarray(sigma2_2, np.float32)
        sc = np.ascontiguousarray(scale_2, np.float32)

        def rows(t, dt):
            if t is None:
                return None, 0
            assert t.dtype == dt and t.is_contiguous() and t.shape[-1] >= cap
            return t, (0 if t.shape[0] == 1 else t.stride(0) * t.element_size())
        mp, mps = rows(has_mp, torch.uint8)
        ur, urs = rows(uright, torch.float32)
        s = C.c_void_p(stream.cuda_stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream)
        _check(self._lib.orbx_search_for_triangulation_pairs_device(
            self._h, C.byref(store), _tp(mp) if mp is not None else None, mps, _tp(ur) if ur is not None else None, urs,
            _tp(pairs), _tp(geom), P, int(max_fv_nodes), _p(s2), _p(sc), len(s2), int(bOnlyStereo), _tp(m12), _tp(nm), s))
        return m12, nm

    def SearchByBoW_KF_F(self, desck, anglek, validk, fvk, descf, anglef, fvf):
        """ORBmatcher::SearchByBoW(KeyFrame*, Frame&, ...) (src/ORBmatcher.cc:161-290).  Returns
        (nmatches, matchF) with matchF[iF] = KF index or -1."""
        dk, df = np.ascontiguousarray(desck, np.uint8), np.ascontiguousarray(descf, np.uint8)
        ak, af = np.ascontiguousarray(anglek, np.float32), np.ascontiguousarray(anglef, np.float32)
        vk = np.ascontiguousarray(validk, np.uint8)
        m = np.zeros(len(df), np.int32)
        n = C.c_int()
        _check(self._lib.orbx_search_by_bow_kff(self._h, _p(dk), _p(ak), _p(vk), len(dk), _featvec(fvk), _p(df),
                                                _p(af), len(df), _featvec(fvf), _p(m), C.byref(n)))
        return n.value, m

    def SearchForTriangulation(self, desc1, kps1, has_mp1, uright1, fv1, desc2, kps2, has_mp2, uright2, fv2, F12,
                               sigma2_2, scale_2, ex, ey, bOnlyStereo=False):
        """ORBmatcher::SearchForTriangulation (src/ORBmatcher.cc:659-825).  Returns (nmatches, match12)."""
        arrs = [np.ascontiguousarray(x, t) for x, t in
                ((desc1, np.uint8), (kps1, KP_DTYPE), (has_mp1, np.uint8), (uright1, np.float32), (desc2, np.uint8),
                 (kps2, KP_DTYPE), (has_mp2, np.uint8), (uright2, np.float32), (F12, np.float32),
                 (sigma2_2, np.float32), (scale_2, np.float32))]
        d1, k1, m1, u1, d2, k2, m2, u2, F, s2, sc2 = arrs
        m = np.zeros(len(d1), np.int32)
        n = C.c_int()
        _check(self._lib.orbx_search_for_triangulation(self._h, _p(d1), _p(k1), _p(m1), _p(u1), len(d1), _featvec(fv1),
                                                       _p(d2), _p(k2), _p(m2), _p(u2), len(d2), _featvec(fv2), _p(F),
                                                       _p(s2), _p(sc2), len(s2), ex, ey, int(bOnlyStereo), _p(m),
                                                       C.byref(n)))
        return n.value, m


    # ---- Frame::UndistortKeyPoints / ComputeImageBounds (src/Frame.cc:404-464) ---------------------------------
    def UndistortKeyPoints(self, kps, K, dist_coef):
        """mvKeysUn from mvKeys: K 3x3 float, dist_coef (k1, k2, p1, p2[, k3]); a zero first coefficient copies."""
        k = np.ascontiguousarray(kps, KP_DTYPE)
        Km = np.ascontiguousarray(K, np.float32).reshape(9)
        d = np.ascontiguousarray(dist_coef, np.float32).reshape(-1)
        out = np.zeros_like(k)
        _check(self._lib.orbx_undistort_keypoints(self._h, _p(k), len(k), _p(Km), _p(d) if len(d) else None, len(d),
                                                   _p(out)))
        return out

    def undistort_keypoints_device(self, kps, counts, K, dist_coef, out=None, stream=None):
        """(B, cap, 28) device keypoints of an extractor batch -> undistorted copy (same layout)."""
        import torch
        B, cap = kps.shape[0], kps.shape[1]
        Km = np.ascontiguousarray(K, np.float32).reshape(9)
        d = np.ascontiguousarray(dist_coef, np.float32).reshape(-1)
        out = out if out is not None else torch.empty_like(kps)
        s = C.c_void_p(stream.cuda_stream if stream is not None else torch.cuda.current_stream(kps.device).cuda_stream)
        _check(self._lib.orbx_undistort_keypoints_device(self._h, _tp(kps), _tp(counts), B, cap, _p(Km),
                                                          _p(d) if len(d) else None, len(d), _tp(out), s))
        return out

    def ComputeImageBounds(self, K, dist_coef, cols, rows):
        """(mnMinX, mnMaxX, mnMinY, mnMaxY) of Frame::ComputeImageBounds."""
        Km = np.ascontiguousarray(K, np.float32).reshape(9)
        d = np.ascontiguousarray(dist_coef, np.float32).reshape(-1)
        b = np.zeros(4, np.float32)
        _check(self._lib.orbx_compute_image_bounds(self._h, _p(Km), _p(d) if len(d) else None, len(d), cols, rows, _p(b)))
        return tuple(float(v) for v in b)

    # ---- MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:246-311) ----------------------------------
    def ComputeDistinctiveDescriptors(self, descriptor_lists):
        """For each MapPoint, its observed descriptors (an (N, 32) uint8 array, in mObservations order, bad
        keyframes skipped): returns (best index per MapPoint, -1 if it has none; (M, 32) chosen descriptors)."""
        lists = [np.ascontiguousarray(d, np.uint8).reshape(-1, 32) for d in descriptor_lists]
        M = len(lists)
        off = np.zeros(M + 1, np.int32)
        off[1:] = np.cumsum([len(d) for d in lists])
        flat = np.ascontiguousarray(np.concatenate(lists) if off[-1] else np.zeros((1, 32), np.uint8))
        best = np.zeros(max(M, 1), np.int32)
        out = np.zeros((max(M, 1), 32), np.uint8)
        _check(self._lib.orbx_distinctive_descriptors(self._h, _p(flat), _p(off), M, _p(best), _p(out)))
        return best[:M], out[:M]

    def distinctive_descriptors_device(self, desc, offsets, out_desc=None, stream=None):
        """Device form: desc (total, 32) uint8, offsets (M+1,) int32 device tensors -> (best (M,), out (M, 32))."""
        import torch
        M = offsets.numel() - 1
        best = torch.empty((max(M, 1),), dtype=torch.int32, device=offsets.device)
        out = out_desc if out_desc is not None else torch.empty((max(M, 1), 32), dtype=torch.uint8, device=offsets.device)
        s = C.c_void_p(stream.cuda_stream if stream is not None else torch.cuda.current_stream(offsets.device).cuda_stream)
        _check(self._lib.orbx_distinctive_descriptors_device(self._h, _tp(desc), _tp(offsets), M, _tp(best), _tp(out), s))
        return best[:M], out[:M]

    def distinctive_descriptors_store_device(self, store: "KfStore", obs, offsets, stream=None):
        """Over a device keyframe store: obs (total, 2) int32 (slot, keypoint index), offsets (M+1,) int32."""
        import torch
        M = offsets.numel() - 1
        best = torch.empty((max(M, 1),), dtype=torch.int32, device=offsets.device)
        out = torch.empty((max(M, 1), 32), dtype=torch.uint8, device=offsets.device)
        s = C.c_void_p(stream.cuda_stream if stream is not None else torch.cuda.current_stream(offsets.device).cuda_stream)
        _check(self._lib.orbx_distinctive_descriptors_store_device(self._h, C.byref(store), _tp(obs), _tp(offsets), M,
                                                                   _tp(best), _tp(out), s))
        return best[:M], out[:M]

    def distinctive_descriptors_neighbours_device(self, store: "KfStore", new_slots, neighbours, match12, stream=None):
        """MapPoints of new keyframes, lists = multiagent.neighbour_observations' (read from match12 in place):
        new_slots (n,), neighbours (n, nn), match12 (n, nn, capacity) int32 device tensors.  Returns (best (n*cap,),
        descriptors (n*cap, 32))."""
        import torch
        n, nn = neighbours.shape
        M = n * store.capacity
        for t in (new_slots, neighbours, match12):
            assert t.dtype == torch.int32 and t.is_contiguous()
        assert match12.shape == (n, nn, store.capacity)
        best = torch.empty((max(M, 1),), dtype=torch.int32, device=new_slots.device)
        out = torch.empty((max(M, 1), 32), dtype=torch.uint8, device=new_slots.device)
        s = C.c_void_p(stream.cuda_stream if stream is not None else torch.cuda.current_stream(new_slots.device).cuda_stream)
        _check(self._lib.orbx_distinctive_descriptors_neighbours_device(self._h, C.byref(store), _tp(new_slots),
                                                                        _tp(neighbours), n, nn, _tp(match12), _tp(best),
                                                                        _tp(out), s))
        return best[:M], out[:M]

    # ---- projection / radius matchers (src/ORBmatcher.cc) ------------------------------
    def proj_search(self, params: ProjParams, grid: Grid, queries, qdesc, kps, desc, uright=None, blocked=None):
        """Generic window search (include/orbx.h orbx_proj_search).  queries: PROJ_QUERY_DTYPE array.
        Returns (nmatches, q_idx, q_dist, owner)."""
        q = np.ascontiguousarray(queries, PROJ_QUERY_DTYPE)
        qd = np.ascontiguousarray(qdesc, np.uint8).reshape(-1, 32)
        k = np.ascontiguousarray(kps, KP_DTYPE)
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        ur = None if uright is None else np.ascontiguousarray(uright, np.float32)
        bl = None if blocked is None else np.ascontiguousarray(blocked, np.uint8)
        nq, n = len(q), len(k)
        qi, qdist = np.zeros(max(nq, 1), np.int32), np.zeros(max(nq, 1), np.int32)
        own = np.zeros(max(n, 1), np.int32)
        nm = C.c_int()
        _check(self._lib.orbx_proj_search(self._h, C.byref(params), grid, _p(q), _p(qd), nq, _p(k), _p(d),
                                          None if ur is None else _p(ur), None if bl is None else _p(bl), n, _p(qi),
                                          _p(qdist), _p(own), C.byref(nm)))
        return nm.value, qi[:nq], qdist[:nq], own[:n]

    def SearchByProjection_MapPoints(self, grid, queries, qdesc, kps, desc, uright, blocked):
        """SearchByProjection(Frame&, vpMapPoints, th) (src/ORBmatcher.cc:45-131): queries from isInFrustum
        (Frame.cc:269-325): window r*scale[level] at (mTrackProjX, mTrackProjY), levels [level-1, level],
        ur = mTrackProjXR, ur_tol = the window radius; flags BLOCKS when the MapPoint has observations."""
        return self.proj_search(ProjParams.make(PROJ_MAPPOINTS, self.TH_HIGH, self.mfNNratio), grid, queries, qdesc, kps,
                                desc, uright, blocked)

    def SearchByProjection_LastFrame(self, grid, queries, qdesc, kps, desc, uright, blocked=None):
        """SearchByProjection(Frame&, const Frame& LastFrame, th, bMono) (src/ORBmatcher.cc:1330-1472)."""
        return self.proj_search(ProjParams.make(PROJ_LASTFRAME, self.TH_HIGH, self.mfNNratio, self.mbCheckOrientation),
                                grid, queries, qdesc, kps, desc, uright, blocked)

    def SearchByProjection_KeyFrame(self, grid, queries, qdesc, kps, desc, blocked, ORBdist):
        """SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th, ORBdist) (src/ORBmatcher.cc:1474-1601)."""
        return self.proj_search(ProjParams.make(PROJ_KEYFRAME, ORBdist, self.mfNNratio, self.mbCheckOrientation), grid,
                                queries, qdesc, kps, desc, None, blocked)

    def SearchByProjection_Sim3(self, grid, queries, qdesc, kps, desc, matched):
        """SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th) (src/ORBmatcher.cc:292-405)."""
        return self.proj_search(ProjParams.make(PROJ_SIM3, self.TH_LOW), grid, queries, qdesc, kps, desc, None, matched)

    def Fuse(self, grid, queries, qdesc, kps, desc, uright, inv_sigma2):
        """The search of Fuse(KeyFrame*, vpMapPoints, th) (src/ORBmatcher.cc:827-977); the caller applies the
        replace / add-observation step (:953-972) to the returned best matches in query order."""
        return self.proj_search(ProjParams.make(PROJ_FUSE, self.TH_LOW, inv_sigma2=inv_sigma2), grid, queries, qdesc,
                                kps, desc, uright, None)

    def Fuse_Scw(self, grid, queries, qdesc, kps, desc):
        """The search of Fuse(KeyFrame*, Scw, vpPoints, th, vpReplacePoint) (src/ORBmatcher.cc:979-1102)."""
        return self.proj_search(ProjParams.make(PROJ_BEST, self.TH_LOW), grid, queries, qdesc, kps, desc)

    def SearchBySim3_direction(self, grid, queries, qdesc, kps, desc):
        """One direction of SearchBySim3 (src/ORBmatcher.cc:1150-1227 / 1230-1307); the caller keeps the
        pairs both directions agree on (:1309-1325)."""
        return self.proj_search(ProjParams.make(PROJ_BEST, self.TH_HIGH), grid, queries, qdesc, kps, desc)

    def SearchForInitialization(self, grid, queries, qdesc, kps, desc):
        """SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize) (src/ORBmatcher.cc:407-522):
        one query per F1 keypoint (window at vbPrevMatched, levels [0, 0], SKIP if its octave > 0)."""
        return self.proj_search(ProjParams.make(PROJ_INIT, self.TH_LOW, self.mfNNratio, self.mbCheckOrientation), grid,
                                queries, qdesc, kps, desc)

    def proj_project(self, mode: int, points, view, scale_factors, log_scale_factor: float):
        """The projection step (include/orbx.h orbx_proj_project): MAP_POINT_DTYPE points, one VIEW_DTYPE view ->
        PROJ_QUERY_DTYPE queries (ORBX_QF_SKIP for points that fail the reference's tests)."""
        p = np.ascontiguousarray(points, MAP_POINT_DTYPE)
        v = np.ascontiguousarray(np.asarray(view, VIEW_DTYPE).reshape(1))
        sc = np.ascontiguousarray(scale_factors, np.float32)
        q = np.zeros(max(len(p), 1), PROJ_QUERY_DTYPE)
        _check(self._lib.orbx_proj_project(self._h, int(mode), _p(p), len(p), _p(v), _p(sc), len(sc),
                                           float(log_scale_factor), _p(q)))
        return q[:len(p)]

    def proj_project_device(self, mode: int, points, counts, views, scale_factors, log_scale_factor: float, out=None,
                            found=None, view_points=None, stream=None):
        """Batched projection: points (S, cap, 48) uint8 device tensor of MAP_POINT_DTYPE records, counts (S,) int32,
        views (V, 112) uint8 device tensor of VIEW_DTYPE -> (V, cap, 40) uint8 queries (PROJ_QUERY_DTYPE); view v
        projects point set view_points[v] ((V,) int32, default v).  found: optional (V, cap) int32 -- points with
        found >= 0 (already matched in the frame) are skipped."""
        import torch
        V, cap = views.shape[0], points.shape[1]
        if out is None:
            out = torch.empty((V, cap, 40), dtype=torch.uint8, device=points.device)
        sc = np.ascontiguousarray(scale_factors, np.float32)
        s = C.c_void_p(stream.cuda_stream if stream is not None else torch.cuda.current_stream(points.device).cuda_stream)
        _check(self._lib.orbx_proj_project_device(self._h, int(mode), _tp(points), _tp(counts), V, cap, _tp(views),
                                                  None if view_points is None else _tp(view_points),
                                                  _p(sc), len(sc), float(log_scale_factor),
                                                  None if found is None else _tp(found), _tp(out), s))
        return out

    def proj_found_device(self, q_idx, owner, found, blocked=None, stream=None):
        """SearchLocalPoints' skip rule after the motion-model search (include/orbx.h orbx_proj_found_device): q_idx
        (S, nq) and owner (S, n) int32 device tensors -> found (S, nq) int32 (0: MapPoint q is in the frame, else -1)
        and, when given, blocked (S, n) bool/uint8 (the keypoint holds a MapPoint), in one launch."""
        import torch
        S, nq = q_idx.shape
        n = owner.shape[1]
        s = C.c_void_p(stream.cuda_stream if stream is not None else torch.cuda.current_stream(q_idx.device).cuda_stream)
        _check(self._lib.orbx_proj_found_device(self._h, _tp(q_idx), _tp(owner), S, nq, n, _tp(found),
                                                None if blocked is None else _tp(blocked), s))
        return found

    def stereo_mappoints_device(self, kps, depth, counts, twc, camera, scale_factors, flags: int, out=None, stream=None):
        """MapPoints of stereo frames (include/orbx.h orbx_stereo_mappoints_device): kps (B, cap, 28) uint8, depth
        (B, cap) float32, counts (B,) int32, twc (B, 12) float32 device tensors -> (B, cap, 48) uint8 MAP_POINT_DTYPE."""
        import torch
        B, cap = kps.shape[0], kps.shape[1]
        if out is None:
            out = torch.empty((B, cap, 48), dtype=torch.uint8, device=kps.device)
        cam = np.ascontiguousarray(camera, np.float32).reshape(4)
        sc = np.ascontiguousarray(scale_factors, np.float32)
        s = C.c_void_p(stream.cuda_stream if stream is not None else torch.cuda.current_stream(kps.device).cuda_stream)
        _check(self._lib.orbx_stereo_mappoints_device(self._h, _tp(kps), _tp(depth), _tp(counts), B, cap, _tp(twc), _p(cam),
                                                      _p(sc), len(sc), int(flags), _tp(out), s))
        return out

    def keyframe_prep_device(self, grid: Grid, kps, depth, counts, twc, camera, scale_factors, flags: int, points, cell_start,
                             cell_idx, stream=None):
        """stereo_mappoints_device and grid_build_device of a batch of new keyframes in one launch (include/orbx.h
        orbx_keyframe_prep_device), written into points (B, cap, 48) uint8 and cell_start / cell_idx int32 (B, cells + 1)
        / (B, cap)."""
        import torch
        B, cap = kps.shape[0], kps.shape[1]
        ncell = grid.cols * grid.rows
        if tuple(cell_start.shape) != (B, ncell + 1) or tuple(cell_idx.shape) != (B, cap) or \
                cell_start.dtype != torch.int32 or cell_idx.dtype != torch.int32 or tuple(points.shape) != (B, cap, 48):
            raise ValueError("keyframe_prep_device: points (B, capacity, 48) uint8, grid int32 (B, cells+1), (B, capacity)")
        cam = np.ascontiguousarray(camera, np.float32).reshape(4)
        sc = np.ascontiguousarray(scale_factors, np.float32)
        s = C.c_void_p(stream.cuda_stream if stream is not None else torch.cuda.current_stream(kps.device).cuda_stream)
        _check(self._lib.orbx_keyframe_prep_device(self._h, _tp(kps), _tp(depth), _tp(counts), B, cap, _tp(twc), _p(cam),
                                                   _p(sc), len(sc), int(flags), _tp(points), grid, _tp(cell_start),
                                                   _tp(cell_idx), s))
        return points, cell_start, cell_idx

    def grid_build_device(self, grid: Grid, kps, counts, stream=None, out=None):
        """Frame::AssignFeaturesToGrid on (B, capacity, 28) device keypoints: (cell_start, cell_idx) tensors
        (written into out = (cell_start, cell_idx) when given)."""
        import torch
        B, cap = kps.shape[0], kps.shape[1]
        ncell = grid.cols * grid.rows
        if out is None:
            cs = torch.empty((B, ncell + 1), dtype=torch.int32, device=kps.device)
            ci = torch.empty((B, cap), dtype=torch.int32, device=kps.device)
        else:
            cs, ci = out
            if tuple(cs.shape) != (B, ncell + 1) or tuple(ci.shape) != (B, cap) or cs.dtype != torch.int32 \
                    or ci.dtype != torch.int32:
                raise ValueError("grid_build_device: out tensors must be int32 (B, cells+1) and (B, capacity)")
        s = C.c_void_p(stream.cuda_stream if stream is not None else torch.cuda.current_stream(kps.device).cuda_stream)
        _check(self._lib.orbx_grid_build_device(self._h, grid, _tp(kps), _tp(counts), B, cap, _tp(cs), _tp(ci), s))
        return cs, ci

    def proj_search_batch_device(self, params: ProjParams, grid: Grid, problems, max_n: int, max_nq: int, stream=None,
                                 grid_counts=None):
        """problems: uint8 device tensor holding n ProjProblem structs (see ProjProblem).  grid_counts: optional (n,)
        int32 device tensor -- problem p's grid is built inside its search from its first grid_counts[p] target
        keypoints and written to its cell_start / cell_idx (orbx_proj_search_grid_batch_device); a problem with
        grid_counts[p] < 0 reads its grid from them."""
        import torch
        s = C.c_void_p(stream.cuda_stream if stream is not None else torch.cuda.current_stream(problems.device).cuda_stream)
        n = problems.numel() // C.sizeof(ProjProblem)
        if grid_counts is None:
            _check(self._lib.orbx_proj_search_batch_device(self._h, C.byref(params), grid, _tp(problems), n, max_n, max_nq, s))
        else:
            _check(self._lib.orbx_proj_search_grid_batch_device(self._h, C.byref(params), grid, _tp(problems), n, max_n,
                                                                max_nq, _tp(grid_counts), s))


@dataclass
class BowResult:
    bow_words: np.ndarray    # uint32, ascending word ids (DBoW2::BowVector keys)
    bow_values: np.ndarray   # float64, normalised weights
    featvec: tuple           # (node_ids, offsets, indices) CSR of DBoW2::FeatureVector


class ORBVocabulary:
    """DBoW2 TemplatedVocabulary<FORB> (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h) on a MI355X:
    loadFromTextFile + transform(features, BowVector&, FeatureVector&, levelsup)."""

    def __init__(self, handle, device):
        self._lib = load_library()
        self._h = handle
        self.device = device
        _register(self)

    @classmethod
    def load_text(cls, path: str, device: int = 0):
        lib = load_library()
        h = C.c_void_p()
        _check(lib.orbx_vocab_load_text(path.encode(), device, C.byref(h)))
        return cls(h, device)

    @classmethod
    def from_arrays(cls, voc: dict, device: int = 0):
        lib = load_library()
        P = np.ascontiguousarray(voc["parent"], np.int32)
        lf = np.ascontiguousarray(voc["is_leaf"], np.uint8)
        D = np.ascontiguousarray(voc["desc"], np.uint8)
        W = np.ascontiguousarray(voc["weight"], np.float64)
        h = C.c_void_p()
        _check(lib.orbx_vocab_create(voc["k"], voc["L"], voc["scoring"], voc["weighting"], len(P), _p(P), _p(lf), _p(D),
                                     _p(W), device, C.byref(h)))
        return cls(h, device)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.orbx_vocab_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self):
        k, L, nn, nw = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        _check(self._lib.orbx_vocab_info(self._h, C.byref(k), C.byref(L), C.byref(nn), C.byref(nw)))
        return dict(k=k.value, L=L.value, n_nodes=nn.value, n_words=nw.value)

    def transform(self, descriptors, levelsup: int = 4) -> BowResult:
        """Frame::ComputeBoW (src/Frame.cc:395-402): BowVector and FeatureVector of a descriptor set."""
        d = np.ascontiguousarray(descriptors, np.uint8).reshape(-1, 32)
        n = len(d)
        bw, bv = np.zeros(max(n, 1), np.uint32), np.zeros(max(n, 1), np.float64)
        fn, fo, fi = np.zeros(max(n, 1), np.uint32), np.zeros(n + 1, np.int32), np.zeros(max(n, 1), np.int32)
        nw, nf = C.c_int(), C.c_int()
        _check(self._lib.orbx_vocab_transform(self._h, _p(d), n, levelsup, _p(bw), _p(bv), C.byref(nw), _p(fn), _p(fo),
                                              _p(fi), C.byref(nf)))
        no = int(fo[nf.value]) if nf.value else 0
        return BowResult(bw[:nw.value].copy(), bv[:nw.value].copy(),
                         (fn[:nf.value].copy(), fo[:nf.value + 1].copy(), fi[:no].copy()))

    def transform_batch_device(self, desc, counts, levelsup: int = 4, stream=None):
        """Batched transform of (B, capacity, 32) device descriptors; returns a dict of device tensors."""
        import torch
        B, cap = desc.shape[0], desc.shape[1]
        dev = desc.device
        t = lambda shape, dt: torch.empty(shape, dtype=dt, device=dev)
        out = dict(word=t((B, cap), torch.int32), weight=t((B, cap), torch.float64), node=t((B, cap), torch.int32),
                   bow_words=t((B, cap), torch.int32), bow_values=t((B, cap), torch.float64), n_words=t((B,), torch.int32),
                   fv_nodes=t((B, cap), torch.int32), fv_offsets=t((B, cap + 1), torch.int32),
                   fv_indices=t((B, cap), torch.int32), n_fv=t((B,), torch.int32))
        s = C.c_void_p(stream.cuda_stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream)
        _check(self._lib.orbx_vocab_transform_batch_device(
            self._h, _tp(desc), _tp(counts), B, cap, levelsup, _tp(out["word"]), _tp(out["weight"]), _tp(out["node"]),
            _tp(out["bow_words"]), _tp(out["bow_values"]), _tp(out["n_words"]), _tp(out["fv_nodes"]),
            _tp(out["fv_offsets"]), _tp(out["fv_indices"]), _tp(out["n_fv"]), s))
        return out


KFDB_LOOP, KFDB_COVIS, KFDB_RELOC = 0, 1, 2
KFDB_AUTO, KFDB_INVERTED, KFDB_PAIRWISE, KFDB_WORDMAP = 0, 1, 2, 3   # how a query finds the keyframes sharing its words
KFDB_COVIS_WIDTH = 10   # GetBestCovisibilityKeyFrames(10)


class KeyFrameDatabase:
    """KeyFrameDatabase (src/KeyFrameDatabase.cc) over a table of keyframe slots on a MI355X.

    Keyframes are slot indices.  A slot carries its BowVector (set_bow), its best-10 covisibility list
    (set_covisibility) and the KeyFrame scratch fields mn*Query / mn*Words / m*Score per query kind
    (include/KeyFrame.h:155-163; get_state / set_state).  DetectLoopCandidates / DetectCovisibility-
    Candidates / DetectRelocalizationCandidates return candidate slots in the reference's order."""

    def __init__(self, n_vocab_words: int, max_slots: int, max_words: int = 4096, device: int = 0):
        self._lib = load_library()
        self._h = C.c_void_p()
        _check(self._lib.orbx_kfdb_create(n_vocab_words, max_slots, max_words, device, C.byref(self._h)))
        self.n_vocab_words, self.max_slots, self.max_words, self.device = n_vocab_words, max_slots, max_words, device
        _register(self)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.orbx_kfdb_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_strategy(self, strategy: int):
        """KFDB_INVERTED (inverted file, as the reference), KFDB_PAIRWISE (intersect with every member),
        KFDB_WORDMAP (rows of the database's word x slot bit matrix; <= 2048 slots) or KFDB_AUTO; results are
        identical."""
        _check(self._lib.orbx_kfdb_set_strategy(self._h, strategy))

    def n_members(self) -> int:
        n = C.c_int()
        _check(self._lib.orbx_kfdb_info(self._h, None, None, None, C.byref(n)))
        return n.value

    def set_bow(self, slot: int, words, values):
        w = np.ascontiguousarray(words, np.uint32)
        v = np.ascontiguousarray(values, np.float64)
        if len(w) != len(v):
            raise ValueError("words and values differ in length")
        _check(self._lib.orbx_kfdb_set_bow(self._h, slot, _p(w), _p(v), len(w)))

    def set_bow_device(self, slots, words, values, n_words, strides=None, stream=None):
        """BowVectors into device int32 slots: words/values/n_words device tensors, BowVector i at
        words[i], values[i], n_words[i] (strides = element strides (word, value, n) if given, e.g. for a
        packet ring; default: row strides of (B, capacity) vocabulary outputs)."""
        import torch
        if strides is None:
            strides = (words.shape[1], values.shape[1], 1)
        s = C.c_void_p(stream.cuda_stream if stream is not None else torch.cuda.current_stream(words.device).cuda_stream)
        _check(self._lib.orbx_kfdb_set_bow_device(self._h, _tp(slots), slots.numel(), _tp(words), strides[0],
                                                  _tp(values), strides[1], _tp(n_words), strides[2], s))

    def set_covisibility(self, slot_lists: dict):
        """{slot: [best covisible slots, best first]} (at most 10 each, KeyFrame::GetBestCovisibilityKeyFrames)."""
        slots = np.array(list(slot_lists.keys()), np.int32)
        best = np.full((len(slots), KFDB_COVIS_WIDTH), -1, np.int32)
        for i, k in enumerate(slots):
            lst = list(slot_lists[int(k)])[:KFDB_COVIS_WIDTH]
            best[i, :len(lst)] = lst
        _check(self._lib.orbx_kfdb_set_covisibility(self._h, _p(slots), len(slots), _p(best)))

    def add(self, slots):
        a = np.atleast_1d(np.ascontiguousarray(slots, np.int32))
        _check(self._lib.orbx_kfdb_add(self._h, _p(a), len(a)))

    def erase(self, slots):
        a = np.atleast_1d(np.ascontiguousarray(slots, np.int32))
        _check(self._lib.orbx_kfdb_erase(self._h, _p(a), len(a)))

    def clear(self):
        _check(self._lib.orbx_kfdb_clear(self._h))

    def get_state(self, kind: int):
        q = np.zeros(self.max_slots, np.uint64)
        w = np.zeros(self.max_slots, np.int32)
        sc = np.zeros(self.max_slots, np.float32)
        _check(self._lib.orbx_kfdb_get_state(self._h, kind, _p(q), _p(w), _p(sc)))
        return q, w, sc

    def set_state(self, kind: int, query, words, score):
        q = np.ascontiguousarray(query, np.uint64)
        w = np.ascontiguousarray(words, np.int32)
        sc = np.ascontiguousarray(score, np.float32)
        if not (len(q) == len(w) == len(sc) == self.max_slots):
            raise ValueError("state arrays must hold max_slots entries")
        _check(self._lib.orbx_kfdb_set_state(self._h, kind, _p(q), _p(w), _p(sc)))

    def score_device(self, pairs, out=None, stream=None):
        """ORBVocabulary::score for (P, 2) int32 device slot pairs; (P,) float64 device tensor."""
        import torch
        out = out if out is not None else torch.empty((pairs.shape[0],), dtype=torch.float64, device=pairs.device)
        _check(self._lib.orbx_kfdb_score_device(self._h, _tp(pairs), pairs.shape[0], _tp(out),
                                                _stream_ptr(stream, pairs.device)))
        return out

    def score(self, pairs) -> np.ndarray:
        """ORBVocabulary::score(bow[a], bow[b]) for (a, b) slot pairs (DBoW2 L1)."""
        pr = np.ascontiguousarray(pairs, np.int32).reshape(-1, 2)
        out = np.zeros(len(pr), np.float64)
        _check(self._lib.orbx_kfdb_score(self._h, _p(pr), len(pr), _p(out)))
        return out

    def detect(self, kind: int, query_slots, query_ids, min_scores=None, exclusions=None, sequential=False):
        """Batch of queries evaluated in order; returns a list of candidate-slot arrays.  sequential=True: the
        query slots were added in query order and query q sees only the members added before its own slot
        (MapFusion's query-then-add order, orbx_kfdb_detect_sequential)."""
        qs = np.atleast_1d(np.ascontiguousarray(query_slots, np.int32))
        nq = len(qs)
        ids = np.atleast_1d(np.ascontiguousarray(query_ids, np.uint64))
        ms = None if min_scores is None else np.atleast_1d(np.ascontiguousarray(min_scores, np.float32))
        eo = ex = None
        if exclusions is not None:
            lens = [len(e) for e in exclusions]
            eo = np.zeros(nq + 1, np.int32)
            eo[1:] = np.cumsum(lens)
            ex = np.ascontiguousarray(np.concatenate([np.asarray(e, np.int32) for e in exclusions]) if sum(lens)
                                      else np.zeros(1, np.int32), np.int32)
        oo = np.zeros(nq + 1, np.int32)
        cap = max(1, nq * self.max_slots)
        out = np.zeros(cap, np.int32)
        fn = self._lib.orbx_kfdb_detect_sequential if sequential else self._lib.orbx_kfdb_detect
        _check(fn(self._h, kind, _p(qs), _p(ids), None if ms is None else _p(ms), nq, None if eo is None else _p(eo),
                  None if ex is None else _p(ex), _p(oo), _p(out), cap))
        return [out[oo[i]:oo[i + 1]].copy() for i in range(nq)]

    def detect_device(self, kind: int, query_slots, query_ids, min_scores=None, excl_offsets=None, excl_slots=None,
                      out=None, out_n=None, status=None, stream=None, sequential=False):
        """Device form: int32 slots, int64 ids, float32 min scores; returns (out, out_n, status) tensors.
        status bit 1: the queries interacted through the scratch fields (results not sequential); bit 2:
        candidate capacity exceeded -- check_status() raises on either."""
        import torch
        nq = query_slots.numel()
        dev = query_slots.device
        out = out if out is not None else torch.empty((nq, self.max_slots), dtype=torch.int32, device=dev)
        out_n = out_n if out_n is not None else torch.empty((nq,), dtype=torch.int32, device=dev)
        status = status if status is not None else torch.zeros((1,), dtype=torch.int32, device=dev)
        s = C.c_void_p(stream.cuda_stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream)
        opt = lambda t: None if t is None else _tp(t)
        fn = self._lib.orbx_kfdb_detect_sequential_device if sequential else self._lib.orbx_kfdb_detect_device
        _check(fn(self._h, kind, _tp(query_slots), _tp(query_ids), opt(min_scores), nq, opt(excl_offsets),
                  opt(excl_slots), _tp(out), out.shape[1], _tp(out_n), _tp(status), s))
        return out, out_n, status

    @staticmethod
    def check_status(status):
        """Raise if a detect_device status word reports interacting queries (1) or exceeded capacity (2)."""
        v = int(status.reshape(-1)[0].item())
        if v & 1:
            raise OrbxError(ORBX_ERR_ARG, "KeyFrameDatabase batch queries interacted through the scratch fields "
                                          "(repeated or stale query ids): results are not the sequential ones")
        if v & 2:
            raise OrbxError(ORBX_ERR_CAPACITY, "KeyFrameDatabase query exceeded its candidate capacity")

    @staticmethod
    def candidate_pairs_device(cand, n_cand, query_slots, k: int, slot_group=None, query_group=None, out=None,
                               stream=None):
        """MapFusion's candidate use (src/MapFusion.cc:136-144, :275): first k candidates of another map per
        query as (query, candidate) SearchByBoW pairs, (query, -1) padded; (nq*k, 2) int32 device tensor."""
        import torch
        nq = query_slots.numel()
        out = out if out is not None else torch.empty((nq * k, 2), dtype=torch.int32, device=cand.device)
        s = C.c_void_p(stream.cuda_stream if stream is not None else torch.cuda.current_stream(cand.device).cuda_stream)
        opt = lambda t: None if t is None else _tp(t)
        _check(load_library().orbx_kfdb_candidate_pairs_device(_tp(cand), cand.shape[1], _tp(n_cand), _tp(query_slots), nq,
                                                               opt(slot_group), opt(query_group), k, _tp(out), s))
        return out

    # the reference's method names (one query each)
    def DetectLoopCandidates(self, slot: int, query_id: int, minScore: float, connected=()):
        return self.detect(KFDB_LOOP, [slot], [query_id], [minScore], [list(connected)])[0]

    def DetectCovisibilityCandidates(self, slot: int, query_id: int, minScore: float, ignore=()):
        return self.detect(KFDB_COVIS, [slot], [query_id], [minScore], [list(ignore)])[0]

    def DetectRelocalizationCandidates(self, slot: int, query_id: int):
        return self.detect(KFDB_RELOC, [slot], [query_id])[0]


PACKET_FIELDS = ("kps", "desc", "fv_nodes", "fv_offsets", "fv_indices", "valid", "bow_words", "bow_values")


def packet_layout(capacity: int):
    """orbx_packet_layout: {field: byte offset}, packet bytes."""
    off = (C.c_size_t * 8)()
    nb = C.c_size_t()
    _check(load_library().orbx_packet_layout(capacity, off, C.byref(nb)))
    return dict(zip(PACKET_FIELDS, list(off))), nb.value


class _DeviceRegion:
    """Device memory owned by liborbx, exposed to torch without a copy (__cuda_array_interface__, which torch's ROCm
    build reads for HIP device pointers); 'owner' stays referenced as long as the tensor's storage is alive."""

    def __init__(self, ptr: int, shape, owner):
        self.owner = owner
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": "|u1", "data": (int(ptr), False),
                                         "version": 2, "strides": None}


def _device_view(ptr: int, shape, device: int, owner):
    import torch
    return torch.as_tensor(_DeviceRegion(ptr, shape, owner), device=torch.device("cuda", device))


def _stream_ptr(stream, device):
    import torch
    return C.c_void_p(stream.cuda_stream if stream is not None else torch.cuda.current_stream(device).cuda_stream)


class KeyframeExchangeRCCL:
    """orbx_exchange: the keyframe all-gather through a native RCCL communicator (liborbx dlopens librccl).
    unique_id() on one rank, distributed by the caller (e.g. torch.distributed.broadcast_object_list)."""

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        _check(load_library().orbx_exchange_unique_id(buf))
        return buf.raw

    def __init__(self, uid: bytes, world: int, rank: int, device: int = 0):
        self._lib = load_library()
        self._h = C.c_void_p()
        b = C.create_string_buffer(bytes(uid), 128)
        _check(self._lib.orbx_exchange_create(b, world, rank, device, C.byref(self._h)))
        _register(self)
        self.world, self.rank, self.device = world, rank, device

    def close(self):
        if getattr(self, "_h", None):
            self._lib.orbx_exchange_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def allgather(self, send, recv, stream=None):
        """send (n, P) uint8 device tensor -> recv (world*n, P), rank-major."""
        _check(self._lib.orbx_exchange_allgather_device(self._h, _tp(send), send.numel(), _tp(recv),
                                                        _stream_ptr(stream, send.device)))
        return recv


class KeyframeFusionEngine:
    """orbx_fusion: one agent's keyframe path into MapFusion in native code (include/orbx.h, "Keyframe fusion") --
    BoW, packets, the exchange into the ring, the sequential DetectLoopCandidates, the other-map candidate pairs
    and the batched SearchByBoW (src/MapFusion.cc:83-88, :133-149, :275-281).  vocab / matcher are kept alive
    here; the matcher is MapFusion's ORBmatcher(0.75, true)."""

    def __init__(self, vocab: "ORBVocabulary", matcher: ORBmatcher, capacity: int, slots: int, max_keyframes: int,
                 candidates: int = 16, levelsup: int = 4, min_matches: int = 20, agent: int = 0, world: int = 1,
                 device: int = 0):
        self._lib = load_library()
        self.vocab, self.matcher = vocab, matcher
        self._h = C.c_void_p()
        _check(self._lib.orbx_fusion_create(vocab._h, matcher._h, capacity, slots, max_keyframes, candidates, levelsup,
                                            min_matches, agent, world, device, C.byref(self._h)))
        self.capacity, self.slots, self.k, self.agent, self.world, self.device = capacity, slots, candidates, agent, world, device
        _register(self)
        pb, ns, ring, st = C.c_size_t(), C.c_int(), C.c_void_p(), KfStore()
        _check(self._lib.orbx_fusion_info(self._h, C.byref(pb), C.byref(ns), C.byref(ring), C.byref(st)))
        self.packet_bytes = pb.value
        self.store = st
        self._pending = 0

    def close(self):
        if getattr(self, "_h", None):
            self._lib.orbx_fusion_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _src(self, kps, desc, counts, depth, valid):
        return (_tp(kps), _tp(desc), _tp(counts), None if depth is None else _tp(depth), None if valid is None else _tp(valid))

    def pack(self, kps, desc, counts, rows: range, frame_base: int, frame_step: int = 1, depth=None, valid=None, send=None,
             stream=None):
        """Phase 1 over extractor batch rows rows.start + j*rows.step (kps (B, cap, 28), desc (B, cap, 32), counts (B,)
        device tensors; depth / valid (B, cap)).  send: (n, P) uint8 tensor for the packets when world > 1."""
        n = len(rows)
        dst, snd = C.c_void_p(), C.c_void_p()
        _check(self._lib.orbx_fusion_pack_device(self._h, *self._src(kps, desc, counts, depth, valid), kps.shape[1],
                                                 rows.start, rows.step, n, frame_base, frame_step,
                                                 None if send is None else _tp(send), C.byref(dst), C.byref(snd),
                                                 _stream_ptr(stream, kps.device)))
        self._pending = n
        self._dst = dst.value
        return n

    def exchange_view(self):
        """The ring slots the last pack() reserved for this step's world * n packets (rank-major), as a (world*n, P)
        uint8 device tensor aliasing them (orbx_fusion_pack_device's d_exchange_dst): all-gather into it, then
        commit(None) -- no gathered buffer and no copy into the ring (70 MB per step at 8 agents)."""
        if not getattr(self, "_dst", None):
            raise OrbxError(ORBX_ERR_ARG, "exchange_view() before pack(): no ring slots are reserved")
        return _device_view(self._dst, (self.world * self._pending, self.packet_bytes), self.device, self)

    def commit(self, exchanged=None, outputs=None, stream=None):
        """Phase 2.  exchanged: (world*n, P) uint8 tensor of the gathered packets when they were gathered elsewhere
        (world > 1), None when they are already in the ring (exchange_view).  outputs: optional (pairs (n*k, 2),
        match12 (n*k, cap), nmatches (n*k,)) int32 tensors to fill."""
        o = outputs or (None, None, None)
        dev = exchanged.device if exchanged is not None else (o[0].device if o[0] is not None else None)
        _check(self._lib.orbx_fusion_commit_device(self._h, None if exchanged is None else _tp(exchanged),
                                                   *[None if t is None else _tp(t) for t in o],
                                                   _stream_ptr(stream, dev if dev is not None else self.device)))
        return outputs

    def step(self, kps, desc, counts, rows: range, frame_base: int, frame_step: int = 1, depth=None, valid=None,
             exchange: "KeyframeExchangeRCCL" = None, outputs=None, stream=None):
        """Both phases (native exchange in between when world > 1)."""
        o = outputs or (None, None, None)
        _check(self._lib.orbx_fusion_step_device(self._h, None if exchange is None else exchange._h,
                                                 *self._src(kps, desc, counts, depth, valid), kps.shape[1], rows.start,
                                                 rows.step, len(rows), frame_base, frame_step,
                                                 *[None if t is None else _tp(t) for t in o],
                                                 _stream_ptr(stream, kps.device)))
        return outputs

    def new_outputs(self, n: int):
        import torch
        dev = torch.device("cuda", self.device)
        return (torch.empty((n * self.k, 2), dtype=torch.int32, device=dev),
                torch.empty((n * self.k, self.capacity), dtype=torch.int32, device=dev),
                torch.empty((n * self.k,), dtype=torch.int32, device=dev))

    def last_step(self):
        v = [C.c_int() for _ in range(4)]
        _check(self._lib.orbx_fusion_last_step(self._h, *[C.byref(x) for x in v]))
        first, n_new, qfirst, nq = (x.value for x in v)
        return range(first, first + n_new), range(qfirst, qfirst + nq)

    def stats(self):
        """(keyframe candidates that passed the 20-match gate so far, database status word); synchronises."""
        g, st = C.c_longlong(), C.c_int()
        _check(self._lib.orbx_fusion_stats(self._h, C.byref(g), C.byref(st)))
        return g.value, st.value

    def check(self):
        _, st = self.stats()
        if st & 1:
            raise OrbxError(ORBX_ERR_ARG, "KeyFrameDatabase batch queries interacted through the scratch fields")
        if st & 2:
            raise OrbxError(ORBX_ERR_CAPACITY, "KeyFrameDatabase query exceeded its candidate capacity")

    def read_ring(self) -> np.ndarray:
        out = np.zeros((self.slots, self.packet_bytes), np.uint8)
        _check(self._lib.orbx_fusion_read_ring(self._h, _p(out)))
        return out
