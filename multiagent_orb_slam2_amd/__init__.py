"""MI355X-native ORB front-end and Hamming matchers for multi-agent ORB-SLAM2.

The compute path is liborbx.so (HIP kernels for gfx950, C-ABI in include/orbx.h); this package is
the host-side mirror of the reference's ORBextractor / ORBmatcher interface plus the multi-agent
(one agent per GPU) driver.
"""
from .orbx import (KFDB_COVIS, KFDB_LOOP, KFDB_RELOC, KP_DTYPE, PROJ_QUERY_DTYPE, Grid, KeyFrameDatabase, KfStore, ORBextractor, ORBmatcher, ORBVocabulary,  # noqa: F401
                   OrbxError, ProjParams, ProjProblem, declared_symbols, device_count, frame_grid, load_library)

__all__ = ["KFDB_COVIS", "KFDB_LOOP", "KFDB_RELOC", "KeyFrameDatabase", "KP_DTYPE", "PROJ_QUERY_DTYPE", "Grid", "ProjParams", "ProjProblem", "frame_grid", "KfStore", "ORBextractor", "ORBmatcher", "ORBVocabulary", "OrbxError", "declared_symbols", "device_count",
           "load_library"]
