"""MI355X-native ORB front-end and Hamming matchers for multi-agent ORB-SLAM2.

The compute path is liborbx.so (HIP kernels for gfx950, C-ABI in include/orbx.h); this package is
the host-side mirror of the reference's ORBextractor / ORBmatcher interface plus the multi-agent
(one agent per GPU) keyframe path.
"""
from .orbx import (KFDB_COVIS, KFDB_LOOP, KFDB_RELOC, KP_DTYPE, PROJ_QUERY_DTYPE, Grid, KeyFrameDatabase,  # noqa: F401
                   KeyframeExchangeRCCL, KeyframeFusionEngine, KfStore, ORBextractor, ORBmatcher, ORBVocabulary,
                   OrbxError, ProjParams, ProjProblem, declared_symbols, device_count, extract_pair, frame_grid,
                   load_library, packet_layout)

__all__ = ["KFDB_COVIS", "KFDB_LOOP", "KFDB_RELOC", "KeyFrameDatabase", "KeyframeExchangeRCCL", "KeyframeFusionEngine",
           "KP_DTYPE", "PROJ_QUERY_DTYPE", "Grid", "ProjParams", "ProjProblem", "frame_grid", "KfStore", "ORBextractor",
           "ORBmatcher", "ORBVocabulary", "OrbxError", "declared_symbols", "device_count", "extract_pair", "load_library",
           "packet_layout"]
