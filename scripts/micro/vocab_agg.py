"""Vocabulary transform timing per aggregation workgroup (ORBX_VOCAB_AGG_WIDE: 1024 threads, else 256) and descent form
(ORBX_VOCAB_SCALAR): 25 keyframes x 2045 descriptors, the bench's keyframe batch; outputs must agree across modes."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import multiagent_orb_slam2_amd as pkg  # noqa: E402
from multiagent_orb_slam2_amd import synthetic as S  # noqa: E402

voc = S.synthetic_vocabulary(2024, k=10, L=6)
rng = np.random.default_rng(1)
B, cap = 25, 2045
desc = torch.from_numpy(rng.integers(0, 256, (B, cap, 32), dtype=np.uint8)).cuda()
cnt = torch.from_numpy(rng.integers(1900, cap + 1, B).astype(np.int32)).cuda()
ref = None
for mode, scalar in (("wide", True), ("wide", False), ("256", False)):
    if mode == "wide":
        os.environ["ORBX_VOCAB_AGG_WIDE"] = "1"
    else:
        os.environ.pop("ORBX_VOCAB_AGG_WIDE", None)
    if scalar:
        os.environ["ORBX_VOCAB_SCALAR"] = "1"
    else:
        os.environ.pop("ORBX_VOCAB_SCALAR", None)
    v = pkg.ORBVocabulary.from_arrays(voc)
    out = v.transform_batch_device(desc, cnt, 4)
    torch.cuda.synchronize()
    h = {k: t.cpu().numpy() for k, t in out.items()}
    # valid prefixes only (the rest of each row is whatever the allocation held)
    for b in range(B):
        nf, nw = int(h["n_fv"][b]), int(h["n_words"][b])
        h["fv_nodes"][b, nf:] = 0
        h["fv_indices"][b, int(h["fv_offsets"][b, nf]):] = 0
        h["fv_offsets"][b, nf + 1:] = 0
        h["bow_words"][b, nw:] = 0
        h["bow_values"][b, nw:] = 0
    if ref is None:
        ref = h
    else:
        bad = [k for k in ref if not np.array_equal(ref[k], h[k])]
        if bad:
            print(f"agg {mode}: MISMATCH in {bad}", flush=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(5):
        v.transform_batch_device(desc, cnt, 4)
    e0.record()
    for _ in range(50):
        v.transform_batch_device(desc, cnt, 4)
    e1.record()
    torch.cuda.synchronize()
    print(f"agg {mode} scalar_descent {scalar}: {e0.elapsed_time(e1) / 50 * 1e3:.1f} us per 25-keyframe transform", flush=True)
print("done")
