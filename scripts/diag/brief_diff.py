"""Diagnostics: descriptor bits that differ between liborbx and the oracle for synthetic KITTI frames (seed list on
the command line): per differing keypoint its level, angle and the differing test indices."""
import sys

import numpy as np

sys.path.insert(0, ".")
import multiagent_orb_slam2_amd as pkg  # noqa: E402
from multiagent_orb_slam2_amd import synthetic as S  # noqa: E402
from oracle import oracle as O  # noqa: E402

ex = pkg.ORBextractor(2000, 1.2, 8, 20, 7, device=0)
for seed in [int(a) for a in sys.argv[1:]] or [21]:
    for name, img in (("left", S.kitti_like_image(seed)), ("right", S.shifted_right_view(S.kitti_like_image(seed), seed))):
        k, d = ex(img)
        ref = O.extract(img, nfeatures=2000)
        rk, rd = ref["kps"], ref["desc"]
        same_k = len(k) == len(rk) and np.array_equal(k, rk)
        bad = np.nonzero((d != rd).any(axis=1))[0] if same_k else []
        print(f"seed {seed} {name}: kps equal {same_k}, {len(bad)} descriptor rows differ")
        for i in bad[:8]:
            bits = np.nonzero(np.unpackbits(d[i] ^ rd[i], bitorder="little"))[0]
            print(f"  kp {i} octave {rk[i]['octave']} angle {rk[i]['angle']!r} xy ({rk[i]['x']}, {rk[i]['y']}) tests {bits.tolist()}")
