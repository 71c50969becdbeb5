"""Regenerate tests/golden/oracle_fixtures.json (oracle regression fixtures; not reference outputs —
the reference cannot be built here).  Run: python tests/golden/make_golden.py"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from multiagent_orb_slam2_amd import synthetic as S  # noqa: E402
from oracle import oracle as O  # noqa: E402

cases = []
for seed, rows, cols, nf in [(0, 375, 1242, 2000), (1, 375, 1242, 2000), (21, 480, 640, 1000), (31, 480, 752, 1200)]:
    img = S.kitti_like_image(seed, rows=rows, cols=cols)
    r = O.extract(img, nfeatures=nf)
    cases.append(dict(seed=seed, rows=rows, cols=cols, nfeatures=nf, n=int(len(r["kps"])),
                      image_sha256=hashlib.sha256(img.tobytes()).hexdigest(),
                      kps_sha256=hashlib.sha256(r["kps"].tobytes()).hexdigest(),
                      desc_sha256=hashlib.sha256(r["desc"].tobytes()).hexdigest(),
                      ncand=r["ncand"].tolist(),
                      first_kps=[[float(v) for v in row] for row in r["kps"][:8].tolist()]))
out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "oracle_fixtures.json")
json.dump({"generator": "tests/golden/make_golden.py", "oracle": "oracle/orb_oracle.cpp", "cases": cases},
          open(out, "w"), indent=1)
print("wrote", out)
