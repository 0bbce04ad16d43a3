"""A/B of engine builds on the lane-schedule legs (diagnostic): python tools/lane_ab.py LIB_DIR
C4 shard (12.5k trees x 200, auto = lane-pair), the same forest on the lane schedule, and the -p
smoother on 20k C5-shaped trees; ms and a checksum of the values (bitwise comparison between builds)."""
import hashlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gfp_gaussian_process_amd import _native  # noqa: E402

_native.LIB_DIR = os.path.abspath(sys.argv[1])
import numpy as np  # noqa: E402
import gfp_gaussian_process_amd as g  # noqa: E402

P = [2.31e-03, 4.36e-02, 9.75e-08, 9.03e+01, 1.60e-02, 1.94e+01, 4.95e-04, 3.35e-04, 8.26e-01, 1.63e-04, 7.48e-01]
out = [sys.argv[1]]
hf = g.HostForest.synthetic(12500, 200)
for kern in ("auto", "lane"):
    f = g.Forest(hf, kernel=kern)
    for _ in range(3):
        v = f.total_likelihood(P)
    t0 = time.perf_counter()
    for _ in range(20):
        v = f.total_likelihood(P)
    out.append(f"{kern} {1e3 * (time.perf_counter() - t0) / 20:.4f} ms ll={v!r}")
    f.close()
hp = g.HostForest.synthetic(20000, 500)
fp = g.Forest(hp)
fp.predict(P, outputs=(False, False, False))
sm = cb = 0.0
for _ in range(5):
    fp.predict(P, outputs=(False, False, False))
    a_, b_ = fp.predict_profile()
    sm += a_
    cb += b_
rows = fp.predict_rows(0, hp.n_rows)
out.append(f"smooth {sm / 5:.4f} ms combine {cb / 5:.4f} ms sha={hashlib.sha256(rows.tobytes()).hexdigest()[:16]}")
print(" | ".join(out), flush=True)
